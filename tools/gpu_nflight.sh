set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 240 python -u tools/n_in_flight.py c3 > gpurun_out/nflight.log 2>&1 && timeout -k 10 240 python -u tools/n_in_flight.py c2 >> gpurun_out/nflight.log 2>&1
rc=$?; cat gpurun_out/nflight.log | grep -v amdgpu.ids; exit $rc
