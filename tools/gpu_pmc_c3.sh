# HBM traffic (FETCH_SIZE, WRITE_SIZE; separate passes) of the C3 stream-decode kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/pmc_c3_fetch -o run -- python3 $R/tools/run_decode.py c3 6 > $R/gpurun_out/pmc_c3_fetch.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/pmc_c3_write -o run -- python3 $R/tools/run_decode.py c3 6 > $R/gpurun_out/pmc_c3_write.log 2>&1
echo rc=$?
