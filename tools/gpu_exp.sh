set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
FWS_DEBUG_MERGE_TWICE=1 timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/twice -o run -- python3 $R/tools/run_decode.py c3 6 > $R/gpurun_out/twice.log 2>&1 || exit 1
echo done
