set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode.py > gpurun_out/it11_tests.log 2>&1 || { tail -30 gpurun_out/it11_tests.log; exit 1; }
tail -1 gpurun_out/it11_tests.log
