set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_decode.py -k "fused" -x -v --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?
tail -30 gpurun_out/t1.log
exit $rc
