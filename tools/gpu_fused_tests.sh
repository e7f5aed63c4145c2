# one-pass decode: its dedicated tests and the shared decode tests in fused mode
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_decode.py -k "fused or test_gpu_fused" -x -v --timeout 120 --timeout-method thread > gpurun_out/fused_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/fused_tests.log | grep -v "test_gpu_decode.py.*PASSED" | tail -30
exit $rc
