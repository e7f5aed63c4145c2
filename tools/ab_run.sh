# ad-hoc pass (overwritten per experiment)
set -o pipefail
O=gpurun_out/ab8; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_configs.py tests/test_gpu_session.py tests/test_gpu_mux.py tests/test_gpu_limits.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
