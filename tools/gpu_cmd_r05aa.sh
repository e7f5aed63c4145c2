set -o pipefail
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mux.py tests/test_gpu_service.py tests/test_gpu_dropin.py tests/test_gpu_session.py > $O/t_final_host.log 2>&1 || { tail -30 $O/t_final_host.log; exit 1; }
tail -2 $O/t_final_host.log
