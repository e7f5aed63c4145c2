# ad-hoc pass (overwritten per experiment)
set -o pipefail
O=gpurun_out/ab3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_configs.py tests/test_gpu_session.py tests/test_gpu_mux.py -x -q --timeout 120 --timeout-method thread > $O/dec_tests.log 2>&1 || { tail -30 $O/dec_tests.log; exit 1; }
tail -1 $O/dec_tests.log
timeout -k 10 300 python tools/prof_scan.py > $O/prof_scan.json 2> $O/prof_scan.err || { tail $O/prof_scan.err; exit 1; }
cat $O/prof_scan.json
