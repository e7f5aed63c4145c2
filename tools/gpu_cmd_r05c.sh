set -o pipefail
O=gpurun_out/r05; mkdir -p $O
bash tools/gpu_round.sh utf8tests || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_inplace.py tests/test_gpu_mux.py tests/test_gpu_dropin.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $O/host_tests.log 2>&1 || { tail -30 $O/host_tests.log; exit 1; }
tail -1 $O/host_tests.log
timeout -k 10 200 python tools/ab_c5d.py > $O/ab_c5d_b.jsonl 2>> $O/ab_c5d.err || exit 1
cat $O/ab_c5d_b.jsonl
