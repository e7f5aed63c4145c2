set -o pipefail
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread > $O/tx_tests.log 2>&1 || { tail -30 $O/tx_tests.log; exit 1; }
tail -1 $O/tx_tests.log
timeout -k 10 200 python tools/ab_tx.py 40 > $O/ab_tx.jsonl 2> $O/ab_tx.err || { tail -5 $O/ab_tx.err; exit 1; }
cat $O/ab_tx.jsonl
bash tools/gpu_cmd_r05c.sh
