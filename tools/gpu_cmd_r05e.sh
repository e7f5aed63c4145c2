set -o pipefail
O=gpurun_out/r05; mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread > $O/tx_tests.log 2>&1 || { tail -30 $O/tx_tests.log; exit 1; }
tail -1 $O/tx_tests.log
$T 200 python tools/ab_tx.py 40 > $O/ab_tx.jsonl 2> $O/ab_tx.err || { tail -5 $O/ab_tx.err; exit 1; }
python3 -c "
import json,collections;d=collections.defaultdict(list)
for l in open('$O/ab_tx.jsonl'): r=json.loads(l); d[r['mode']].append(r['ms'])
print({k:sorted(v) for k,v in d.items()})"
bash tools/gpu_round.sh utf8tests || exit 1
$T 200 python tools/ab_c5d.py > $O/ab_c5d_b.jsonl 2>> $O/ab_c5d.err || exit 1
$T 200 python tools/ab_c5s.py > $O/ab_c5s.jsonl 2>> $O/ab_c5s.err || exit 1
cat $O/ab_c5s.jsonl
cat $O/ab_c5d_b.jsonl
$T 600 python -u -m pytest tests/test_gpu_inplace.py tests/test_gpu_mux.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $O/host_tests.log 2>&1 || { tail -30 $O/host_tests.log; exit 1; }
tail -1 $O/host_tests.log
$T 300 python -u -m pytest tests/test_gpu_service.py -x -v --timeout 120 --timeout-method thread > $O/service_tests.log 2>&1 || { tail -30 $O/service_tests.log; exit 1; }
tail -3 $O/service_tests.log
$T 600 python -u -m pytest tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread > $O/dropin_tests.log 2>&1 || { tail -30 $O/dropin_tests.log; exit 1; }
tail -1 $O/dropin_tests.log
$T 400 python tools/ab_echo.py 2 > $O/ab_echo.jsonl 2> $O/ab_echo.err || { tail -5 $O/ab_echo.err; exit 1; }
cat $O/ab_echo.jsonl
