set -o pipefail
O=gpurun_out/r05; mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_service.py -x -v --timeout 120 --timeout-method thread > $O/service_tests.log 2>&1 || { tail -30 $O/service_tests.log; exit 1; }
tail -3 $O/service_tests.log
for v in abl1 abl2 abl3; do FWS_LIB_VARIANT=$v $T 200 python tools/ab_c5d.py > $O/ab_c5d_$v.jsonl 2>> $O/ab_c5d.err || exit 1; head -2 $O/ab_c5d_$v.jsonl; done
$T 600 python -u -m pytest tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread > $O/dropin_tests.log 2>&1 || { tail -30 $O/dropin_tests.log; exit 1; }
tail -1 $O/dropin_tests.log
$T 500 python tools/ab_echo.py 2 > $O/ab_echo.jsonl 2> $O/ab_echo.err || { tail -5 $O/ab_echo.err; exit 1; }
python3 -c "
import json
for l in open('$O/ab_echo.jsonl'):
    r=json.loads(l); print(r['mode'],r['clients'],r['persistent'],r['rep'],r['goodput_rx_tx_mbps'],r['rtt_us'].get('p50'),r['gpu_reads'],r['gpu_batches'])"
