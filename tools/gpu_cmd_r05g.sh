set -o pipefail
O=gpurun_out/r05; mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_service.py -x -v --timeout 120 --timeout-method thread > $O/service_tests.log 2>&1 || { tail -30 $O/service_tests.log; exit 1; }
tail -3 $O/service_tests.log
AB_CAPS=131072,262144,1048576 $T 300 python tools/ab_c5d.py > $O/ab_c5d_caps.jsonl 2> $O/ab_c5d.err || { tail -5 $O/ab_c5d.err; exit 1; }
cat $O/ab_c5d_caps.jsonl
$T 500 python tools/ab_echo.py 2 > $O/ab_echo2.jsonl 2> $O/ab_echo.err || { tail -5 $O/ab_echo.err; exit 1; }
python3 -c "
import json
for l in open('$O/ab_echo2.jsonl'):
    r=json.loads(l); print(r['mode'],r['clients'],r['persistent'],r['rep'],r['goodput_rx_tx_mbps'],r['rtt_us'].get('p50'),r['gpu_reads'],r['gpu_batches'])"
