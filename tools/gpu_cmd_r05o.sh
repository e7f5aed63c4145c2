set -o pipefail
O=gpurun_out/r05; mkdir -p $O
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_service.py -x -v --timeout 120 --timeout-method thread > $O/service_tests.log 2>&1 || { tail -30 $O/service_tests.log; exit 1; }
tail -2 $O/service_tests.log
$T 120 tools/bin/lat_feed 3000 > $O/lat_feed_push.jsonl 2> $O/lat_feed.err || { cat $O/lat_feed.err; exit 1; }
cat $O/lat_feed_push.jsonl
$T 500 python tools/ab_echo.py 1 > $O/ab_echo_push.jsonl 2> $O/ab_echo.err || { tail -5 $O/ab_echo.err; exit 1; }
python3 -c "
import json
for l in open('$O/ab_echo_push.jsonl'):
    r=json.loads(l); print(r['mode'],r['clients'],r['persistent'],r['rep'],r['goodput_rx_tx_mbps'],r['rtt_us'].get('p50'),r['gpu_reads'],r['gpu_batches'])"
