set -o pipefail
O=gpurun_out/r05; mkdir -p $O
T="timeout -k 10"
$T 800 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_session.py tests/test_gpu_inplace.py tests/test_gpu_mux.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > $O/small_tests.log 2>&1 || { tail -30 $O/small_tests.log; exit 1; }
tail -1 $O/small_tests.log
$T 200 tools/bin/lat_feed 2000 > $O/lat_fast.jsonl 2> $O/lat_feed.err || { cat $O/lat_feed.err; exit 1; }
grep '"workers": 16\|"workers": 0, "buffer": "registered", "payload": 4096\|mux.*16' $O/lat_fast.jsonl
$T 500 python tools/ab_echo.py 1 > $O/ab_echo_fast.jsonl 2> $O/ab_echo.err || { tail -5 $O/ab_echo.err; exit 1; }
python3 -c "
import json
for l in open('$O/ab_echo_fast.jsonl'):
    r=json.loads(l); print(r['mode'],r['clients'],r['persistent'],r['rep'],r['goodput_rx_tx_mbps'],r['rtt_us'].get('p50'),r['gpu_reads'],r['gpu_batches'])"
