set -o pipefail
O=gpurun_out/r05; mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_session.py tests/test_gpu_inplace.py tests/test_gpu_mux.py -x -q --timeout 120 --timeout-method thread > $O/small_tests.log 2>&1 || { tail -30 $O/small_tests.log; exit 1; }
tail -2 $O/small_tests.log
LAT_TRACE=1 $T 120 tools/bin/lat_feed 2000 > $O/lat_trace2.jsonl 2> $O/lat_feed.err || { cat $O/lat_feed.err; exit 1; }
cat $O/lat_trace2.jsonl
$T 120 tools/bin/lat_feed 3000 > $O/lat_feed3.jsonl 2> $O/lat_feed.err || { cat $O/lat_feed.err; exit 1; }
cat $O/lat_feed3.jsonl
