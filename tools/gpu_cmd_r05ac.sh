set -o pipefail
O=gpurun_out/r05; mkdir -p $O
LAT_TRACE=1 timeout -k 10 200 ./tools/bin/lat_feed 3000 > $O/lat_trace_fast2.jsonl 2> $O/lat_trace_fast2.err || { tail -5 $O/lat_trace_fast2.err; exit 1; }
grep trace $O/lat_trace_fast2.jsonl
