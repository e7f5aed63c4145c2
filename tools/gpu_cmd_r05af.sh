set -o pipefail
O=gpurun_out/r05; mkdir -p $O
LAT_TRACE=1 timeout -k 10 200 ./tools/bin/lat_feed 3000 > $O/lat_trace_pf2.jsonl 2> $O/lat_trace_pf2.err || { tail -5 $O/lat_trace_pf2.err; exit 1; }
grep trace $O/lat_trace_pf2.jsonl | head -2
timeout -k 10 500 python tools/ab_rtt1.py ab_nopf 3 > $O/ab_rtt1_pf2.jsonl 2> $O/ab_rtt1.err || { tail -5 $O/ab_rtt1.err; exit 1; }
cat $O/ab_rtt1_pf2.jsonl
