set -o pipefail
O=gpurun_out/r05; mkdir -p $O
LAT_TRACE=1 timeout -k 10 200 ./tools/bin/lat_feed 3000 > $O/lat_trace_fast.jsonl 2> $O/lat_trace_fast.err || { tail -5 $O/lat_trace_fast.err; exit 1; }
grep -v mux $O/lat_trace_fast.jsonl
timeout -k 10 200 ./tools/bin/vram_probe 3000 > $O/vram_probe2.jsonl 2>&1 || { tail -5 $O/vram_probe2.jsonl; exit 1; }
cat $O/vram_probe2.jsonl
