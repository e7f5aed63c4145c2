set -o pipefail
O=gpurun_out/r05; mkdir -p $O
T="timeout -k 10"
$T 120 tools/bin/lat_feed 3000 > $O/lat_feed.jsonl 2> $O/lat_feed.err || { cat $O/lat_feed.err; exit 1; }
cat $O/lat_feed.jsonl
$T 200 python tools/ab_c5d.py > $O/ab_c5d_new.jsonl 2>> $O/ab_c5d.err || exit 1
head -3 $O/ab_c5d_new.jsonl
AB_CAPS=32768,65536,262144,1048576 $T 400 python tools/ab_c5s.py > $O/ab_c5s_caps.jsonl 2> $O/ab_c5s.err || { tail -5 $O/ab_c5s.err; exit 1; }
cat $O/ab_c5s_caps.jsonl
