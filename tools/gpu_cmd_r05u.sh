set -o pipefail
O=gpurun_out/r05; mkdir -p $O
T="timeout -k 10"
$T 400 python tools/ab_c5s.py > $O/ab_c5s_pf_grid.jsonl 2> $O/ab_c5s.err || { tail -5 $O/ab_c5s.err; exit 1; }
cat $O/ab_c5s_pf_grid.jsonl | cut -c1-120
: > $O/ab_c5d_wpe.jsonl
for v in wpe8 "" wpe8 ""; do
  FWS_LIB_VARIANT=$v $T 200 python tools/ab_c5d.py >> $O/ab_c5d_wpe.jsonl 2>> $O/ab_c5d.err || exit 1
done
grep pipe0 $O/ab_c5d_wpe.jsonl
bash tools/gpu_round.sh share2 || exit 1
