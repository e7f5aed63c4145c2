set -o pipefail
O=gpurun_out/r05; mkdir -p $O
T="timeout -k 10"
: > $O/ab_c5d_lookup_vs_swar.jsonl
for v in swar "" swar ""; do
  FWS_LIB_VARIANT=$v $T 200 python tools/ab_c5d.py >> $O/ab_c5d_lookup_vs_swar.jsonl 2>> $O/ab_c5d.err || exit 1
done
grep -v plain $O/ab_c5d_lookup_vs_swar.jsonl
: > $O/ab_c5_lookup_vs_swar.jsonl
for v in swar "" swar ""; do
  FWS_LIB_VARIANT=$v $T 300 python bench.py --only c5s --no-cpu --no-batch-extra --steps 16 --warmup 4 > $O/ab_c5s_one.json 2>> $O/ab_c5.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/ab_c5s_one.json').read().splitlines()[-1]);print('variant=${v:-product}', d['extra']['C5_utf8_text_decode']['ms_per_step'])" | tee -a $O/ab_c5_lookup_vs_swar.jsonl
done
