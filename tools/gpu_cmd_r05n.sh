set -o pipefail
O=gpurun_out/r05; mkdir -p $O
T="timeout -k 10"
: > $O/ab_st.jsonl
for v in st256 "" st256 ""; do
  FWS_LIB_VARIANT=$v $T 300 python bench.py --only c3,dense,c2s,c5s --no-cpu --no-batch-extra --steps 20 --warmup 5 > $O/ab_st_one.json 2>> $O/ab_st.err || { tail -5 $O/ab_st.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/ab_st_one.json').read().splitlines()[-1])
print('variant=${v:-product}', [(k[:6], e.get('ms_per_step')) for k,e in d['extra'].items()])" | tee -a $O/ab_st.jsonl
done
