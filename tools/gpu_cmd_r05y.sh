set -o pipefail
O=gpurun_out/r05; mkdir -p $O
: > $O/ab_scan_rec.jsonl
for v in recall "" recall "" ; do
  FWS_LIB_VARIANT=$v timeout -k 10 300 python bench.py --only c2s,c3,dense,c5s --no-cpu --no-batch-extra --steps 20 --warmup 5 >> $O/ab_scan_rec.jsonl 2>> $O/ab_scan_rec.err || { tail -5 $O/ab_scan_rec.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/ab_scan_rec.jsonl').read().splitlines()[-1]);e=d['extra'];print('variant=${v:-product}', [(k[:6], v.get('ms_per_step'), (v.get('two_in_flight') or {}).get('ms_per_batch')) for k,v in e.items() if isinstance(v,dict) and 'ms_per_step' in v])"
done
