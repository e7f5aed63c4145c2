set -o pipefail
O=gpurun_out/r05; mkdir -p $O
T="timeout -k 10"
: > $O/ab_land.jsonl
for v in land7 "" land7 ""; do
  FWS_LIB_VARIANT=$v $T 300 python bench.py --only c3,c2s,dense,c5s --no-cpu --no-batch-extra --steps 20 --warmup 5 > $O/ab_scan_one.json 2>> $O/ab_scan.err || { tail -5 $O/ab_scan.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/ab_scan_one.json').read().splitlines()[-1])
print('variant=${v:-product}', [(k[:6], e.get('ms_per_step'), (e.get('two_in_flight') or {}).get('ms_per_batch')) for k,e in d['extra'].items()])" | tee -a $O/ab_land.jsonl
done
$T 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $O/dec_tests.log 2>&1 || { tail -30 $O/dec_tests.log; exit 1; }
tail -1 $O/dec_tests.log
