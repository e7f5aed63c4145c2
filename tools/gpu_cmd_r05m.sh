set -o pipefail
O=gpurun_out/r05; mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_configs.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $O/dec_tests.log 2>&1 || { tail -30 $O/dec_tests.log; exit 1; }
tail -1 $O/dec_tests.log
$T 400 python bench.py --only c5s,c3,dense --no-cpu --no-batch-extra --steps 20 --warmup 5 > $O/bench_dec.json 2> $O/bench_dec.err || { tail -5 $O/bench_dec.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$O/bench_dec.json').read().splitlines()[-1])
for k,e in d['extra'].items(): print(k, e.get('ms_per_step'), e.get('roofline',{}).get('frac'), e.get('big_super_tiles'), e.get('flags_match_generator'))"
