set -o pipefail
O=gpurun_out/r05; mkdir -p $O
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread > $O/tx_tests.log 2>&1 || { tail -30 $O/tx_tests.log; exit 1; }
tail -1 $O/tx_tests.log
$T 300 python bench.py --only tx --no-cpu --no-batch-extra --steps 20 --warmup 5 > $O/bench_tx.json 2> $O/bench_tx.err || { tail -5 $O/bench_tx.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_tx.json').read().splitlines()[-1]);e=d['extra']['C2_tx_encode'];print(e['ms_per_step'], e.get('roofline',{}).get('frac'))"
