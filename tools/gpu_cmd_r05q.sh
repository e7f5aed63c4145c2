set -o pipefail
O=gpurun_out/r05; mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread > $O/dropin_tests.log 2>&1 || { tail -30 $O/dropin_tests.log; exit 1; }
tail -1 $O/dropin_tests.log
$T 400 python bench.py --only c1 --no-cpu --no-batch-extra --steps 5 --warmup 2 > $O/bench_c1.json 2> $O/bench_c1.err || { tail -5 $O/bench_c1.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$O/bench_c1.json').read().splitlines()[-1])
for k,v in d['extra']['C1_echo'].items():
    if isinstance(v, dict): print(k, v.get('goodput_rx_tx_mbps'), (v.get('rtt_us') or {}).get('p50'), v.get('gpu_reads'), v.get('gpu_batches'))"
