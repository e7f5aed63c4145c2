set -o pipefail
O=gpurun_out/r05; mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_sorted_utf8.py tests/test_gpu_decode.py tests/test_gpu_configs.py -k "utf8 or c5 or C5 or text" -x -q --timeout 120 --timeout-method thread > $O/utf8_tests.log 2>&1 || { tail -30 $O/utf8_tests.log; exit 1; }
tail -1 $O/utf8_tests.log
$T 300 python bench.py --only c5d --no-cpu --no-batch-extra --steps 20 --warmup 5 > $O/bench_c5d.json 2> $O/bench_c5d.err || { tail -5 $O/bench_c5d.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_c5d.json').read().splitlines()[-1]);e=d['extra']['C5_utf8_descriptor'];print(e['ms_per_step'], e.get('roofline',{}).get('frac'), e.get('checked_call_status'))"
(cd /tmp && TMPDIR=/tmp $T 300 rocprofv3 --kernel-trace --stats -f csv -d $OLDPWD/$O/prof_c5d2 -o run -- python3 $OLDPWD/bench.py --only c5d --no-cpu --no-batch-extra --steps 10 --warmup 3) > $O/prof_c5d2.log 2>&1 || { tail -5 $O/prof_c5d2.log; exit 1; }
cut -d, -f1-4 $O/prof_c5d2/run_kernel_stats.csv | head -8
