# full GPU pass: tests, smoke, bench (+extras, C5, CPU baseline), kernel stats of the same bench
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python bench.py --extra --c5 --cpu-seconds 10 > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_full -o run -- python3 $R/bench.py --extra --c5 --no-cpu --steps 20 --warmup 2 > $R/gpurun_out/prof_full.log 2>&1
echo done
