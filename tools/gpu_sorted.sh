# fws_gpu_unmask_sorted: parity tests, bench (value + batch extra), kernel stats, PMC traffic
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_unmask.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_unmask_tests.log 2>&1 || { tail -30 gpurun_out/gpu_unmask_tests.log; exit 1; }
tail -1 gpurun_out/gpu_unmask_tests.log
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/bench_sorted.log 2>&1 || { tail -20 gpurun_out/bench_sorted.log; exit 1; }
tail -1 gpurun_out/bench_sorted.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_sorted -o run -- python3 $R/bench.py --no-extra --no-cpu > $R/gpurun_out/prof_sorted.log 2>&1 || { tail -5 $R/gpurun_out/prof_sorted.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/pmc_fetch_s -o run -- python3 $R/bench.py --no-extra --no-cpu --no-batch-extra --steps 10 --warmup 2 > $R/gpurun_out/pmc_fetch_s.log 2>&1 || { tail -5 $R/gpurun_out/pmc_fetch_s.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/pmc_write_s -o run -- python3 $R/bench.py --no-extra --no-cpu --no-batch-extra --steps 10 --warmup 2 > $R/gpurun_out/pmc_write_s.log 2>&1 || { tail -5 $R/gpurun_out/pmc_write_s.log; exit 1; }
echo done
