# Round measurement pass on one MI355X: GPU tests, smoke, full bench (extras,
# C5, CPU baseline), PMC traffic passes for the headline kernel, kernel stats
# (headline bench, C4 gather, TX encode; rocprofv3 of the --extra bench
# segfaults at interpreter exit on this image, so the extras are profiled by
# their own small drivers).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python bench.py --extra --c5 --cpu-seconds 10 > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --no-extra --no-cpu --no-batch-extra --steps 10 --warmup 2 > $R/gpurun_out/pmc_fetch.log 2>&1 || { tail -5 $R/gpurun_out/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --no-extra --no-cpu --no-batch-extra --steps 10 --warmup 2 > $R/gpurun_out/pmc_write.log 2>&1 || { tail -5 $R/gpurun_out/pmc_write.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_main -o run -- python3 $R/bench.py --no-extra --no-cpu > $R/gpurun_out/prof_main.log 2>&1 || { tail -5 $R/gpurun_out/prof_main.log; exit 1; }
timeout -k 10 100 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_c4 -o run -- python3 $R/tools/run_c4.py > $R/gpurun_out/prof_c4.log 2>&1 || { tail -5 $R/gpurun_out/prof_c4.log; exit 1; }
timeout -k 10 100 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_tx -o run -- python3 $R/tools/run_tx.py > $R/gpurun_out/prof_tx.log 2>&1 || { tail -5 $R/gpurun_out/prof_tx.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_c5d -o run -- python3 $R/tools/run_c5_desc.py > $R/gpurun_out/prof_c5d.log 2>&1 || { tail -5 $R/gpurun_out/prof_c5d.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_c5 -o run -- python3 $R/tools/run_c5.py > $R/gpurun_out/prof_c5.log 2>&1 || { tail -5 $R/gpurun_out/prof_c5.log; exit 1; }
echo done
