# all GPU parity tests + bench extras + kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --extra --no-cpu --steps 50 > gpurun_out/bench_extra.log 2>&1 || { tail -20 gpurun_out/bench_extra.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_q -o run -- python3 $R/bench.py --extra --no-cpu --steps 20 --warmup 2 > $R/gpurun_out/prof_q.log 2>&1
echo done
