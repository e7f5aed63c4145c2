set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_session.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe_tests.log 2>&1 || { tail -30 gpurun_out/pipe_tests.log; exit 1; }
tail -1 gpurun_out/pipe_tests.log
timeout -k 10 300 python bench.py --extra --no-cpu --steps 50 > gpurun_out/bench_extra.log 2>&1 || { tail -20 gpurun_out/bench_extra.log; exit 1; }
echo ok
