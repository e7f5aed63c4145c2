# decode parity tests (both resolve paths) + phase profile + bench extras
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_session.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dec_tests.log 2>&1 || { tail -30 gpurun_out/dec_tests.log; exit 1; }
tail -1 gpurun_out/dec_tests.log
timeout -k 10 200 python tools/prof_scan.py > gpurun_out/prof_scan.json 2>gpurun_out/prof_scan.err || { tail -5 gpurun_out/prof_scan.err; exit 1; }
timeout -k 10 300 python bench.py --extra --no-cpu --steps 50 > gpurun_out/bench_extra.log 2>&1 || { tail -20 gpurun_out/bench_extra.log; exit 1; }
echo ok
