# decode-path GPU tests, then the C2/C3 kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_pipe.py tests/test_gpu_configs.py tests/test_gpu_session.py tests/test_gpu_limits.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/dec_tests.log 2>&1 || { tail -30 gpurun_out/dec_tests.log; exit 1; }
tail -2 gpurun_out/dec_tests.log
bash tools/gpu_kt_decode.sh

timeout -k 10 200 python tools/prof_merge_trace.py > gpurun_out/merge_trace.json 2> gpurun_out/merge_trace.err || true
