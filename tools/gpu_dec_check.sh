# decode parity tests after a resolve change, then the decode kernel traces
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_configs.py tests/test_gpu_session.py tests/test_gpu_mux.py tests/test_gpu_pipe.py tests/test_gpu_limits.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/dec_tests.log 2>&1 || { tail -30 gpurun_out/dec_tests.log; exit 1; }
tail -1 gpurun_out/dec_tests.log
bash tools/gpu_kt_decode.sh || exit 1
echo dec-done
