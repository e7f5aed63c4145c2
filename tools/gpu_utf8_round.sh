# UTF-8 paths after a change: the parity tests that cover them, the C5
# descriptor timing per variant library, and a kernel trace of the C5 stream
# decode with UTF-8 flags (product library)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_sorted_utf8.py tests/test_gpu_decode.py tests/test_gpu_configs.py tests/test_gpu_pipe.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/utf8_tests.log 2>&1 || { tail -30 gpurun_out/utf8_tests.log; exit 1; }
tail -1 gpurun_out/utf8_tests.log
bash tools/gpu_utf8_exp.sh "$@" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_c5s -o run -- python3 $R/tools/run_c5.py > $R/gpurun_out/prof_c5s.log 2>&1 || { tail -5 $R/gpurun_out/prof_c5s.log; exit 1; }
echo done
