# stream-mode UTF-8 seam records: utf8 decode tests, full C5 configs, C5 stream trace
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_configs.py tests/test_gpu_sorted_utf8.py tests/test_gpu_pipe.py -k "utf8 or c5 or C5 or pipe" -x -q --timeout 200 --timeout-method thread > gpurun_out/iter3_tests.log 2>&1
rc=$?
tail -4 gpurun_out/iter3_tests.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/kt_c5s -o run -- python3 $GRAFT_REPO_ROOT/tools/run_c5.py > $GRAFT_REPO_ROOT/gpurun_out/kt_c5s.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && f=$(find gpurun_out/kt_c5s -name "*kernel_stats.csv" | head -1) && cut -d, -f1-4 $f | head -10
