# seam records (C5 descriptor UTF-8) + fused tests
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sorted_utf8.py tests/test_gpu_fused.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/iter2_tests.log 2>&1
rc=$?
tail -5 gpurun_out/iter2_tests.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/kt_c5d -o run -- python3 $GRAFT_REPO_ROOT/tools/run_c5_desc.py > $GRAFT_REPO_ROOT/gpurun_out/kt_c5d.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && f=$(find gpurun_out/kt_c5d -name "*kernel_stats.csv" | head -1) && cut -d, -f1-8 $f | head -8
