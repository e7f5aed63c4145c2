set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_fused.py tests/test_gpu_configs.py tests/test_gpu_pipe.py > gpurun_out/it9_tests.log 2>&1 || { tail -30 gpurun_out/it9_tests.log; exit 1; }
tail -1 gpurun_out/it9_tests.log
cd /tmp && export TMPDIR=/tmp
for c in dense c3; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/kt_$c -o run -- python3 $R/tools/run_decode.py $c 12 > $R/gpurun_out/kt_$c.log 2>&1 || exit 1
done
echo done
