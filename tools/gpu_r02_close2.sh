# round-2 closing pass (after the k_scan direct-node path and the k_merge walk fix):
# full -m gpu suite, smoke, the default bench line under a kernel trace, decode traces
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke-ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || { tail -5 $R/gpurun_out/prof_bench.err; exit 1; }
echo bench-ok
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_c5s -o run -- python3 $R/tools/run_c5.py > $R/gpurun_out/prof_c5s.log 2>&1 || exit 1
bash $R/tools/gpu_kt_decode.sh || exit 1
echo close-done
