# round-2 closing measurements: full -m gpu suite + smoke + default bench line,
# a kernel trace (stats) of the same default bench command, the decode kernel
# traces, the C5 stream-decode trace, and the C1 echo table
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_r02_tests.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || { tail -5 $R/gpurun_out/prof_bench.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_c5s -o run -- python3 $R/tools/run_c5.py > $R/gpurun_out/prof_c5s.log 2>&1 || exit 1
bash $R/tools/gpu_kt_decode.sh || exit 1
cd $R
bash tools/gpu_echo.sh || exit 1
echo final-done
