# round-2 closing pass on the committed tree: full -m gpu suite, smoke, default bench
# line, rocprofv3 kernel stats of the same bench command, decode kernel traces
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_r02_tests.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || { tail -5 $R/gpurun_out/prof_bench.err; exit 1; }
bash $R/tools/gpu_kt_decode.sh || exit 1
echo close-done
