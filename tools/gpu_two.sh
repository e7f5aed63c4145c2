set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 120 python3 tools/run_two.py 16 > gpurun_out/two.log 2>&1 || { tail -5 gpurun_out/two.log; exit 1; }
cat gpurun_out/two.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/two_trace -o run -- python3 $R/tools/run_two.py 16 > $R/gpurun_out/two_trace.log 2>&1 || { tail -5 $R/gpurun_out/two_trace.log; exit 1; }
echo done
