set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 python tools/prof_merge_trace.py > gpurun_out/merge_trace.json 2> gpurun_out/merge_trace.err || { tail -5 gpurun_out/merge_trace.err; exit 1; }
echo done
