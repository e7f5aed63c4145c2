set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 200 python -u tools/prof_merge_trace.py > gpurun_out/prof_merge.json 2> gpurun_out/prof_merge.err || exit 1
timeout -k 10 200 python -u tools/prof_merge_trace.py > gpurun_out/prof_merge2.json 2> gpurun_out/prof_merge2.err || exit 1
echo done
