# phase clocks of k_scan and per-workgroup timelines of k_merge / k_link / k_emit (FWS_SCAN_PROF build)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 200 python -u tools/prof_scan.py > gpurun_out/prof_scan.json 2> gpurun_out/prof_scan.err &&
timeout -k 10 200 python -u tools/prof_merge_trace.py > gpurun_out/prof_merge.json 2> gpurun_out/prof_merge.err
rc=$?; tail -3 gpurun_out/prof_scan.err gpurun_out/prof_merge.err; exit $rc
