# one-pass decode A/B and a kernel trace of the C3 decode (tools/run_fused_ab.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/run_fused_ab.py 40 > gpurun_out/fused_ab.txt 2>&1 || { cat gpurun_out/fused_ab.txt; exit 1; }
cat gpurun_out/fused_ab.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fused_c3 -o run -- python3 $GRAFT_REPO_ROOT/tools/run_decode.py c3 12 > $GRAFT_REPO_ROOT/gpurun_out/prof_fused_c3.log 2>&1
cd $GRAFT_REPO_ROOT && find gpurun_out/prof_fused_c3 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/fused_c3_kernel_stats.csv && cut -d, -f1-8 gpurun_out/fused_c3_kernel_stats.csv | head -12
