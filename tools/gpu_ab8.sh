#!/bin/bash
# r06: k_scan LDS-DMA staging vs register staging: SQ counters of the C3 decode per build, and k_scan alone x5
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
R=${GRAFT_REPO_ROOT:-$(pwd)}
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM"
for v in scandma ""; do
  tag=${v:-product}
  (cd /tmp && FWS_LIB_VARIANT=$v TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc $C -f csv -d $R/$O/sq_scan_$tag -o run -- python3 $R/tools/run_decode.py c3) > $O/sq_scan_$tag.log 2>&1 || { tail -5 $O/sq_scan_$tag.log; exit 1; }
done
for rep in 1 2 3 4 5; do
  for lib in libfws_gpu_scandma.so libfws_gpu.so; do
    timeout -k 10 200 python tools/scan_ablation.py --lib flashws_amd/lib/$lib 100 2>/dev/null | grep -v amdgpu >> $O/ab_scandma2.jsonl || exit 1
  done
done
cat $O/ab_scandma2.jsonl
