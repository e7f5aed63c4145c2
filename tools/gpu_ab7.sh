#!/bin/bash
# r06: k_scan with LDS-DMA tile staging (libfws_gpu_scandma.so, FWS_SCAN_DMA=1, 6 workgroups per CU)
# against the product scan (register staging, 8 per CU): parity of the decode suite, then k_scan alone and
# whole decodes, alternating builds
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
FWS_LIB_VARIANT=scandma timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > $O/t_scandma.log 2>&1 || { tail -30 $O/t_scandma.log; exit 1; }
tail -1 $O/t_scandma.log
for rep in 1 2; do
  for lib in libfws_gpu_scandma.so libfws_gpu.so; do
    timeout -k 10 200 python tools/scan_ablation.py --lib flashws_amd/lib/$lib 50 2>/dev/null | grep -v amdgpu >> $O/ab_scandma.jsonl || exit 1
    timeout -k 10 200 python tools/time_decode.py 20 --lib flashws_amd/lib/$lib 2>/dev/null | grep -v amdgpu >> $O/ab_scandma.jsonl || exit 1
  done
done
cat $O/ab_scandma.jsonl
