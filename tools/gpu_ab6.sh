#!/bin/bash
# r06: TX encode with the seam chunks after the full ones (k_tx_encode_late) at 8 / 7 / 6 waves per SIMD
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread > $O/t_txlate.log 2>&1 || { tail -30 $O/t_txlate.log; exit 1; }
tail -1 $O/t_txlate.log
for v in "" txw7 txw6; do
  FWS_LIB_VARIANT=$v timeout -k 10 200 python -u tools/ab_tx.py 100 plan,plan_late > $O/ab_txlate_${v:-w8}.jsonl 2>&1 || { tail -5 $O/ab_txlate_${v:-w8}.jsonl; exit 1; }
  grep -v amdgpu.ids $O/ab_txlate_${v:-w8}.jsonl
done
