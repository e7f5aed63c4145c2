#!/bin/bash
# r06: write-through nontemporal streaming stores in the unmask kernels (default
# build) against the r05 nontemporal stores (libfws_gpu_ntst.so: FWS_UNMASK_WT=0),
# parity first, then alternating bench runs
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_unmask.py tests/test_gpu_sorted_utf8.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > $O/t_wt2.log 2>&1 || { tail -30 $O/t_wt2.log; exit 1; }
tail -1 $O/t_wt2.log
summ() {
python3 - $1 $2 <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ex = d.get("extra", {})
out = {"lib": sys.argv[2], "C2_us": d["roofline"]["kernel_us"], "C2_frac": d["roofline"]["frac"]}
for k in ("C3_mixed_stream_decode", "dense_64B_stream_decode", "C2_stream_decode", "C4_fragmented_reassemble",
          "C2_tx_encode", "C5_utf8_text_decode", "C5_utf8_descriptor"):
    if k in ex: out[k] = ex[k].get("ms_per_step")
print(json.dumps(out))
PY
}
for rep in 1 2; do
  for v in "" ntst; do
    tag=${v:-wt}
    FWS_LIB_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu --no-batch-extra --only c3,dense,c2s,c4,tx --steps 100 --warmup 10 > $O/ab_wt_${tag}_$rep.json 2> $O/ab_wt_${tag}_$rep.err || { tail -5 $O/ab_wt_${tag}_$rep.err; exit 1; }
    summ $O/ab_wt_${tag}_$rep.json $tag
  done
done
for v in "" ntst; do
  tag=${v:-wt}
  FWS_LIB_VARIANT=$v timeout -k 10 400 python bench.py --no-cpu --no-batch-extra --c5 --only c5s,c5d --steps 20 --warmup 5 > $O/ab_wt5_${tag}.json 2> $O/ab_wt5_${tag}.err || { tail -5 $O/ab_wt5_${tag}.err; exit 1; }
  summ $O/ab_wt5_${tag}.json $tag
done
