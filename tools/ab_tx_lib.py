#!/usr/bin/env python3
"""Time the C2-shaped TX encode (4 rotating sources) with the library named by
FWS_LIB_VARIANT (an in-tree `make exp` build) -- one process per build, for
ablations that change the kernel's output (no cross-build compare).
usage: FWS_LIB_VARIANT=tag python tools/ab_tx_lib.py [reps]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import run_tx  # noqa: E402
from flashws_amd import _lib, gpu  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    ctx, outs, srcs, dd, n, total = run_tx.setup()
    for i in range(40):
        gpu.encode_frames(ctx, outs[i % 4], srcs[i % 4], dd, n)
    for rep in range(3):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            gpu.encode_frames(ctx, outs[i % 4], srcs[i % 4], dd, n)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "rep": rep, "ms": round(ms, 4),
                          "frac": round((n * 4096 + total) / ms / 1e-3 / 8e12, 4)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
