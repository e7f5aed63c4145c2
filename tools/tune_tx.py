#!/usr/bin/env python3
"""A/B of k_tx_encode (compiler's allocation, 4 waves/SIMD) vs k_tx_encode_w5 (the default)
(5 waves/SIMD) on the C2 TX shape, HIP events; outputs checked equal.

usage: python tools/tune_tx.py [--lib PATH]   (--lib: an A/B build; the output's sha256 is printed)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib  # noqa: E402
if "--lib" in sys.argv:
    _lib.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
from flashws_amd import gpu, lib  # noqa: E402
import run_tx  # noqa: E402


def main(steps=100):
    ctx, outs, srcs, dd, n, total = run_tx.setup()
    src = srcs[0]   # (r06: setup returns 4 rotating copies; this tool times one)
    res, ref = {}, None
    for w5 in ((1, 0, 1, 0, 1, 0) if "--rev" in sys.argv else (0, 1, 0, 1)):
        lib().fws_internal_set_tx_w5(w5)
        for i in range(10):
            gpu.encode_frames(ctx, outs[i % 4], src, dd, n)
        torch.cuda.synchronize()
        got = outs[0][:total].clone()
        ref = got if ref is None else ref
        assert torch.equal(ref, got)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(steps):
            gpu.encode_frames(ctx, outs[i % 4], src, dd, n)
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(f"w5={w5}", []).append(round(e0.elapsed_time(e1) / steps * 1e3, 2))
    lib().fws_internal_set_tx_w5(1)
    import hashlib
    sha = hashlib.sha256(ref.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "tx_step_us": res, "out_sha16": sha}))
    ctx.close()


if __name__ == "__main__":
    main()
