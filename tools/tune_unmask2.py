#!/usr/bin/env python3
"""Interleaved A/B timing of descriptor-mode unmask variants (tuning hook
fws_internal_set_unmask_variant: 5 = k_unmask_fast nt grid-stride, 6 =
k_unmask_one, one unit per wave) on BASELINE C2 and C3 descriptors, kernel
only (unmask_run) and whole step (plan + run). Parity vs variant 0 first."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu, lib  # noqa: E402

VARIANTS = [int(v) for v in os.environ.get("FWS_VARIANTS", "5,6").split(",")]


def main():
    dev = torch.device("cuda:0")
    L = lib()
    setv = L.fws_internal_set_unmask_variant
    setv.argtypes = [C.c_int]
    setv.restype = C.c_int
    setg = L.fws_internal_set_grid_cap
    setg.argtypes = [C.c_int]
    setg.restype = C.c_int
    caps = [int(c) for c in os.environ.get("FWS_GRID_CAPS", "16384").split(",")]
    res = {}
    for cfg in ("C2", "C3"):
        wire, descs, _ = gpu.config_c2() if cfg == "C2" else gpu.config_c3()
        n = len(descs)
        ctx = gpu.Ctx(0, max_frames=n, max_stream_bytes=len(wire))
        bufs = [torch.from_numpy(wire).to(dev) for _ in range(4)]
        dd = gpu.descs_to_device(descs, dev)
        gpu.unmask_plan(ctx, bufs[0], dd, n)
        setv(0)
        ref = bufs[0].clone()
        gpu.unmask_run(ctx, ref, dd, n)
        for v in VARIANTS:
            setv(v)
            t = bufs[1].clone()
            gpu.unmask_run(ctx, t, dd, n)
            assert torch.equal(t, ref), f"variant {v} mismatch on {cfg}"
        alg = len(wire) + int(descs["payload_len"].sum())
        times = {}
        steps = 40
        for rnd in range(6):
            for v, cap in [(v, c) for v in VARIANTS for c in caps]:
                for mode in ("run", "step"):
                    setv(v)
                    setg(cap)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    e0.record()
                    for i in range(steps):
                        if mode == "run":
                            gpu.unmask_run(ctx, bufs[i % 4], dd, n)
                        else:
                            gpu.unmask_batch(ctx, bufs[i % 4], dd, n)
                    e1.record()
                    torch.cuda.synchronize()
                    times.setdefault(f"v{v}_g{cap}_{mode}", []).append(e0.elapsed_time(e1) / steps * 1e3)
        out = {}
        for k, ts in times.items():
            us = float(np.median(ts))
            out[k] = {"us_median": round(us, 2), "us_min": round(min(ts), 2),
                      "alg_GB_per_s": round(alg / us / 1e3, 1)}
        res[cfg] = out
        ctx.close()
        print(cfg, json.dumps(out), flush=True)
    json.dump(res, open(sys.argv[1] if len(sys.argv) > 1 else "/dev/stdout", "w"), indent=1)


if __name__ == "__main__":
    main()
