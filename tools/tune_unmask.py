#!/usr/bin/env python3
"""Interleaved A/B timing of the k_unmask variants on BASELINE C2 (and C3
descriptors), plus torch's device copy of the same bytes as the box's
achievable read+write HBM reference. Variants via the tuning hook
fws_internal_set_unmask_variant (0 = per-lane search, 1..3 = fast G=1/2/4,
5..7 = same + nontemporal). Each variant's parity is checked first."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu, lib  # noqa: E402

VARIANTS = [0, 1, 5]


def main():
    dev = torch.device("cuda:0")
    L = lib()
    setv = L.fws_internal_set_unmask_variant
    setv.argtypes = [C.c_int]
    setv.restype = C.c_int
    setg = L.fws_internal_set_grid_cap
    setg.argtypes = [C.c_int]
    setg.restype = C.c_int
    res = {}
    for cfg in ("C2", "C3"):
        wire, descs, _ = gpu.config_c2() if cfg == "C2" else gpu.config_c3()
        n = len(descs)
        ctx = gpu.Ctx(0, max_frames=n, max_stream_bytes=len(wire))
        bufs = [torch.from_numpy(wire).to(dev) for _ in range(4)]
        dd = gpu.descs_to_device(descs, dev)
        gpu.unmask_plan(ctx, bufs[0], dd, n)
        ref = bufs[0].clone()
        gpu.unmask_run(ctx, ref, dd, n)
        for v in VARIANTS:                      # parity of every variant vs variant 0 output
            setv(v)
            t = bufs[1].clone()
            gpu.unmask_run(ctx, t, dd, n)
            setv(0)
            assert torch.equal(t, ref) or v == 0, f"variant {v} mismatch"
        alg = len(wire) + int(descs["payload_len"].sum())
        keys = VARIANTS + ["copy", "mask_single", "g1nt_grid2048", "g1nt_grid4096", "g1nt_grid16384",
                           "g1_grid16384"]
        times = {v: [] for v in keys}
        dst = torch.empty_like(bufs[0])
        steps = 20
        for rnd in range(5):
            for v in keys:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                if isinstance(v, int):
                    setv(v)
                elif v.startswith("g"):
                    setv(5 if v.startswith("g1nt") else 1)
                    setg(int(v.split("grid")[1]))
                torch.cuda.synchronize()
                e0.record()
                for i in range(steps):
                    if v == "copy":
                        dst.copy_(bufs[i % 4])
                    elif v == "mask_single":
                        gpu.ws_mask_bytes_fast(bufs[i % 4], 0x12345678)
                    else:
                        gpu.unmask_run(ctx, bufs[i % 4], dd, n)
                setg(8192)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / steps * 1e3)
        out = {}
        for v, ts in times.items():
            us = float(np.median(ts))
            nbytes = 2 * len(wire) if v in ("copy", "mask_single") else alg
            out[str(v)] = {"us_median": round(us, 2), "us_min": round(min(ts), 2),
                           "GB_per_s": round(nbytes / us / 1e3, 1)}
        res[cfg] = out
        ctx.close()
        del bufs
    setv(5)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
