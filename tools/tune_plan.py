#!/usr/bin/env python3
"""Timing experiments on k_plan (fws_internal_set_plan_dbg: 1 no ticket, 2 no
look-back, 4 no unit maps; results are wrong except for 0 -- timing only):
plan-only launches on C2 / C3 descriptors, HIP events."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu, lib  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    L = lib()
    setd = L.fws_internal_set_plan_dbg
    setd.argtypes = [C.c_int]
    setd.restype = C.c_int
    res = {}
    for cfg in ("C2", "C3"):
        wire, descs, _ = gpu.config_c2() if cfg == "C2" else gpu.config_c3()
        n = len(descs)
        ctx = gpu.Ctx(0, max_frames=n, max_stream_bytes=len(wire))
        buf = torch.from_numpy(wire).to(dev)
        dd = gpu.descs_to_device(descs, dev)
        times = {}
        bufs = [buf] + [torch.from_numpy(wire).to(dev) for _ in range(3)]
        for rnd in range(3):
            for with_run in (0, 1):
                for dbg in (0, 1, 2, 3, 4, 7):
                    setd(dbg)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    e0.record()
                    for i in range(20):
                        gpu.unmask_plan(ctx, bufs[i % 4], dd, n)
                        if with_run:
                            setd(0)
                            gpu.unmask_run(ctx, bufs[i % 4], dd, n)
                            setd(dbg)
                    e1.record()
                    torch.cuda.synchronize()
                    times.setdefault(f"{dbg}{'r' if with_run else ''}", []).append(e0.elapsed_time(e1) / 20 * 1e3)
        setd(0)
        res[cfg] = {str(k): round(float(np.median(v)), 2) for k, v in times.items()}
        print(cfg, res[cfg], flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
