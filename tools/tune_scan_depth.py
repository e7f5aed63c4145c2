#!/usr/bin/env python3
"""k_scan prefetch depth (fws_internal_set_scan_depth: tiles in flight per
wavefront, 2..4): C2-stream and C3 decode per depth, HIP events, results
checked equal across depths. Run under rocprofv3 --kernel-trace to split the
k_scan time (dispatches come in depth order, 12 per depth per config)."""
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
    setd = lib().fws_internal_set_scan_depth
    setd.argtypes = [C.c_int]
    setd.restype = C.c_int
    out = {}
    for name, mk in (("C2", gpu.config_c2), ("C3", gpu.config_c3)):
        wire, descs, _ = mk()
        n = len(descs)
        ctx = gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(wire))
        bufs = [torch.from_numpy(wire).to(dev) for _ in range(4)]
        cap = n + 64
        frames = torch.empty(cap * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev)
        res = torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev)
        ref = None
        for depth in (2, 3, 4):
            setd(depth)
            for i in range(12):
                rc, _, _, _ = gpu.decode_stream(ctx, bufs[i % 4], cap, frames=frames, result=res)
                assert rc == 0
            torch.cuda.synchronize()
            r = gpu.read_result(res)
            fr = frames[:n * gpu.FRAME_INFO.itemsize].cpu()
            if ref is None:
                ref = (int(r["n_frames"]), fr)
            assert int(r["n_frames"]) == ref[0] == n and torch.equal(fr, ref[1]), (name, depth)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(20):
                gpu.decode_stream(ctx, bufs[i % 4], cap, frames=frames, result=res)
            e1.record()
            torch.cuda.synchronize()
            out.setdefault(name, {})[depth] = round(e0.elapsed_time(e1) / 20 * 1e3, 2)
        setd(2)
        ctx.close()
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
