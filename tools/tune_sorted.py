#!/usr/bin/env python3
"""Early-load on/off x grid-cap sweep of k_unmask_sorted on the C2 batch (HIP events, 4 rotating
buffers). usage: python tools/tune_sorted.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu, lib  # noqa: E402



def main():
    dev = torch.device("cuda:0")
    wire, descs, _ = gpu.config_c2()
    n = len(descs)
    ctx = gpu.Ctx(0, max_frames=n, max_stream_bytes=len(wire))
    bufs = [torch.from_numpy(wire).to(dev) for _ in range(4)]
    dd = gpu.descs_to_device(descs, dev)
    out = {}
    for early, cap in [(e, c) for e in (1, 0) for c in (8192, 16384, 32768)]:
        lib().fws_internal_set_sorted_early(early)
        lib().fws_internal_set_grid_cap(cap)
        for i in range(20):
            gpu.unmask_sorted(ctx, bufs[i % 4], dd, n)
        ts = []
        for rep in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for i in range(200):
                gpu.unmask_sorted(ctx, bufs[i % 4], dd, n)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 200 * 1e3)
        out[f"early{early}_grid{cap}"] = round(min(ts), 2)
        print(early, cap, out[f"early{early}_grid{cap}"], flush=True)
    lib().fws_internal_set_grid_cap(0)
    lib().fws_internal_set_sorted_early(0)
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
