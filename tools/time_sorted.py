#!/usr/bin/env python3
"""The headline step alone: fws_gpu_unmask_sorted on the C2 batch (4 rotating
256 MiB buffers, HIP events over back-to-back calls, repeated 5 times; median
and min), for A/B builds. usage: python tools/time_sorted.py [--lib PATH] [steps]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib  # noqa: E402
if "--lib" in sys.argv:
    _lib.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
from flashws_amd import gpu  # noqa: E402

ALG = 537_395_200


def main():
    steps = int(sys.argv[-1]) if sys.argv[-1].isdigit() else 200
    dev = torch.device("cuda:0")
    wire, descs, _ = gpu.config_c2()
    n = len(descs)
    ctx = gpu.Ctx(0, max_frames=n, max_stream_bytes=len(wire))
    bufs = [torch.from_numpy(wire).to(dev) for _ in range(4)]
    dd = gpu.descs_to_device(descs, dev)
    for i in range(20):
        gpu.unmask_sorted(ctx, bufs[i % 4], dd, n)
    torch.cuda.synchronize()
    runs = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(steps):
            gpu.unmask_sorted(ctx, bufs[i % 4], dd, n)
        e1.record()
        torch.cuda.synchronize()
        runs.append(e0.elapsed_time(e1) * 1e3 / steps)
    runs.sort()
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "us_median": round(runs[2], 2), "us_min": round(runs[0], 2),
                      "frac_median": round(ALG / runs[2] / 8e6, 4), "runs": [round(r, 2) for r in runs]}))
    ctx.close()


if __name__ == "__main__":
    main()
