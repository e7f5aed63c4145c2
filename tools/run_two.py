#!/usr/bin/env python3
"""C3 stream decode with two batches in flight (two contexts, two streams,
batches alternate) for a kernel-trace look at how the two streams overlap.

usage: python tools/run_two.py [reps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    wire, descs, _ = gpu.config_c3()
    dev = torch.device("cuda:0")
    n = len(descs)
    ctxs = [gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(wire)) for _ in range(2)]
    ws = [torch.from_numpy(wire).to(dev) for _ in range(4)]
    sts = [gpu.hip_stream(), gpu.hip_stream()]
    fr = [torch.empty((n + 64) * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]
    rs = [torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]

    def step(i):
        rc, _, _, _ = gpu.decode_stream(ctxs[i % 2], ws[i % 4], n + 64, frames=fr[i % 2], result=rs[i % 2],
                                        stream=sts[i % 2])
        assert rc == 0
    for i in range(4):
        step(i)
    torch.cuda.synchronize()
    for mode in ("serial", "two"):
        t0 = time.perf_counter()
        for i in range(reps):
            if mode == "serial":
                rc, _, _, _ = gpu.decode_stream(ctxs[0], ws[i % 4], n + 64, frames=fr[0], result=rs[0], stream=sts[0])
            else:
                step(i)
        torch.cuda.synchronize()
        print(mode, round((time.perf_counter() - t0) / reps * 1e3, 4), "ms per batch")
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
