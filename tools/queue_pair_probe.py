#!/usr/bin/env python3
"""Are two streams that serialize two decodes the ones sharing a hardware
queue? Creates 8 non-blocking HIP streams in a row and times two alternating
C3 decodes on (s0, s_k) for k = 1..7 (GPU_MAX_HW_QUEUES is 4 on the box, HIP's
default: with round-robin assignment s0 and s4 would share one).

usage: python tools/queue_pair_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu  # noqa: E402


def main():
    wire, descs, _ = gpu.config_c3()
    n = len(descs)
    dev = torch.device("cuda:0")
    ws = [torch.from_numpy(wire).to(dev) for _ in range(4)]
    fr = [torch.empty((n + 64) * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]
    rs = [torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]
    ctxs = [gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(wire)) for _ in range(2)]
    print("GPU_MAX_HW_QUEUES =", os.environ.get("GPU_MAX_HW_QUEUES"), flush=True)
    for trial in range(2):
        st = [gpu.hip_stream() for _ in range(8)]
        row = []
        for k in range(1, 8):
            sts = [st[0], st[k]]
            for i in range(4):
                gpu.decode_stream(ctxs[i % 2], ws[i % 4], n + 64, frames=fr[i % 2], result=rs[i % 2], stream=sts[i % 2])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(30):
                gpu.decode_stream(ctxs[i % 2], ws[i % 4], n + 64, frames=fr[i % 2], result=rs[i % 2], stream=sts[i % 2])
            torch.cuda.synchronize()
            row.append((time.perf_counter() - t0) / 30 * 1e6)
        print(f"trial {trial}: (s0, s1..s7) " + " ".join(f"{x:6.1f}" for x in row) + " us/batch", flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
