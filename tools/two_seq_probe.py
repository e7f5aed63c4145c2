#!/usr/bin/env python3
"""Why do two C3 decodes overlap in tools/stream_pair_probe.py but not in
bench.py's two_in_flight record? Replays bench's sequence (context A used for
50 single-stream calls on the current stream, then context B created, then the
pair on two non-blocking HIP streams) beside fresh contexts, and variants in
between. Prints us per batch.

usage: python tools/two_seq_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu  # noqa: E402


def pair_time(ctxs, ws, fr, rs, n, sts, reps=30):
    for i in range(4):
        gpu.decode_stream(ctxs[i % 2], ws[i % 4], n + 64, frames=fr[i % 2], result=rs[i % 2], stream=sts[i % 2])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        rc, _, _, _ = gpu.decode_stream(ctxs[i % 2], ws[i % 4], n + 64, frames=fr[i % 2], result=rs[i % 2],
                                        stream=sts[i % 2])
        assert rc == 0
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    wire, descs, _ = gpu.config_c3()
    n = len(descs)
    dev = torch.device("cuda:0")
    ws = [torch.from_numpy(wire).to(dev) for _ in range(4)]
    fr = [torch.empty((n + 64) * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]
    rs = [torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]
    for trial in range(2):
        # bench's order: A single-stream first (current stream), then B
        a = gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(wire))
        for i in range(50):
            gpu.decode_stream(a, ws[i % 4], n + 64, frames=fr[0], result=rs[0])
        torch.cuda.synchronize()
        b = gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(wire))
        t_bench = pair_time([a, b], ws, fr, rs, n, [gpu.hip_stream(), gpu.hip_stream()])
        # same contexts, A's single-stream calls on a HIP stream instead
        a2 = gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(wire))
        s0 = gpu.hip_stream()
        for i in range(50):
            gpu.decode_stream(a2, ws[i % 4], n + 64, frames=fr[0], result=rs[0], stream=s0)
        torch.cuda.synchronize()
        b2 = gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(wire))
        t_hip = pair_time([a2, b2], ws, fr, rs, n, [s0, gpu.hip_stream()])
        # fresh pair
        c = [gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(wire)) for _ in range(2)]
        t_fresh = pair_time(c, ws, fr, rs, n, [gpu.hip_stream(), gpu.hip_stream()])
        # fresh pair, reversed roles
        t_rev = pair_time([b, a], ws, fr, rs, n, [gpu.hip_stream(), gpu.hip_stream()])
        print(f"trial {trial}: bench order {t_bench:6.1f}  A on HIP stream first {t_hip:6.1f}  fresh {t_fresh:6.1f}  "
              f"bench pair reversed {t_rev:6.1f} us/batch", flush=True)
        for x in (a, b, a2, b2, *c):
            x.close()


if __name__ == "__main__":
    main()
