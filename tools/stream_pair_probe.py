#!/usr/bin/env python3
"""Does the way two streams are created decide whether two C3 decodes overlap?
(tools/two_c3_repeat.py saw 177 or 205 us per batch from one run to the next.)
Each variant creates a fresh pair of streams 5 times and times 30 alternating
batches on it: torch pool streams; a high-priority + a default one; raw
hipStreamCreateWithFlags(non-blocking) streams wrapped as external streams.

usage: python tools/stream_pair_probe.py"""
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu  # noqa: E402

hip = C.CDLL("libamdhip64.so")


def raw_stream():
    s = C.c_void_p()
    assert hip.hipStreamCreateWithFlags(C.byref(s), C.c_uint(1)) == 0
    return torch.cuda.ExternalStream(s.value)


def main():
    wire, descs, _ = gpu.config_c3()
    n = len(descs)
    dev = torch.device("cuda:0")
    ctxs = [gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(wire)) for _ in range(2)]
    src = torch.from_numpy(wire).to(dev)
    ws = [src.clone() for _ in range(4)]
    fr = [torch.empty((n + 64) * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]
    rs = [torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]
    variants = {
        "torch pool": lambda: [torch.cuda.Stream(), torch.cuda.Stream()],
        "prio high+default": lambda: [torch.cuda.Stream(priority=-1), torch.cuda.Stream()],
        "raw non-blocking": lambda: [raw_stream(), raw_stream()],
    }
    for name, mk in variants.items():
        out = []
        for _ in range(5):
            sts = mk()
            for i in range(4):
                gpu.decode_stream(ctxs[i % 2], ws[i % 4], n + 64, frames=fr[i % 2], result=rs[i % 2],
                                  stream=sts[i % 2])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(30):
                rc, _, _, _ = gpu.decode_stream(ctxs[i % 2], ws[i % 4], n + 64, frames=fr[i % 2],
                                                result=rs[i % 2], stream=sts[i % 2])
                assert rc == 0
            torch.cuda.synchronize()
            out.append((time.perf_counter() - t0) / 30 * 1e6)
        print(f"{name:18s}: " + " ".join(f"{x:6.1f}" for x in out) + " us/batch", flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
