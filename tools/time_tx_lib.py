#!/usr/bin/env python3
"""TX encode (C2 shape, 65 536 x 4 KiB client frames) timed in one process, for
A/B of library builds (FWS_LIB_VARIANT): ms per call over 200 back-to-back
calls after >= 60 ms of warm-up, with source payloads at offset 0 (16-B
aligned) and at offset 3 (byte-misaligned), plus a checksum of the output.

usage: [FWS_LIB_VARIANT=tag] python tools/time_tx_lib.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import run_tx  # noqa: E402
from flashws_amd import gpu  # noqa: E402


def main():
    ctx, outs, srcs, dd, n, total = run_tx.setup()
    src = srcs[0]   # (r06: setup returns 4 rotating copies; this tool times one)
    out = {"lib": os.environ.get("FWS_LIB_VARIANT", "default")}
    for shift in (0, 3):
        d = dd.view(n, -1).clone()
        if shift:   # src_off += shift (first 8 bytes of each descriptor, little-endian u64)
            d[:, 0] += shift
        s = src if not shift else torch.cat([src, torch.zeros(16, dtype=torch.uint8, device=src.device)])
        d = d.reshape(-1)
        fn = lambda i: gpu.encode_frames(ctx, outs[i % 4], s, d, n)
        t0 = time.perf_counter()
        i = 0
        while time.perf_counter() - t0 < 0.06 or i < 20:
            fn(i); i += 1
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(200):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        fn(0); torch.cuda.synchronize()
        out[f"ms_shift{shift}"] = round(e0.elapsed_time(e1) / 200, 4)
        out[f"sum_shift{shift}"] = int(outs[0][:total].to(torch.int64).sum())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
