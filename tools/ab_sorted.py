#!/usr/bin/env python3
"""Interleaved A/B of fws_gpu_unmask_sorted's kernels on the C2 batch (4
rotating buffers, HIP events around back-to-back calls): every round times
each variant once, so box drift hits all of them alike. Prints one JSON line
per variant with the median / min per-launch time and the HBM fraction.
usage: python tools/ab_sorted.py [rounds] [steps] [variants, comma-separated]
  variant 0 = k_unmask_sorted (lookup first), 1 = _early, 3 = XCD-run order"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib, gpu  # noqa: E402

ALG = 537_395_200


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    variants = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 3]
    L = _lib.lib()
    dev = torch.device("cuda:0")
    wire, descs, _ = gpu.config_c2()
    n = len(descs)
    ctx = gpu.Ctx(0, max_frames=n, max_stream_bytes=len(wire))
    bufs = [torch.from_numpy(wire).to(dev) for _ in range(4)]
    dd = gpu.descs_to_device(descs, dev)
    times = {v: [] for v in variants}
    old = L.fws_internal_set_sorted_early(0)
    for r in range(rounds):
        for v in (variants if r % 2 == 0 else variants[::-1]):
            L.fws_internal_set_sorted_early(v)
            for i in range(20):
                gpu.unmask_sorted(ctx, bufs[i % 4], dd, n)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for i in range(steps):
                gpu.unmask_sorted(ctx, bufs[i % 4], dd, n)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) * 1e3 / steps)
        print(json.dumps({"round": r, **{str(v): round(times[v][-1], 2) for v in variants}}), flush=True)
    L.fws_internal_set_sorted_early(old)
    for v in variants:
        med = statistics.median(times[v])
        print(json.dumps({"variant": v, "us_median": round(med, 2), "us_min": round(min(times[v]), 2),
                          "frac_median": round(ALG / med / 8e6, 4), "runs": [round(t, 2) for t in times[v]]}))
    ctx.close()


if __name__ == "__main__":
    main()
