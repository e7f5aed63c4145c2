#!/usr/bin/env python3
"""Does the 256 MB Infinity Cache (MALL) serve part of C4's and TX's source?
Both benches re-read ONE 256 MiB source every step (4 rotating destinations),
while every other config rotates >= 1 GiB of inputs. Interleaved A/B, one
process: the same step with 1 source against 4 rotating sources (each a copy
of the same bytes), HIP events around back-to-back calls.
usage: python tools/ab_mall.py [rounds] [steps]"""
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu  # noqa: E402


def timed(fn, steps):
    for i in range(8):
        fn(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for i in range(steps):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / steps


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    dev = torch.device("cuda:0")
    # C4
    w4, d4, _ = gpu.config_c4()
    c = gpu.Ctx(0, max_frames=len(d4) + 8, max_stream_bytes=len(w4))
    srcs = [torch.from_numpy(w4).to(dev) for _ in range(4)]
    total = int(d4["payload_len"].sum())
    dsts = [torch.empty(total + 64, dtype=torch.uint8, device=dev) for _ in range(4)]
    dd4 = gpu.descs_to_device(d4, dev)
    alg4 = len(w4) + total
    # TX (bench.py tx_extra's shape)
    n, pl = 65536, 4096
    rng = np.random.default_rng(7)
    txd = np.zeros(n, dtype=gpu.TX_DESC)
    txd["src_off"] = np.arange(n, dtype=np.uint64) * pl
    txd["len"] = pl
    txd["key"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    txd["opcode"] = 2
    txd["fin"] = 1
    txd["masked"] = 1
    payload = rng.integers(0, 256, n * pl, dtype=np.uint8)
    tsrcs = [torch.from_numpy(payload).to(dev) for _ in range(4)]
    tdd = torch.from_numpy(txd.view(np.uint8).copy()).to(dev)
    tx_total = n * (pl + 8)
    ct = gpu.Ctx(0, max_frames=n, max_stream_bytes=tx_total)
    touts = [torch.empty(tx_total, dtype=torch.uint8, device=dev) for _ in range(4)]
    algt = n * pl + tx_total
    forms = {
        "c4_1src": (lambda i: gpu.unmask_gather(c, dsts[i % 4], srcs[0], dd4, len(d4)), alg4),
        "c4_4src": (lambda i: gpu.unmask_gather(c, dsts[i % 4], srcs[i % 4], dd4, len(d4)), alg4),
        "tx_1src": (lambda i: gpu.encode_frames(ct, touts[i % 4], tsrcs[0], tdd, n), algt),
        "tx_4src": (lambda i: gpu.encode_frames(ct, touts[i % 4], tsrcs[i % 4], tdd, n), algt),
    }
    times = {k: [] for k in forms}
    names = list(forms)
    for r in range(rounds):
        for k in (names if r % 2 == 0 else names[::-1]):
            times[k].append(timed(forms[k][0], steps))
        print(json.dumps({"round": r, **{k: round(v[-1], 2) for k, v in times.items()}}), flush=True)
    for k in names:
        med = statistics.median(times[k])
        print(json.dumps({"form": k, "us_median": round(med, 2), "us_min": round(min(times[k]), 2),
                          "frac_median": round(forms[k][1] / med / 8e6, 4),
                          "runs": [round(t, 2) for t in times[k]]}))
    c.close()
    ct.close()


if __name__ == "__main__":
    main()
