#!/usr/bin/env python3
"""Interleaved A/B of k_gather_one forms on BASELINE C4 (one 256 MiB message in
1 427 fragments, 4 rotating destinations, HIP events around back-to-back
fws_gpu_unmask_gather calls): 0 = two loads per chunk (r05), 1 = one
nontemporal load per chunk + the neighbour lane's block by DPP, 2 =
k_gather_one_w8 (8 waves per SIMD), 3 = 2 with 1's loads
(fws_internal_set_gather_dpp), at 512 or 256 threads per workgroup; -1 =
the plan launch + k_gather_fast<kFlat> (one wave per unit, fws_internal_set_gather_one(0));
-2 = the same with k_gather_fast's two-load form (fws_internal_set_gather_flat(0)). Every
round times each form once. The source rotates over 4 copies (1 GiB, past the
256 MB Infinity Cache) unless FWS_AB_ONE_SRC=1.
usage: python tools/ab_c4.py [rounds] [steps] [dpp:threads:mult,...]"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib, gpu  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    L = _lib.lib()
    dev = torch.device("cuda:0")
    w4, d4, _ = gpu.config_c4()
    c = gpu.Ctx(0, max_frames=len(d4) + 8, max_stream_bytes=len(w4))
    srcs = [torch.from_numpy(w4).to(dev) for _ in range(1 if os.environ.get("FWS_AB_ONE_SRC") == "1" else 4)]
    total = int(d4["payload_len"].sum())
    alg = len(w4) + total
    dsts = [torch.empty(total + 64, dtype=torch.uint8, device=dev) for _ in range(4)]
    dd = gpu.descs_to_device(d4, dev)
    forms = [tuple(int(x) for x in f.split(":")) for f in sys.argv[3].split(",")] if len(sys.argv) > 3 else \
        [(2, 512, 4), (3, 512, 4), (1, 512, 4), (3, 256, 4)]
    times = {f: [] for f in forms}
    for r in range(rounds):
        for f in (forms if r % 2 == 0 else forms[::-1]):
            L.fws_internal_set_gather_one(0 if f[0] < 0 else 1)   # dpp -1: plan launch + k_gather_fast
            L.fws_internal_set_gather_flat(0 if f[0] == -2 else 1)   # -2: its r05 two-load form
            L.fws_internal_set_gather_dpp(max(f[0], 0))
            L.fws_internal_set_gather_shape(f[1], f[2])
            for i in range(10):
                gpu.unmask_gather(c, dsts[i % 4], srcs[i % len(srcs)], dd, len(d4))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for i in range(steps):
                gpu.unmask_gather(c, dsts[i % 4], srcs[i % len(srcs)], dd, len(d4))
            e1.record()
            torch.cuda.synchronize()
            times[f].append(e0.elapsed_time(e1) * 1e3 / steps)
    L.fws_internal_set_gather_one(0)                   # the library default (plan + k_gather_fast)
    L.fws_internal_set_gather_flat(1)
    L.fws_internal_set_gather_dpp(2)
    L.fws_internal_set_gather_shape(0, 0)
    for f in forms:
        med = statistics.median(times[f])
        print(json.dumps({"dpp": f[0], "threads": f[1], "mult": f[2], "us_median": round(med, 2), "us_min": round(min(times[f]), 2),
                          "frac_median": round(alg / med / 8e6, 4), "runs": [round(t, 2) for t in times[f]]}))
    c.close()


if __name__ == "__main__":
    main()
