#!/usr/bin/env python3
"""A/B of fws_gpu_unmask_batch's two forms: one launch per region wavefront
(k_unmask_any + k_unmask_pieces, fws_internal_set_unmask_any 1) against
k_plan + k_unmask_desc (0), on C2 (65 536 x 4 KiB, sorted and permuted), C3
(mixed 64 B-64 KiB) and C4 (1 427 regions of 4 KiB-1 MiB, permuted), in place
on 4 rotating buffers; HIP events over back-to-back calls, modes alternated;
one call of each mode on a fresh copy compared byte for byte first.

usage: python tools/ab_batch.py [reps]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib, gpu  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    L = _lib.lib()
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(5)
    cfgs = []
    w2, d2, _ = gpu.config_c2()
    cfgs += [("C2_sorted", w2, d2), ("C2_permuted", w2, d2[rng.permutation(len(d2))])]
    w3, d3, _ = gpu.config_c3()
    cfgs.append(("C3_sorted", w3, d3))
    w4, d4, _ = gpu.config_c4()
    cfgs.append(("C4_in_place", w4, d4))
    for name, wire, descs in cfgs:
        n = len(descs)
        c = gpu.Ctx(0, max_frames=n + 8, max_stream_bytes=len(wire))
        dd = gpu.descs_to_device(descs, dev)
        outs = []
        for mode in (1, 0):
            L.fws_internal_set_unmask_any(mode)
            b = torch.from_numpy(wire).to(dev)
            gpu.unmask_batch(c, b, dd, n)
            torch.cuda.synchronize()
            outs.append(b.cpu())
        same = bool(torch.equal(outs[0], outs[1]))
        bufs = [torch.from_numpy(wire).to(dev) for _ in range(4)]
        for rep in range(3):
            for mode in (1, 0):
                L.fws_internal_set_unmask_any(mode)
                for i in range(8):
                    gpu.unmask_batch(c, bufs[i % 4], dd, n)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(reps):
                    gpu.unmask_batch(c, bufs[i % 4], dd, n)
                e1.record()
                torch.cuda.synchronize()
                print(json.dumps({"cfg": name, "regions": n, "any": mode, "rep": rep,
                                  "ms": round(e0.elapsed_time(e1) / reps, 4), "same_output": same}), flush=True)
        L.fws_internal_set_unmask_any(1)
        c.close()
        del bufs


if __name__ == "__main__":
    main()
