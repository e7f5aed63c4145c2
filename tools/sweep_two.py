#!/usr/bin/env python3
"""Stream decode with one batch vs two batches in flight (two contexts on two
streams, batches alternate) across the co-residency knobs of the streaming
kernels: k_scan workgroups per CU (fws_internal_set_scan_blocks_per_cu, read
when a context first sizes its workspace) and the unmask grid cap
(fws_internal_set_grid_cap). Prints ms per batch.

usage: python tools/sweep_two.py [c3|c2] [reps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib, gpu  # noqa: E402


def run(wire, n, dev, reps, bpc, cap):
    L = _lib.lib()
    L.fws_internal_set_scan_blocks_per_cu(bpc)
    old_cap = L.fws_internal_set_grid_cap(cap)
    ctxs = [gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(wire)) for _ in range(2)]
    src = torch.from_numpy(wire).to(dev)
    ws = [src.clone() for _ in range(4)]
    sts = [gpu.hip_stream(), gpu.hip_stream()]
    fr = [torch.empty((n + 64) * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]
    rs = [torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]

    def step(i, two):
        c = i % 2 if two else 0
        rc, _, _, _ = gpu.decode_stream(ctxs[c], ws[i % 4], n + 64, frames=fr[c], result=rs[c], stream=sts[c])
        assert rc == 0
    for i in range(4):
        step(i, True)
    torch.cuda.synchronize()
    out = {}
    for two in (False, True):
        best = 1e9
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(reps):
                step(i, two)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / reps * 1e3)
        out[two] = best
    r = gpu.read_result(rs[0])
    assert int(r["status"]) == 0 and int(r["n_frames"]) == n, r
    for c in ctxs:
        c.close()
    L.fws_internal_set_grid_cap(old_cap)
    L.fws_internal_set_scan_blocks_per_cu(0)
    return out


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "c3"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    wire, descs, _ = {"c3": gpu.config_c3, "c2": gpu.config_c2}[which]()
    dev = torch.device("cuda:0")
    n = len(descs)
    pay = int(descs["payload_len"].sum())
    for bpc in (8, 6, 4, 3, 2):
        for cap in (16384, 2048, 1024, 512):
            o = run(wire, n, dev, reps, bpc, cap)
            alg = (len(wire) + pay) / 1e9
            print(f"{which} scan_bpc={bpc} grid_cap={cap:5d}: one {o[False]*1e3:7.1f} us  two-in-flight "
                  f"{o[True]*1e3:7.1f} us/batch ({alg / (o[True] * 1e-3) / 8000 * 100:4.1f}% of 8 TB/s)",
                  flush=True)


if __name__ == "__main__":
    main()
