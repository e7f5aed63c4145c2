#!/usr/bin/env python3
"""Phase clocks of the one-pass decode (k_fused, fused_kernels.hip) per super
tile: L (scan + in-ST resolve), F (frontier wait + fast table), B (look-back),
U (frames + unmask), look-back window and spins; start-time spread by ticket.

usage: python tools/prof_fused.py [c2|c3|dense64] [calls]"""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib, gpu  # noqa: E402

W = 12


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "c2"
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    L = _lib.lib()
    L.fws_internal_fused_trace_read.restype = C.c_longlong
    mk = {"c2": gpu.config_c2, "c3": gpu.config_c3,
          "dense64": lambda: gpu.config_c2(n_frames=200_000, payload=64)}[which]
    wire, descs, _ = mk()
    dev = torch.device("cuda:0")
    ctx = gpu.Ctx(0, max_frames=len(descs) + 64, max_stream_bytes=len(wire))
    src = torch.from_numpy(wire).to(dev)
    buf = src.clone()
    cap = len(descs) + 64
    L.fws_internal_set_fused(1)
    L.fws_internal_fused_trace(1)
    for c in range(calls):
        buf.copy_(src)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc, _, res, _ = gpu.decode_stream(ctx, buf, cap=cap)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        r = gpu.read_result(res)
        cn = (C.c_uint32 * 32)()
        L.fws_internal_decode_counters(ctx.h, cn, 32)
        print(f"call {c}: rc={rc} status={int(r['status'])} n_frames={int(r['n_frames'])}/{len(descs)} "
              f"host {dt*1e6:.0f} us  fmode={cn[13]} ffail=~{(~cn[14]) & 0xffffffff if cn[14] else -1} "
              f"ftimeout={cn[17]:#x} big={cn[12]}", flush=True)
    n_st = (len(wire) + 32767) // 32768
    out = np.zeros(n_st * W, dtype=np.uint64)
    got = L.fws_internal_fused_trace_read(out.ctypes.data_as(C.POINTER(C.c_uint64)), n_st)
    L.fws_internal_fused_trace(0)
    t = out.reshape(-1, W)[:got].astype(np.int64)
    ok = t[:, 4] > 0
    print(f"STs {got}, finished {int(ok.sum())}")
    t = t[ok]
    if len(t) == 0:
        ctx.close()
        return
    t0 = t[:, 0].min()
    us = lambda x: x / 100.0   # wall clock 100 MHz
    ph = {"load": t[:, 8] - t[:, 0], "scan": t[:, 9] - t[:, 8], "res": t[:, 10] - t[:, 9],
          "pub": t[:, 1] - t[:, 10], "F": t[:, 2] - t[:, 1], "B": t[:, 3] - t[:, 2], "U": t[:, 4] - t[:, 3],
          "all": t[:, 4] - t[:, 0]}
    for k, v in ph.items():
        print(f"  {k:4s} us: mean {us(v.mean()):8.2f} p50 {us(np.median(v)):8.2f} p90 {us(np.percentile(v, 90)):8.2f} "
              f"max {us(v.max()):8.2f}")
    print(f"  span {us(t[:, 4].max() - t0):.1f} us; start of ST k (us) at k = 0, n/4, n/2, 3n/4, n-1: " +
          ", ".join(f"{us(t[min(int(f * (len(t) - 1)), len(t) - 1), 0] - t0):.1f}" for f in (0, .25, .5, .75, 1)))
    for name, col in (("window", 5), ("lb spins", 6), ("fr spins", 7)):
        v = t[:, col]
        print(f"  {name:9s}: mean {v.mean():8.1f} p50 {np.median(v):6.0f} p90 {np.percentile(v, 90):6.0f} max {v.max()}")
    ctx.close()


if __name__ == "__main__":
    main()
