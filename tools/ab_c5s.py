#!/usr/bin/env python3
"""A/B of the C5 stream decode (fws_gpu_decode_stream + UTF-8 flags on one 4 GiB
C5 batch) with and without the cross-unit prefetch of k_unmask_stream<utf8>
(fws_internal_set_stream_utf8_pf) and, with AB_CAPS=a,b,..., at those caps
on every streaming kernel's grid (fws_internal_set_grid_cap), in one process; every timed call decodes a
freshly masked copy (4 copies rotated, re-masked by a device copy between
repetitions, outside the timed region). One JSON line per (mode, rep)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu  # noqa: E402
from flashws_amd._lib import lib  # noqa: E402


def main(k=4, reps=3):
    dev = torch.device("cuda:0")
    w5, d5, ok5 = gpu.config_c5()
    n = len(d5)
    cap = n + 64
    ctx = gpu.Ctx(0, max_frames=cap, max_stream_bytes=len(w5))
    master = torch.from_numpy(w5).to(dev)
    bufs = [master.clone() for _ in range(k)]
    frames = torch.empty(cap * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev)
    res = torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev)
    ok = torch.zeros(cap, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:                     # warm clocks (re-masked below)
        gpu.decode_stream(ctx, bufs[0], cap, frames=frames, result=res, utf8_ok=ok)
        torch.cuda.synchronize()
    modes = [(1, 0), (0, 0)] + [(1, int(c)) for c in (os.environ.get("AB_CAPS") or "").split(",") if c]
    for rep in range(reps):
        for pf, gcap in (modes if rep % 2 == 0 else modes[::-1]):
            lib().fws_internal_set_stream_utf8_pf(pf)
            lib().fws_internal_set_grid_cap(gcap)       # 0: the library's default grids
            for b in bufs:
                b.copy_(master)
            torch.cuda.synchronize()
            e0.record(s)
            for b in bufs:
                rc, _, _, _ = gpu.decode_stream(ctx, b, cap, frames=frames, result=res, utf8_ok=ok)
                assert rc == 0
            e1.record(s)
            torch.cuda.synchronize()
            r = gpu.read_result(res)
            flags_ok = bool(np.array_equal(ok[:n].cpu().numpy(), np.asarray(ok5, dtype=np.uint8)[:n]))
            lib().fws_internal_set_grid_cap(0)
            print(json.dumps({"pf": pf, "grid_cap": gcap, "rep": rep, "ms": round(e0.elapsed_time(e1) / k, 4),
                              "status": int(r["status"]), "frames_ok": int(r["n_frames"]) == n,
                              "flags_ok": flags_ok}), flush=True)
    lib().fws_internal_set_stream_utf8_pf(1)
    ctx.close()


if __name__ == "__main__":
    main()
