#!/usr/bin/env python3
"""A/B timing of the C5 descriptor-mode passes on one 4 GiB C5 batch, in one
process (the library variant from FWS_LIB_VARIANT): the plain unmask
(k_unmask_sorted, the HBM floor of the pass), fws_gpu_unmask_sorted_utf8 in
its plain form (pipe 0), the software-pipelined form (pipe 1) and the
early-load form (pipe 2, the default: the unit's loads before the owner
lookup). HIP events, 20 calls
per repetition after a warm-up of >= 0.5 s; prints one JSON line per mode."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu  # noqa: E402
from flashws_amd._lib import lib  # noqa: E402


def main(calls=20, reps=3):
    dev = torch.device("cuda:0")
    w5, d5, ok5 = gpu.config_c5()
    n = len(d5)
    ctx = gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(w5))
    w = torch.from_numpy(w5).to(dev)
    dd = gpu.descs_to_device(d5, dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    def utf8(pipe, cap=0):
        def f():
            lib().fws_internal_set_sorted_utf8_pipe(pipe)
            lib().fws_internal_set_grid_cap(cap)          # 0: the library's default grid
            gpu.unmask_sorted_utf8(ctx, w, dd, n, ok)
            lib().fws_internal_set_grid_cap(0)
        return f
    modes = {"plain_unmask": lambda: gpu.unmask_sorted(ctx, w, dd, n),
             "utf8_pipe0": utf8(0), "utf8_pipe2": utf8(2)}
    for cap in (os.environ.get("AB_CAPS") or "").split(","):
        if cap:
            modes[f"utf8_pipe0_cap{cap}"] = utf8(0, int(cap))
            modes[f"utf8_pipe2_cap{cap}"] = utf8(2, int(cap))
    for name in list(modes) + list(modes)[::-1]:
        fn = modes[name]
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.5:
            for _ in range(4):
                fn()
            torch.cuda.synchronize()
        ms = []
        for _ in range(reps):
            e0.record(s)
            for _ in range(calls):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            ms.append(round(e0.elapsed_time(e1) / calls, 4))
        print(json.dumps({"variant": os.environ.get("FWS_LIB_VARIANT", "") or "product", "mode": name,
                          "ms": sorted(ms)[len(ms) // 2], "reps": ms}), flush=True)
    lib().fws_internal_set_sorted_utf8_pipe(2)
    # correctness of the product setting on the masked batch
    w.copy_(torch.from_numpy(w5).to(dev))
    gpu.unmask_sorted_utf8(ctx, w, dd, n, ok)
    torch.cuda.synchronize()
    if not os.environ.get("FWS_LIB_VARIANT", "").startswith("abl"):      # ablation builds skip work
        assert np.array_equal(ok.cpu().numpy(), np.asarray(ok5, dtype=np.uint8)[:n]), "utf8 flags differ"
    ctx.close()


if __name__ == "__main__":
    main()
