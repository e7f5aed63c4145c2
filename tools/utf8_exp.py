#!/usr/bin/env python3
"""C5 descriptor-mode fused unmask + UTF-8 (fws_gpu_unmask_sorted_utf8) timed
through a variant library (tools/build_variant.sh); the flags of the first run
are checked against the generator's.

usage: python tools/utf8_exp.py flashws_amd/lib/libfws_gpu_<tag>.so [kernel variant] [reps]
(kernel variant: fws_internal_set_sorted_utf8_pipe's argument, default 0)"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flashws_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, sys.argv[1])
from flashws_amd import gpu  # noqa: E402


def main():
    variant = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    _lib.lib().fws_internal_set_sorted_utf8_pipe(variant)
    dev = torch.device("cuda:0")
    w5, d5, ok5 = gpu.config_c5()
    n = len(d5)
    payload = int(d5["payload_len"].sum())
    ctx = gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(w5))
    w = torch.from_numpy(w5).to(dev)
    del w5
    dd = gpu.descs_to_device(d5, dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    gpu.unmask_sorted_utf8(ctx, w, dd, n, ok)
    torch.cuda.synchronize()
    good = bool(np.array_equal(ok.cpu().numpy(), np.asarray(ok5, dtype=np.uint8)[:n]))
    s = torch.cuda.current_stream()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(reps):
        e[0].record(s)
        gpu.unmask_sorted_utf8(ctx, w, dd, n, ok)
        e[1].record(s)
        torch.cuda.synchronize()
        ts.append(e[0].elapsed_time(e[1]))
    t = float(np.median(ts))
    tp = []
    for _ in range(reps):                             # the plain unmask of the same batch, for reference
        e[0].record(s)
        gpu.unmask_sorted(ctx, w, dd, n)
        e[1].record(s)
        torch.cuda.synchronize()
        tp.append(e[0].elapsed_time(e[1]))
    print(json.dumps({"lib": os.path.basename(sys.argv[1]), "variant": variant, "flags_ok": good, "ms": round(t, 4),
                      "GiB_per_s": round(payload / (t / 1e3) / 2**30, 1),
                      "plain_unmask_ms": round(float(np.median(tp)), 4)}))
    ctx.close()


if __name__ == "__main__":
    main()
