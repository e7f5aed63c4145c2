#!/usr/bin/env python3
"""Grid-cap sweep of the C5 descriptor-mode kernels (262 144 x 16 KiB TEXT
frames, 4 GiB): k_unmask_sorted and k_unmask_sorted_utf8 + k_utf8_seam_sorted
(HIP events; runs come in pairs, so the bytes are masked again after each
pair), and with --stream the C5 stream decode (fws_gpu_decode_stream + UTF-8
flags). Cap 0 = the library's per-kernel defaults.
usage: python tools/tune_c5.py [--lib PATH] [--caps 0,16384,65536] [--stream]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib  # noqa: E402
if "--lib" in sys.argv:
    _lib.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
from flashws_amd import gpu, lib  # noqa: E402


def main():
    caps = [0, 16384, 65536, 262144]
    if "--caps" in sys.argv:
        caps = [int(c) for c in sys.argv[sys.argv.index("--caps") + 1].split(",")]
    dev = torch.device("cuda:0")
    w5, d5, _ = gpu.config_c5()
    n = len(d5)
    payload = int(d5["payload_len"].sum())
    ctx = gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(w5))
    w = torch.from_numpy(w5).to(dev)
    del w5
    dd = gpu.descs_to_device(d5, dev)
    ok = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
    fr = torch.empty((n + 64) * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev)
    res = torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev)
    out = {"lib": os.path.basename(_lib.LIB_PATH)}
    for cap in caps:
        lib().fws_internal_set_grid_cap(cap)
        kernels = [("plain", lambda: gpu.unmask_sorted(ctx, w, dd, n)),
                   ("utf8", lambda: gpu.unmask_sorted_utf8(ctx, w, dd, n, ok))]
        if "--stream" in sys.argv:
            kernels.append(("stream", lambda: gpu.decode_stream(ctx, w, n + 64, frames=fr, result=res, utf8_ok=ok)))
        for name, fn in kernels:
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 8
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            out[f"{name}_grid{cap}"] = {"ms": round(ms, 4), "alg_TB_per_s": round(2 * payload / ms / 1e9, 3)}
            print(name, cap, out[f"{name}_grid{cap}"], flush=True)
    lib().fws_internal_set_grid_cap(0)
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
