#!/usr/bin/env python3
"""BASELINE C5 per-GPU share (262 144 x 16 KiB TEXT frames, 4 GiB) in
descriptor mode: fws_gpu_unmask_sorted + fws_gpu_validate_utf8 (frame
offsets known, as a batch split at frame boundaries has them). Checks the
flags against the generator's, then times the pair with HIP events."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu  # noqa: E402


def main(reps=6):
    dev = torch.device("cuda:0")
    w5, d5, ok5 = gpu.config_c5()
    n = len(d5)
    payload = int(d5["payload_len"].sum())
    ctx = gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(w5))
    w = torch.from_numpy(w5).to(dev)
    del w5
    dd = gpu.descs_to_device(d5, dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    gpu.unmask_sorted(ctx, w, dd, n)
    gpu.validate_utf8(ctx, w, dd, n, ok)
    torch.cuda.synchronize()
    got = ok.cpu().numpy()
    assert np.array_equal(got, np.asarray(ok5, dtype=np.uint8)[:n]), "utf8 flags differ"
    s = torch.cuda.current_stream()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tu = tv = 0.0
    for _ in range(reps):
        e[0].record(s)
        gpu.unmask_sorted(ctx, w, dd, n)
        e[1].record(s)
        gpu.validate_utf8(ctx, w, dd, n, ok)
        e[2].record(s)
        torch.cuda.synchronize()
        tu += e[0].elapsed_time(e[1]) / reps
        tv += e[1].elapsed_time(e[2]) / reps
    t = tu + tv
    # fused: one pass (k_unmask_sorted_utf8 + k_utf8_seam_sorted)
    w.copy_(torch.from_numpy(gpu.config_c5()[0]).to(dev))
    gpu.unmask_sorted_utf8(ctx, w, dd, n, ok)
    torch.cuda.synchronize()
    assert np.array_equal(ok.cpu().numpy(), np.asarray(ok5, dtype=np.uint8)[:n]), "fused utf8 flags differ"
    from flashws_amd import lib
    for pipe in (1, 0, 2):
        old = lib().fws_internal_set_sorted_utf8_pipe(pipe)
        tf = 0.0
        for _ in range(reps):
            e[0].record(s)
            gpu.unmask_sorted_utf8(ctx, w, dd, n, ok)
            e[1].record(s)
            torch.cuda.synchronize()
            tf += e[0].elapsed_time(e[1]) / reps
        lib().fws_internal_set_sorted_utf8_pipe(old)
        print(json.dumps({"C5_descriptor_fused": {"form": pipe,
                                                  "GiB_per_s": round(payload / (tf / 1e3) / 2**30, 1),
                                                  "ms_per_step": round(tf, 4)}}))
    print(json.dumps({"C5_descriptor_unmask_utf8": {"GiB_per_s": round(payload / (t / 1e3) / 2**30, 1),
                                                    "ms_per_step": round(t, 4), "unmask_ms": round(tu, 4),
                                                    "validate_ms": round(tv, 4), "frames": n,
                                                    "invalid_frames": int((got == 0).sum())}}))
    ctx.close()


if __name__ == "__main__":
    main()
