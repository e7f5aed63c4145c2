#!/usr/bin/env python3
"""A/B of fws_gpu_decode_stream with the one-pass decode (k_fused) on and off,
per BASELINE-shaped stream (C2 stream, C3, the 200 000 x 64 B workload): mean
ms per call over 4 rotating device copies, and the k_fused counters of the
last call (finished / failed / timeouts).

usage: python tools/run_fused_ab.py [reps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib, gpu  # noqa: E402


def counters(ctx):
    import ctypes as C
    out = (C.c_uint32 * 32)()
    assert _lib.lib().fws_internal_decode_counters(ctx.h, out, 32) == 0
    return list(out)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    L = _lib.lib()
    dev = torch.device("cuda:0")
    cfgs = {"c2": gpu.config_c2, "c3": gpu.config_c3,
            "dense64": lambda: gpu.config_c2(n_frames=200_000, payload=64)}
    for name, mk in cfgs.items():
        wire, descs, _ = mk()
        ctx = gpu.Ctx(0, max_frames=len(descs) + 64, max_stream_bytes=len(wire))
        src = torch.from_numpy(wire).to(dev)
        ws = [src.clone() for _ in range(4)]
        cap = len(descs) + 64
        fr = torch.empty(cap * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev)
        rs = torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev)
        for mode in (1, 0, 1):
            L.fws_internal_set_fused(mode)
            for i in range(4):
                ws[i].copy_(src)
            for i in range(4):   # warm-up (allocations)
                rc, _, res, _ = gpu.decode_stream(ctx, ws[i], cap=len(descs) + 64)
                assert rc == 0
            torch.cuda.synchronize()
            r = gpu.read_result(res)
            assert int(r["status"]) == 0 and int(r["n_frames"]) == len(descs), r
            c = counters(ctx)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(reps):
                gpu.decode_stream(ctx, ws[i % 4], cap=cap, frames=fr, result=rs)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            gib = (int(descs["payload_len"].sum()) / 2**30) / (ms / 1e3)
            alg = (len(wire) + int(descs["payload_len"].sum())) / (ms / 1e3) / 1e9
            print(f"{name:8s} fused={mode} {ms*1e3:8.1f} us  {gib:7.1f} GiB/s payload  {alg:7.1f} GB/s alg "
                  f"({alg/8000*100:4.1f}% of 8 TB/s)  fmode={c[13]} ffail={c[14]:#x} ftimeout={c[17]:#x} "
                  f"surv={int(r['n_survivors'])}", flush=True)
        ctx.close()
        time.sleep(0.1)
    L.fws_internal_set_fused(1)


if __name__ == "__main__":
    main()
