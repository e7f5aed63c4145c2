#!/usr/bin/env python3
"""Can the stream decode's two passes share the GPU by CU partition? On C3:
k_scan alone (fws_internal_scan_only) and the whole fws_gpu_decode_stream on
HIP streams restricted to a CU subset (hipExtStreamCreateWithCUMask), for
several splits, then the two co-running: k_scan of one batch on subset X while
another batch decodes on the complement Y. HIP events per stream; one JSON line
per measurement.

usage: python tools/cumask_probe.py [reps]"""
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib, gpu  # noqa: E402

hip = C.CDLL("libamdhip64.so")


def masked_stream(bits):
    words = (C.c_uint32 * 8)()
    for i in range(256):
        if bits(i):
            words[i // 32] |= 1 << (i % 32)
    s = C.c_void_p()
    r = hip.hipExtStreamCreateWithCUMask(C.byref(s), C.c_uint32(8), words)
    if r != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask {r}")
    return s.value


def ev_time(stream, fn, reps):
    e0, e1 = C.c_void_p(), C.c_void_p()
    hip.hipEventCreate(C.byref(e0))
    hip.hipEventCreate(C.byref(e1))
    hip.hipEventRecord(e0, C.c_void_p(stream))
    for i in range(reps):
        fn(i)
    hip.hipEventRecord(e1, C.c_void_p(stream))
    return e0, e1


def elapsed(e0, e1):
    hip.hipEventSynchronize(e1)
    ms = C.c_float()
    hip.hipEventElapsedTime(C.byref(ms), e0, e1)
    return ms.value


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    L = _lib.lib()
    wire, descs, _ = gpu.config_c3()
    dev = torch.device("cuda:0")
    n = len(descs)
    ctxs = [gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(wire)) for _ in range(2)]
    ws = [torch.from_numpy(wire).to(dev) for _ in range(4)]
    fr = [torch.empty((n + 64) * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]
    rs = [torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]
    N = len(wire)

    def scan(ci, st, i):
        r = L.fws_internal_scan_only(ctxs[ci].h, C.c_void_p(ws[(2 * i + ci) % 4].data_ptr()), C.c_uint64(N),
                                     C.c_void_p(st))
        assert r == 0

    wrapped = {}

    def dec(ci, st, i):
        if st not in wrapped:
            wrapped[st] = torch.cuda.ExternalStream(st)
        rc, _, _, _ = gpu.decode_stream(ctxs[ci], ws[(2 * i + ci) % 4], n + 64, frames=fr[ci], result=rs[ci],
                                        stream=wrapped[st])
        assert rc == 0

    splits = {
        "all": (lambda i: True, None),
        "even_odd": (lambda i: i % 2 == 0, lambda i: i % 2 == 1),
        "lo_hi": (lambda i: i < 128, lambda i: i >= 128),
        "mod8_0123": (lambda i: i % 8 < 4, lambda i: i % 8 >= 4),
        "even_odd_5_3": (lambda i: i % 8 < 5, lambda i: i % 8 >= 5),
        "even_odd_3_5": (lambda i: i % 8 < 3, lambda i: i % 8 >= 3),
    }
    for name, (fx, fy) in splits.items():
        sx = masked_stream(fx)
        sy = masked_stream(fy) if fy else None
        for _ in range(2):
            for i in range(3):
                scan(0, sx, i)
                dec(1, sy or sx, i)
            hip.hipDeviceSynchronize()
            out = {"split": name}
            # alone: scan on X, decode on X, decode on Y
            e = ev_time(sx, lambda i: scan(0, sx, i), reps)
            out["scan_X_us"] = round(elapsed(*e) / reps * 1e3, 1)
            e = ev_time(sx, lambda i: dec(0, sx, i), reps)
            out["decode_X_us"] = round(elapsed(*e) / reps * 1e3, 1)
            if sy:
                e = ev_time(sy, lambda i: dec(1, sy, i), reps)
                out["decode_Y_us"] = round(elapsed(*e) / reps * 1e3, 1)
                # co-running: scan loop on X, decode loop on Y, issued interleaved
                hip.hipDeviceSynchronize()
                t0 = time.perf_counter()
                ex0, ex1, ey0, ey1 = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
                for ev in (ex0, ex1, ey0, ey1):
                    hip.hipEventCreate(C.byref(ev))
                hip.hipEventRecord(ex0, C.c_void_p(sx))
                hip.hipEventRecord(ey0, C.c_void_p(sy))
                for i in range(reps):
                    scan(0, sx, i)
                    dec(1, sy, i)
                hip.hipEventRecord(ex1, C.c_void_p(sx))
                hip.hipEventRecord(ey1, C.c_void_p(sy))
                hip.hipDeviceSynchronize()
                wall = (time.perf_counter() - t0) * 1e3
                out["co_scan_X_us"] = round(elapsed(ex0, ex1) / reps * 1e3, 1)
                out["co_decode_Y_us"] = round(elapsed(ey0, ey1) / reps * 1e3, 1)
                out["co_wall_per_pair_us"] = round(wall / reps * 1e3, 1)
            print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
