#!/usr/bin/env python3
"""Phase clocks of the decode scan (k_scan) from the FWS_SCAN_PROF build
(make -C flashws_amd/csrc prof -> flashws_amd/lib/libfws_gpu_prof.so).

Prints average shader clocks per block for each phase, candidate and survivor
counts, and pointer-jumping rounds, for the C2 and C3 streams."""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flashws_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "flashws_amd", "lib", "libfws_gpu_prof.so")
from flashws_amd import gpu  # noqa: E402

PHASES = ["load", "cand+scan", "pos+first_hop", "live+jump+records"]


def main():
    dev = torch.device("cuda:0")
    L = _lib.lib()
    prof = L.fws_internal_scan_prof
    prof.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    prof.restype = C.c_int
    out = {}
    for name, mk in (("C2", gpu.config_c2), ("C3", gpu.config_c3),
                     ("C5_256M", lambda: gpu.config_c5(n_frames=16384))):
        wire, descs, _ = mk()
        n = len(descs)
        ctx = gpu.Ctx(0, max_frames=n + 16, max_stream_bytes=len(wire))
        w = torch.from_numpy(wire).to(dev)
        tiles = (len(wire) + 2047) // 2048
        reps = 5
        for _ in range(2):
            gpu.decode_stream(ctx, w.clone(), cap=n + 16)
        torch.cuda.synchronize()
        arr = (C.c_ulonglong * 16)()
        prof(arr, 1)
        for _ in range(reps):
            gpu.decode_stream(ctx, w.clone(), cap=n + 16)
            torch.cuda.synchronize()
        prof(arr, 1)
        blocks = tiles * reps
        r = {PHASES[i]: round(arr[i] / blocks, 1) for i in range(len(PHASES))}
        r["candidates_per_tile"] = round(arr[5] / blocks, 1)
        r["live_per_tile"] = round(arr[6] / blocks, 2)
        r["jump_rounds_per_tile"] = round(arr[7] / blocks, 2)
        # clock64 ticks -> GHz via the 100 MHz wall clock over the same wavefronts
        r["clock_GHz"] = round(arr[13] / (arr[12] * 10.0), 3) if arr[12] else None
        out[name] = r
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
