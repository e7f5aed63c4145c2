#!/usr/bin/env python3
"""k_scan alone (fws_internal_scan_only) over the C2 / C3 streams, HIP events
around back-to-back launches on 4 rotating 256 MiB buffers: the time of the
product scan, or of an ablation build (make -C flashws_amd/csrc exp
EXP_DEFS=-DFWS_ABL=1: stage only; 2: + candidate bits and scan).

usage: python tools/scan_ablation.py [--lib PATH] [reps]"""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib  # noqa: E402
if "--lib" in sys.argv:
    _lib.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
from flashws_amd import gpu  # noqa: E402


def main():
    reps = int(sys.argv[-1]) if sys.argv[-1].isdigit() else 50
    L = _lib.lib()
    f = L.fws_internal_scan_only
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
    f.restype = C.c_int
    dev = torch.device("cuda:0")
    out = {"lib": os.path.basename(_lib.LIB_PATH)}
    for name, mk in (("C2", gpu.config_c2), ("C3", gpu.config_c3)):
        wire, _, _ = mk()
        bufs = [torch.from_numpy(wire).to(dev) for _ in range(4)]
        ctx = gpu.Ctx(0, max_frames=1 << 17, max_stream_bytes=len(wire))
        st = torch.cuda.current_stream().cuda_stream
        for i in range(3):
            assert f(ctx.h, bufs[i % 4].data_ptr(), len(wire), st) == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            f(ctx.h, bufs[i % 4].data_ptr(), len(wire), st)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        out[name] = {"k_scan_us": round(us, 2), "read_TB_s": round(len(wire) / us / 1e6, 2)}
        ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
