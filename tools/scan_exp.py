#!/usr/bin/env python3
"""k_scan timing experiments: runs the C3 stream decode 12 times through a
variant library built with -DFWS_SCAN_EXP=n (phases skipped, so the results
are not checked) for a rocprofv3 kernel trace of k_scan alone.

usage: python tools/scan_exp.py flashws_amd/lib/libfws_gpu_expN.so"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flashws_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, sys.argv[1])
from flashws_amd import gpu  # noqa: E402


def main():
    wire, descs, _ = gpu.config_c3()
    dev = torch.device("cuda:0")
    ctx = gpu.Ctx(0, max_frames=len(descs) + 64, max_stream_bytes=len(wire))
    ws = [torch.from_numpy(wire).to(dev) for _ in range(4)]
    for i in range(12):
        gpu.decode_stream(ctx, ws[i % 4], cap=len(descs) + 64)
    torch.cuda.synchronize()
    ctx.close()
    print("ok", sys.argv[1])


if __name__ == "__main__":
    main()
