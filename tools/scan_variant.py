#!/usr/bin/env python3
"""Run the C2 stream decode 20x with a given build of the library (e.g. the
FWS_SCAN_STOP cut-offs from `make -C flashws_amd/csrc stops`); meant to run
under rocprofv3 --kernel-trace --stats to read k_scan's duration per build."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flashws_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "flashws_amd", "lib", sys.argv[1] if len(sys.argv) > 1 else "libfws_gpu.so")
from flashws_amd import gpu  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    wire, descs, _ = gpu.config_c2()
    n = len(descs)
    ctx = gpu.Ctx(0, max_frames=n + 16, max_stream_bytes=len(wire))
    bufs = [torch.from_numpy(wire).to(dev) for _ in range(4)]
    for i in range(24):
        rc, _, _, _ = gpu.decode_stream(ctx, bufs[i % 4], cap=n + 16)
        assert rc == 0
    torch.cuda.synchronize()
    print("ok", _lib.LIB_PATH)


if __name__ == "__main__":
    main()
