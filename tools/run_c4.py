#!/usr/bin/env python3
"""BASELINE C4 (one 256 MiB fragmented message) through fws_gpu_unmask_gather,
repeatedly, for rocprofv3 kernel traces; the source rotates over 4 copies as in
bench.py (past the 256 MB Infinity Cache)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu  # noqa: E402


def main(steps=20):
    dev = torch.device("cuda:0")
    w4, d4, _ = gpu.config_c4()
    c = gpu.Ctx(0, max_frames=len(d4) + 8, max_stream_bytes=len(w4))
    srcs = [torch.from_numpy(w4).to(dev) for _ in range(4)]
    total = int(d4["payload_len"].sum())
    dsts = [torch.empty(total + 64, dtype=torch.uint8, device=dev) for _ in range(4)]
    dd = gpu.descs_to_device(d4, dev)
    for i in range(steps):
        gpu.unmask_gather(c, dsts[i % 4], srcs[i % 4], dd, len(d4))
    torch.cuda.synchronize()
    c.close()


if __name__ == "__main__":
    main()
