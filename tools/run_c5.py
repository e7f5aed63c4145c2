#!/usr/bin/env python3
"""BASELINE C5 per-GPU share (262 144 x 16 KiB TEXT frames, 4 GiB) through
fws_gpu_decode_stream with UTF-8 flags, a few times, for rocprofv3 traces."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu  # noqa: E402


def main(reps=4):
    dev = torch.device("cuda:0")
    w5, d5, ok5 = gpu.config_c5()
    n = len(d5)
    ctx = gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(w5))
    w = torch.from_numpy(w5).to(dev)
    del w5
    ok = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
    for _ in range(reps):
        rc, _, res, _ = gpu.decode_stream(ctx, w, cap=n + 64, utf8_ok=ok)
        assert rc == 0
    torch.cuda.synchronize()
    r = gpu.read_result(res)
    assert int(r["status"]) == 0 and int(r["n_frames"]) == n, r
    ctx.close()


if __name__ == "__main__":
    main()
