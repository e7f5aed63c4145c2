#!/usr/bin/env python3
"""C2-shaped TX encode (65 536 x 4 KiB client frames) run repeatedly, for
rocprofv3 kernel traces of the fws_gpu_encode_frames launch sequence; the
payloads rotate over 4 copies as in bench.py (past the 256 MB Infinity Cache)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu  # noqa: E402


def setup(n=65536, pl=4096):
    """Context, 4 output buffers, 4 copies of the source payloads, device TX
    descriptors, n, total out bytes."""
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(7)
    txd = np.zeros(n, dtype=gpu.TX_DESC)
    txd["src_off"] = np.arange(n, dtype=np.uint64) * pl
    txd["len"] = pl
    txd["key"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    txd["opcode"], txd["fin"], txd["masked"] = 2, 1, 1
    payload = rng.integers(0, 256, n * pl, dtype=np.uint8)
    srcs = [torch.from_numpy(payload).to(dev) for _ in range(4)]
    dd = torch.from_numpy(txd.view(np.uint8).copy()).to(dev)
    total = n * (pl + 8)
    ctx = gpu.Ctx(0, max_frames=n, max_stream_bytes=total)
    outs = [torch.empty(total, dtype=torch.uint8, device=dev) for _ in range(4)]
    return ctx, outs, srcs, dd, n, total


def main(steps=20):
    ctx, outs, srcs, dd, n, _ = setup()
    if os.environ.get("FWS_TX_FORM"):          # fws_internal_set_tx_w5: 0 w4, 1 w5, 2 dpp5, 3 so, 4 sod, 5 sr
        from flashws_amd import _lib
        _lib.lib().fws_internal_set_tx_w5(int(os.environ["FWS_TX_FORM"]))
    for i in range(steps):
        gpu.encode_frames(ctx, outs[i % 4], srcs[i % 4], dd, n)
    torch.cuda.synchronize()
    ctx.close()


if __name__ == "__main__":
    main()
