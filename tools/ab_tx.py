#!/usr/bin/env python3
"""A/B of k_tx_encode grid sizes on the bench's TX workload (C2 shape: 65 536 x
4 KiB payloads framed + masked by fws_gpu_encode_frames): one wave per output
unit (0, the default) against grid caps of k x the resident workgroups
(fws_internal_set_tx_blocks), HIP events over back-to-back calls rotating four
outputs, modes alternated in one process; outputs compared across modes. One
JSON line per (mode, rep).

usage: python tools/ab_tx.py [reps]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib, gpu  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    L = _lib.lib()
    dev = torch.device("cuda:0")
    n, pl = 65536, 4096
    rng = np.random.default_rng(7)
    txd = np.zeros(n, dtype=gpu.TX_DESC)
    txd["src_off"] = np.arange(n, dtype=np.uint64) * pl
    txd["len"] = pl
    txd["key"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    txd["opcode"], txd["fin"], txd["masked"] = 2, 1, 1
    tsrc = torch.from_numpy(rng.integers(0, 256, n * pl, dtype=np.uint8)).to(dev)
    tdd = torch.from_numpy(txd.view(np.uint8).copy()).to(dev)
    total = n * (pl + 8)
    c = gpu.Ctx(0, max_frames=n, max_stream_bytes=total)
    outs = [torch.empty(total, dtype=torch.uint8, device=dev) for _ in range(4)]
    olen = torch.empty(1, dtype=torch.int64, device=dev)
    ref = None
    for rep in range(3):
        for blocks in (0, 2560, 5120, 7680, 10240):
            L.fws_internal_set_tx_blocks(blocks)
            for i in range(4):
                gpu.encode_frames(c, outs[i % 4], tsrc, tdd, n, out_len=olen)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(reps):
                gpu.encode_frames(c, outs[i % 4], tsrc, tdd, n, out_len=olen)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            got = outs[(reps - 1) % 4]
            if ref is None:
                ref = got.clone()
            same = bool(torch.equal(ref, got))
            print(json.dumps({"tx_blocks": blocks, "rep": rep, "ms": round(ms, 4),
                              "frac": round((n * pl + total) / ms / 1e-3 / 8e12, 4), "same_output": same}), flush=True)
            assert same
    L.fws_internal_set_tx_blocks(0)
    c.close()


if __name__ == "__main__":
    main()
