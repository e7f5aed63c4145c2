#!/usr/bin/env python3
"""A/B of fws_gpu_encode_frames forms on the bench's TX workload (C2 shape:
65 536 x 4 KiB payloads framed + masked): k_out_plan + k_tx_encode ("plan")
against the one-launch k_tx_one at several output spans per workgroup
(fws_internal_set_tx_one), HIP events over back-to-back calls rotating four
outputs, modes alternated in one process (order reversed every other
repetition); outputs compared across modes. One JSON line per (mode, rep).
(r04 used it for k_tx_encode grid caps, profiles/r04/ab_tx.jsonl.) r06: the
source rotates over 4 copies (1 GiB, past the 256 MB Infinity Cache; one
source re-read every step was served partly from it) unless FWS_AB_ONE_SRC=1;
modes (fws_internal_set_tx_w5): w4, dpp5 (one load + DPP), so / sod (full
chunks only, two loads / DPP, + k_tx_seams), sr (seam chunks built by the plan).

usage: python tools/ab_tx.py [reps] [mode,mode,...]"""
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
    payload = rng.integers(0, 256, n * pl, dtype=np.uint8)
    tsrcs = [torch.from_numpy(payload).to(dev) for _ in range(1 if os.environ.get("FWS_AB_ONE_SRC") == "1" else 4)]
    tdd = torch.from_numpy(txd.view(np.uint8).copy()).to(dev)
    total = n * (pl + 8)
    c = gpu.Ctx(0, max_frames=n, max_stream_bytes=total)
    outs = [torch.empty(total, dtype=torch.uint8, device=dev) for _ in range(4)]
    olen = torch.empty(1, dtype=torch.int64, device=dev)
    ref = None
    modes = [("plan", 0, 0, 1), ("dpp5", 0, 0, 2), ("w4", 0, 0, 0), ("so", 0, 0, 3), ("sod", 0, 0, 4),
             ("sr", 0, 0, 5)] + \
        [(f"one_span{k}k", 1, k, 1) for k in (32, 64, 128, 256)]
    if len(sys.argv) > 2:
        modes = [m for m in modes if m[0] in sys.argv[2].split(",")]
    # warm the clocks before the first timed mode (tools/c4_thermal_probe.py)
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        gpu.encode_frames(c, outs[0], tsrcs[0], tdd, n, out_len=olen)
        torch.cuda.synchronize()
    for rep in range(3):
        for name, one, span, w in (modes if rep % 2 == 0 else modes[::-1]):
            L.fws_internal_set_tx_one(one, span)
            L.fws_internal_set_tx_w5(w)
            for i in range(4):
                gpu.encode_frames(c, outs[i % 4], tsrcs[i % len(tsrcs)], tdd, n, out_len=olen)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(reps):
                gpu.encode_frames(c, outs[i % 4], tsrcs[i % len(tsrcs)], tdd, n, out_len=olen)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            got = outs[(reps - 1) % 4]
            if ref is None:
                ref = got.clone()
            same = bool(torch.equal(ref, got))
            print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "mode": name, "rep": rep, "ms": round(ms, 4),
                              "frac": round((n * pl + total) / ms / 1e-3 / 8e12, 4), "same_output": same}), flush=True)
            assert same
    L.fws_internal_set_tx_one(0, 64)
    L.fws_internal_set_tx_w5(1)
    c.close()


if __name__ == "__main__":
    main()
