#!/usr/bin/env python3
"""A/B of the path resolve inside k_emit_path (fws_internal_set_emit_path 1)
against k_link + k_emit (0) on the C2-stream, C3 and dense 64 B decodes: HIP
events over back-to-back calls on >= 1 GiB of rotating device batches, modes
alternated ABAB in one process. Prints one JSON line per (config, mode, rep).

usage: python tools/ab_emit_path.py [reps]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib, gpu  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    L = _lib.lib()
    dev = torch.device("cuda:0")
    for name, (wire, descs, _) in (("C2", gpu.config_c2()), ("C3", gpu.config_c3()),
                                   ("dense64", gpu.config_c2(n_frames=200_000, payload=64))):
        n = len(descs)
        nbuf = max(4, -(-(1 << 30) // len(wire)))
        bufs = [torch.from_numpy(wire).to(dev) for _ in range(nbuf)]
        ctx = gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(wire))
        cap = n + 64
        frames = torch.empty(cap * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev)
        res = torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev)
        for rep in range(3):
            for mode in (1, 0):
                L.fws_internal_set_emit_path(mode)
                for i in range(4):
                    gpu.decode_stream(ctx, bufs[i % nbuf], cap, frames=frames, result=res)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(reps):
                    gpu.decode_stream(ctx, bufs[i % nbuf], cap, frames=frames, result=res)
                e1.record()
                torch.cuda.synchronize()
                r = gpu.read_result(res)
                print(json.dumps({"cfg": name, "emit_path": mode, "rep": rep,
                                  "ms": round(e0.elapsed_time(e1) / reps, 4), "status": int(r["status"]),
                                  "frames_ok": int(r["n_frames"]) == n}), flush=True)
        L.fws_internal_set_emit_path(1)
        ctx.close()
        del bufs


if __name__ == "__main__":
    main()
