#!/usr/bin/env python3
"""Stream-decode timing of C2-stream, C3 and the dense 64 B workload (HIP events
over back-to-back calls, >= 1 GiB of rotating device batches). Prints one JSON
object; checks frame counts.

usage: python tools/time_decode.py [reps] [--lib PATH]   (--lib: an A/B build, e.g. libfws_gpu_exp.so)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib  # noqa: E402
if "--lib" in sys.argv:
    _lib.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
from flashws_amd import gpu  # noqa: E402


def time_cfg(name, wire, n, reps):
    L = _lib.lib()
    dev = torch.device("cuda:0")
    nbuf = max(4, -(-(1 << 30) // len(wire)))
    bufs = [torch.from_numpy(wire).to(dev) for _ in range(nbuf)]
    ctx = gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(wire))
    cap = n + 64
    frames = torch.empty(cap * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev)
    res = torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev)
    for i in range(2):
        gpu.decode_stream(ctx, bufs[i % nbuf], cap, frames=frames, result=res)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        gpu.decode_stream(ctx, bufs[i % nbuf], cap, frames=frames, result=res)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / reps
    r = gpu.read_result(res)
    c = gpu.decode_counters(ctx)

    payload = int(gpu.read_frames(frames, n)["payload_len"].sum())
    alg = len(wire) + payload
    ctx.close()
    return {"ms": round(t * 1e3, 4), "frac": round(alg / t / 8e12, 4), "status": int(r["status"]),
            "frames_ok": int(r["n_frames"]) == n, "survivors": c["survivors"], "big": c["big_super_tiles"]}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 20
    out = {}
    cfgs = [("C2", gpu.config_c2()), ("C3", gpu.config_c3()),
            ("dense64", gpu.config_c2(n_frames=200_000, payload=64))]
    for name, (wire, descs, _) in cfgs:
        out[name] = time_cfg(name, wire, len(descs), reps)
        print(name, out[name], flush=True, file=sys.stderr)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
