#!/usr/bin/env python3
"""A/B of the stream unmask variants (fws_internal_set_stream_variant): the
fused decode of C2 / C3 / C5 batches, 4 rotating device buffers per config
(>= 1 GiB apart from C5, so a step starts cold), ms per decode.

usage: python tools/tune_stream.py [steps]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib, gpu  # noqa: E402


def bench(name, wire, n, steps, nbuf, utf8=False):
    dev = torch.device("cuda:0")
    ctx = gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(wire))
    bufs = [torch.from_numpy(wire).to(dev) for _ in range(nbuf)]
    cap = n + 64
    fr = torch.empty(cap * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev)
    res = torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev)
    ok = torch.zeros(cap, dtype=torch.uint8, device=dev) if utf8 else None
    out = {}
    L = _lib.lib()
    for v in (0, 1, 2, 3, 0, 1):
        L.fws_internal_set_stream_variant(v)
        for i in range(4):
            gpu.decode_stream(ctx, bufs[i % nbuf], cap, frames=fr, result=res, utf8_ok=ok)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            rc, _, _, _ = gpu.decode_stream(ctx, bufs[i % nbuf], cap, frames=fr, result=res, utf8_ok=ok)
            assert rc == 0
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / steps
        out.setdefault(f"v{v}", []).append(round(t * 1e3, 4))
    r = gpu.read_result(res)
    assert int(r["status"]) == 0 and int(r["n_frames"]) == n
    L.fws_internal_set_stream_variant(0)
    ctx.close()
    return out


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    res = {}
    w, d, _ = gpu.config_c2()
    res["C2"] = bench("C2", w, len(d), steps, 4)
    w, d, _ = gpu.config_c3()
    res["C3"] = bench("C3", w, len(d), steps, 4)
    w, d, _ = gpu.config_c5()
    res["C5"] = bench("C5", w, len(d), max(4, steps // 8) // 2 * 2, 1, utf8=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
