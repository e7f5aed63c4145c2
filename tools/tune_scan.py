#!/usr/bin/env python3
"""Stream-decode time vs persistent k_scan residency (workgroups per CU, via
fws_internal_set_scan_blocks_per_cu). Frames/bytes of every setting are
checked against the first one."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu, lib  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    setb = lib().fws_internal_set_scan_blocks_per_cu
    setb.argtypes = [C.c_int]
    setb.restype = C.c_int
    settings = [int(x) for x in (sys.argv[1:] or ["1", "2", "3", "4", "8"])]
    out = {}
    for name, mk in (("C2", gpu.config_c2), ("C3", gpu.config_c3)):
        wire, descs, _ = mk()
        n = len(descs)
        src = torch.from_numpy(wire).to(dev)
        bufs = [src.clone() for _ in range(4)]
        ref = None
        res = {}
        for bpc in settings:
            setb(bpc)
            ctx = gpu.Ctx(0, max_frames=n + 16, max_stream_bytes=len(wire))
            w = src.clone()
            rc, fr, rs, _ = gpu.decode_stream(ctx, w, cap=n + 16)
            assert rc == 0
            got = (w, fr[:n * 24].clone())
            if ref is None:
                ref = got
            else:
                assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]), bpc
            times = []
            for rnd in range(3):
                for b in bufs:
                    b.copy_(src)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(20):
                    gpu.decode_stream(ctx, bufs[i % 4], cap=n + 16, frames=fr, result=rs)
                e1.record()
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1) / 20)
            res[bpc] = round(min(times) * 1000, 1)
            del ctx
        out[name] = {"us_per_decode": res}
    setb(0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
