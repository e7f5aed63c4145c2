#!/usr/bin/env python3
"""Runs fws_gpu_decode_stream on one BASELINE config a few times (for
rocprofv3 --pmc / --kernel-trace runs of the decode kernels).

usage: python tools/run_decode.py [c2|c3|dense|c5_256m] [reps] [stream variant]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib, gpu  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "c3"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    if len(sys.argv) > 3:
        _lib.lib().fws_internal_set_stream_variant(int(sys.argv[3]))
    mk = {"c2": gpu.config_c2, "c3": gpu.config_c3,
          "dense": lambda: gpu.config_c2(n_frames=200_000, payload=64),
          "c5_256m": lambda: gpu.config_c5(n_frames=16384)}[which]
    wire, descs, _ = mk()
    dev = torch.device("cuda:0")
    ctx = gpu.Ctx(0, max_frames=len(descs) + 64, max_stream_bytes=len(wire))
    ws = [torch.from_numpy(wire).to(dev) for _ in range(4)]
    for i in range(reps):
        rc, _, res, _ = gpu.decode_stream(ctx, ws[i % 4], cap=len(descs) + 64)
        assert rc == 0
    torch.cuda.synchronize()
    r = gpu.read_result(res)
    assert int(r["status"]) == 0 and int(r["n_frames"]) == len(descs), r
    ctx.close()
    print("ok", which, reps)


if __name__ == "__main__":
    main()
