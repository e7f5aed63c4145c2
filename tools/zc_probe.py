#!/usr/bin/env python3
"""C2 batch end to end from pinned host memory, two ways (ms per batch, GiB/s of
payload): (a) H2D copy + fws_gpu_unmask_sorted + D2H copy on one stream, (b) the
kernel run directly on the pinned host buffer (zero copy: its loads and stores
cross PCIe), checks the bytes. usage: python tools/zc_probe.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu  # noqa: E402

GIB = 1 << 30


def timeit(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda:0")
    wire, descs, _ = gpu.config_c2()
    n = len(descs)
    payload = int(descs["payload_len"].sum())
    ctx = gpu.Ctx(0, max_frames=n, max_stream_bytes=len(wire))
    dd = gpu.descs_to_device(descs, dev)
    host = torch.from_numpy(wire.copy()).pin_memory()
    dbuf = torch.empty(len(wire), dtype=torch.uint8, device=dev)
    out = {}

    def copy_path():
        dbuf.copy_(host, non_blocking=True)
        gpu.unmask_sorted(ctx, dbuf, dd, n)
        host.copy_(dbuf, non_blocking=True)
    ms = timeit(copy_path, 6)
    out["h2d_kernel_d2h"] = {"ms": round(ms, 3), "GiB_per_s": round(payload / (ms / 1e3) / GIB, 1)}

    # zero copy: the kernel on the pinned host buffer itself
    ms = timeit(lambda: gpu.unmask_sorted(ctx, host, dd, n), 6)
    out["zero_copy"] = {"ms": round(ms, 3), "GiB_per_s": round(payload / (ms / 1e3) / GIB, 1)}
    # 7 copy-path + 7 zero-copy in-place passes: masked again
    out["zero_copy_bytes_ok"] = bool(np.array_equal(host.numpy(), wire))
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
