#!/usr/bin/env python3
"""C3 stream decode with k batches in flight (k contexts on k non-blocking HIP
streams, batches round-robin), k = 1..4: ms per batch, median of 3
repetitions on fresh streams.

usage: python tools/n_in_flight.py [c3|c2] [steps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "c3"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    wire, descs, _ = {"c3": gpu.config_c3, "c2": gpu.config_c2}[which]()
    n = len(descs)
    dev = torch.device("cuda:0")
    src = torch.from_numpy(wire).to(dev)
    bufs = [src.clone() for _ in range(8)]
    alg = len(wire) + int(descs["payload_len"].sum())
    ctxs = [gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=len(wire)) for _ in range(4)]
    frs = [torch.empty((n + 64) * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev) for _ in range(4)]
    rss = [torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev) for _ in range(4)]
    for k in (1, 2, 3, 4):
        reps = []
        for _ in range(3):
            sts = [gpu.hip_stream() for _ in range(k)]
            def step(i):
                j = i % k
                rc, _, _, _ = gpu.decode_stream(ctxs[j], bufs[i % 8], n + 64, frames=frs[j], result=rss[j], stream=sts[j])
                assert rc == 0
            for i in range(2 * k):
                step(i)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(steps):
                step(i)
            torch.cuda.synchronize()
            reps.append((time.perf_counter() - t0) / steps)
        for j in range(k):
            r = gpu.read_result(rss[j])
            assert int(r["status"]) == 0 and int(r["n_frames"]) == n, r
        t = sorted(reps)[1]
        print(f"{which} {k} in flight: {t * 1e3:.4f} ms per batch ({alg / t / 1e9 / 8000 * 100:.1f} % of 8 TB/s), "
              f"reps {[round(x * 1e3, 4) for x in reps]}", flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
