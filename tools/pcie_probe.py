#!/usr/bin/env python3
"""PCIe copy probe: pinned H2D alone, D2H alone, and both at once on two
streams (is the link used full duplex?). Prints one JSON object."""
import json
import time

import torch


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    n = 256 << 20
    dev = torch.device("cuda:0")
    h_in = torch.empty(n, dtype=torch.uint8).pin_memory()
    h_out = torch.empty(n, dtype=torch.uint8).pin_memory()
    d_a = torch.empty(n, dtype=torch.uint8, device=dev)
    d_b = torch.empty(n, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out = {}

    def h2d():
        with torch.cuda.stream(s1):
            d_a.copy_(h_in, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h_out.copy_(d_b, non_blocking=True)

    def both():
        h2d()
        d2h()

    for name, fn in (("h2d", h2d), ("d2h", d2h), ("both_2_streams", both)):
        t = timed(fn)
        out[name] = {"ms": round(t * 1e3, 3), "GB_per_s_each": round(n / t / 1e9, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
