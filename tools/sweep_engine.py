#!/usr/bin/env python3
"""fws_decode_engine on C3 (and C2): per-batch time of one run of J distinct
256 MiB batches for each schedule -- mode 0 (whole decodes alternating over two
streams), mode 1 (scans on one stream, resolve + unmask on the other) with
scan_cus CUs for the scans (0 = no partition) -- HIP events on the caller's
stream, median of 3 runs; results checked. One JSON line per (config, schedule).

usage: python tools/sweep_engine.py [J] [mode:scan_cus ...]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import gpu  # noqa: E402


def main():
    J = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    sweep = [tuple(int(v) for v in x.split(":")) for x in sys.argv[2:]] or [(0, 0), (1, 0), (1, 128)]
    dev = torch.device("cuda:0")
    for name, (wire, descs, _) in (("C3", gpu.config_c3()), ("C2", gpu.config_c2())):
        n = len(descs)
        cap = n + 64
        bufs = [torch.from_numpy(wire).to(dev) for _ in range(J)]
        fr = [torch.empty(cap * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev) for _ in range(J)]
        rs = [torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev) for _ in range(J)]
        jobs = [(bufs[j], cap, fr[j], rs[j]) for j in range(J)]
        payload = int(descs["payload_len"].sum())
        for mode, sc in sweep:
            eng = gpu.DecodeEngine(0, max_frames=cap, max_stream_bytes=len(wire), mode=mode, scan_cus=sc)
            s = torch.cuda.current_stream()
            assert eng.run(jobs, stream=s) == 0
            torch.cuda.synchronize()
            reps = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                assert eng.run(jobs, stream=s) == 0
                e1.record(s)
                torch.cuda.synchronize()
                reps.append(e0.elapsed_time(e1) / J)
            ok = all(int(gpu.read_result(r)["status"]) == 0 and int(gpu.read_result(r)["n_frames"]) == n for r in rs)
            ms = sorted(reps)[1]
            print(json.dumps({"cfg": name, "jobs": J, "mode": mode, "scan_cus": sc, "ms_per_batch": round(ms, 4),
                              "reps": [round(x, 4) for x in reps],
                              "frac": round((len(wire) + payload) / ms / 1e-3 / 8e12, 4), "results_ok": ok}),
                  flush=True)
            eng.close()
        del bufs, fr, rs


if __name__ == "__main__":
    main()
