#!/usr/bin/env python3
"""C4 reassembly step timing (fws_gpu_unmask_gather on the 256 MiB fragmented
message, 4 rotating destinations, HIP events); prints the step time and the
output's sha256 so an A/B build can be checked equal.

usage: python tools/time_c4.py [--lib PATH] [steps]"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib  # noqa: E402
if "--lib" in sys.argv:
    _lib.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
from flashws_amd import gpu  # noqa: E402


def main():
    steps = int(sys.argv[-1]) if sys.argv[-1].isdigit() else 100
    dev = torch.device("cuda:0")
    w4, d4, _ = gpu.config_c4()
    c = gpu.Ctx(0, max_frames=len(d4) + 8, max_stream_bytes=len(w4))
    src = torch.from_numpy(w4).to(dev)
    total = int(d4["payload_len"].sum())
    dsts = [torch.empty(total + 64, dtype=torch.uint8, device=dev) for _ in range(4)]
    dd = gpu.descs_to_device(d4, dev)
    out = {"lib": os.path.basename(_lib.LIB_PATH), "step_us": []}
    for rep in range(3):
        for i in range(10):
            gpu.unmask_gather(c, dsts[i % 4], src, dd, len(d4))
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(steps):
            gpu.unmask_gather(c, dsts[i % 4], src, dd, len(d4))
        e1.record()
        torch.cuda.synchronize()
        out["step_us"].append(round(e0.elapsed_time(e1) * 1e3 / steps, 2))
    out["out_sha16"] = hashlib.sha256(dsts[0][:total].cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps(out))
    c.close()


if __name__ == "__main__":
    main()
