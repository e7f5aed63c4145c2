#!/usr/bin/env python3
"""C5 descriptor-mode pass (fws_gpu_unmask_sorted_utf8, 4 GiB) timed in two blocks of 10 calls
after one warm-up call, alone or after what bench.py runs before it (modes: plain, stream,
pre, pre_stream). usage: python tools/c5_warmup_probe.py MODE"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flashws_amd import gpu
dev = torch.device("cuda:0")
mode = sys.argv[1]
keep = []
if "pre" in mode:   # what the bench holds before C5: the C2 headline buffers and a decoded C3 set
    w2, d2, _ = gpu.config_c2()
    keep += [torch.from_numpy(w2).to(dev) for _ in range(4)]
    w3, d3, _ = gpu.config_c3()
    c3 = gpu.Ctx(0, max_frames=len(d3) + 64, max_stream_bytes=len(w3))
    b3 = [torch.from_numpy(w3).to(dev) for _ in range(4)]
    for i in range(20): gpu.decode_stream(c3, b3[i % 4], len(d3) + 64)
    torch.cuda.synchronize(); c3.close(); del b3
w5, d5, ok5 = gpu.config_c5()
def timeit(fn, steps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(); torch.cuda.synchronize(); e0.record()
    for i in range(steps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps
out = {"mode": mode}
if "stream" in mode:
    c = gpu.Ctx(0, max_frames=len(d5) + 64, max_stream_bytes=len(w5))
    b = torch.from_numpy(w5).to(dev)
    ok = torch.zeros(len(d5) + 64, dtype=torch.uint8, device=dev)
    out["stream_ms"] = timeit(lambda: gpu.decode_stream(c, b, len(d5) + 64, utf8_ok=ok), 20)
    c.close(); del b
c = gpu.Ctx(0, max_frames=len(d5) + 8, max_stream_bytes=len(w5))
wd = torch.from_numpy(w5).to(dev)
dd5 = gpu.descs_to_device(d5, dev)
ok = torch.empty(len(d5), dtype=torch.uint8, device=dev)
gpu.unmask_sorted_utf8(c, wd, dd5, len(d5), ok); torch.cuda.synchronize()
out["flags_ok"] = bool(np.array_equal(ok.cpu().numpy(), np.asarray(ok5, dtype=np.uint8)[:len(d5)]))
out["desc_ms"] = timeit(lambda: gpu.unmask_sorted_utf8(c, wd, dd5, len(d5), ok), 10)
out["desc_ms_2"] = timeit(lambda: gpu.unmask_sorted_utf8(c, wd, dd5, len(d5), ok), 10)
print(json.dumps(out))
