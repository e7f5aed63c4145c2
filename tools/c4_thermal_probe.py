#!/usr/bin/env python3
"""Does C4 slow down after sustained load? k_gather_one step times fresh, after
15 s of back-to-back C3 stream decodes, and after 10 s idle (one process)."""
import sys, os, json, time
sys.path.insert(0, '/root/repo') if os.path.exists('/root/repo') else None
import torch
from flashws_amd import gpu
dev = torch.device('cuda:0')
w4, d4, _ = gpu.config_c4()
c = gpu.Ctx(0, max_frames=len(d4) + 8, max_stream_bytes=len(w4))
src = torch.from_numpy(w4).to(dev)
total = int(d4["payload_len"].sum())
dsts = [torch.empty(total + 64, dtype=torch.uint8, device=dev) for _ in range(4)]
dd4 = gpu.descs_to_device(d4, dev)
stream = torch.cuda.current_stream()
def tm(steps=100, warm=10):
    for i in range(warm): gpu.unmask_gather(c, dsts[i % 4], src, dd4, len(d4))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(steps): gpu.unmask_gather(c, dsts[i % 4], src, dd4, len(d4))
    e1.record(stream); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps
print(json.dumps({"phase": "fresh", "ms": [round(tm(), 4) for _ in range(3)]}), flush=True)
# heavy load: 20 s of C3-like stream decodes on 4 GiB
w3, d3, _ = gpu.config_c3()
ctx3 = gpu.Ctx(0, max_frames=len(d3) + 64, max_stream_bytes=len(w3))
bufs = [torch.from_numpy(w3).to(dev) for _ in range(4)]
t0 = time.time(); k = 0
while time.time() - t0 < 15:
    for i in range(50): gpu.decode_stream(ctx3, bufs[i % 4], len(d3) + 64)
    torch.cuda.synchronize(); k += 50
print(json.dumps({"phase": "after_load", "decodes": k, "ms": [round(tm(), 4) for _ in range(3)]}), flush=True)
time.sleep(10)
print(json.dumps({"phase": "after_10s_idle", "ms": [round(tm(), 4) for _ in range(3)]}), flush=True)
