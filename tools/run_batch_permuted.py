#!/usr/bin/env python3
"""C2 with its descriptors permuted through the planned fws_gpu_unmask_batch, 10 calls (for kernel traces)."""
import sys, os
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '/root/repo'))
import numpy as np, torch
from flashws_amd import _lib, gpu
L = _lib.lib(); L.fws_internal_set_unmask_any(0)
dev = torch.device('cuda:0')
w2, d2, _ = gpu.config_c2()
d2 = d2[np.random.default_rng(5).permutation(len(d2))]
c = gpu.Ctx(0, max_frames=len(d2) + 8, max_stream_bytes=len(w2))
dd = gpu.descs_to_device(d2, dev)
b = torch.from_numpy(w2).to(dev)
for i in range(10): gpu.unmask_batch(c, b, dd, len(d2))
torch.cuda.synchronize()
print(gpu.plan_mode(c))
