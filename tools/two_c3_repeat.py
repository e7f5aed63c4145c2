import sys, os
sys.path.insert(0, os.getcwd())
sys.argv = ["x"]
import tools.sweep_two as sw
import torch
from flashws_amd import gpu
wire, descs, _ = gpu.config_c3()
dev = torch.device("cuda:0")
for rep in range(3):
    o = sw.run(wire, len(descs), dev, 30, 8, 16384)
    print("c3 default: one %.1f us, two %.1f us/batch" % (o[False]*1e3, o[True]*1e3), flush=True)
