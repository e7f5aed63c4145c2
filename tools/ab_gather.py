#!/usr/bin/env python3
"""A/B of the one-launch gather (k_gather_one, fws_internal_set_gather_one 1)
against the plan launch + k_gather_fast (0) on C4 (one 256 MiB message in
1 427 fragments, sources in any order) and on a 600-fragment variant: HIP
events over back-to-back fws_gpu_unmask_gather calls rotating four
destinations, modes alternated ABAB in one process; the one-launch form also
at fixed grid sizes (fws_internal_set_gather_blocks; 0 = the resident count). One JSON line per
(config, mode, rep).

usage: python tools/ab_gather.py [reps] [--lib PATH]"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib, gpu  # noqa: E402

if "--lib" in sys.argv:                      # an A/B build (make exp), e.g. libfws_gpu_w6.so
    _lib.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
    del sys.argv[sys.argv.index("--lib"):sys.argv.index("--lib") + 2]
LIB = os.path.basename(_lib.LIB_PATH)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    L = _lib.lib()
    dev = torch.device("cuda:0")
    for name, target in (("C4", 256 << 20), ("C4_64MiB", 64 << 20)):
        w, d, _ = gpu.config_c4(target=target)
        c = gpu.Ctx(0, max_frames=len(d) + 8, max_stream_bytes=len(w))
        src = torch.from_numpy(w).to(dev)
        total = int(d["payload_len"].sum())
        dsts = [torch.empty(total + 64, dtype=torch.uint8, device=dev) for _ in range(4)]
        dd = gpu.descs_to_device(d, dev)
        outs = {}
        L.fws_internal_gather_one_grid.restype = ctypes.c_uint64
        L.fws_internal_gather_one_grid.argtypes = [ctypes.c_uint64]
        print(json.dumps({"cfg": name, "default_grid": L.fws_internal_gather_one_grid(len(w))}), flush=True)
        for rep in range(3):
            for mode, blocks in ((0, 0), (1, 0), (512, 5), (512, 6), (512, 8), (512, 4)):
                # mode 0: plan + k_gather_fast; 1: k_gather_one default; 256 / 512: k_gather_one with that
                # many threads per workgroup and `blocks` x the resident workgroups
                L.fws_internal_set_gather_one(1 if mode else 0)
                if mode > 1:
                    L.fws_internal_set_gather_shape(mode, blocks)
                else:
                    L.fws_internal_set_gather_shape(0, 0)       # the library's default shape
                for i in range(4):
                    gpu.unmask_gather(c, dsts[i % 4], src, dd, len(d))
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(reps):
                    gpu.unmask_gather(c, dsts[i % 4], src, dd, len(d))
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
                outs[mode] = dsts[(reps - 1) % 4][:total].clone()
                print(json.dumps({"lib": LIB, "cfg": name, "fragments": len(d), "gather_one": mode, "blocks": blocks, "rep": rep,
                                  "ms": round(ms, 4), "GiB_per_s": round(total / ms / 1e-3 / 2**30, 1)}), flush=True)
            assert torch.equal(outs[0], outs[1])
        L.fws_internal_set_gather_one(1)
        L.fws_internal_set_gather_shape(0, 0)
        c.close()
        del src, dsts


if __name__ == "__main__":
    main()
