#!/usr/bin/env python3
"""Debug aid for the one-pass decode: decode C3 (or C2) with k_fused forced,
compare the bytes with the descriptor-mode unmask of the same input and print
the mismatching 32 KiB super tiles, the k_fused counters and those STs' phase
records (tools/prof_fused.py layout).

usage: python tools/debug_fused.py [c3|c2] [calls]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flashws_amd import _lib, gpu  # noqa: E402

W = 12


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "c3"
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    L = _lib.lib()
    L.fws_internal_fused_trace_read.restype = C.c_longlong
    wire, descs, _ = {"c3": gpu.config_c3, "c2": gpu.config_c2}[which]()
    dev = torch.device("cuda:0")
    ctx = gpu.Ctx(0, max_frames=len(descs) + 64, max_stream_bytes=len(wire))
    ref = torch.from_numpy(wire).to(dev)
    gpu.unmask_batch(ctx, ref, gpu.descs_to_device(descs, dev), len(descs))
    want = ref.cpu().numpy()
    n_st = (len(wire) + 32767) // 32768
    L.fws_internal_set_fused(2)
    L.fws_internal_fused_trace(1)
    for c in range(calls):
        buf = torch.from_numpy(wire).to(dev)
        rc, fr, res, _ = gpu.decode_stream(ctx, buf, cap=len(descs) + 64)
        torch.cuda.synchronize()
        r = gpu.read_result(res)
        cn = (C.c_uint32 * 32)()
        L.fws_internal_decode_counters(ctx.h, cn, 32)
        got = buf.cpu().numpy()
        bad = np.nonzero(got != want)[0]
        sts = np.unique(bad // 32768)
        print(f"call {c}: rc={rc} status={int(r['status'])} n_frames={int(r['n_frames'])}/{len(descs)} "
              f"ffail={'~%d' % ((~cn[14]) & 0xffffffff) if cn[14] else '-'} ftimeout={cn[17]:#x} "
              f"bad bytes={len(bad)} in {len(sts)} STs: {sts[:20].tolist()}", flush=True)
        out = np.zeros(n_st * W, dtype=np.uint64)
        L.fws_internal_fused_trace_read(out.ctypes.data_as(C.POINTER(C.c_uint64)), n_st)
        t = out.reshape(-1, W).astype(np.int64)
        for s in sts[:6]:
            b = bad[bad // 32768 == s]
            print(f"  ST {s}: bytes {b[0] - s * 32768}..{b[-1] - s * 32768} ({len(b)}), done={t[s, 4] > 0} "
                  f"window={t[s, 5]} lbspins={t[s, 6]}", flush=True)
            # frames around the first bad byte
            po = descs["payload_off"]
            i = int(np.searchsorted(po, b[0], side="right")) - 1
            for f in range(max(i - 1, 0), min(i + 2, len(descs))):
                print(f"    frame {f}: payload [{po[f]}, {po[f] + descs['payload_len'][f]}) ST {po[f] // 32768}"
                      f"..{(po[f] + descs['payload_len'][f]) // 32768}", flush=True)
    L.fws_internal_fused_trace(0)
    L.fws_internal_set_fused(0)
    ctx.close()


if __name__ == "__main__":
    main()
