#!/usr/bin/env python3
"""Per-super-tile clocks of the one-launch decode (k_stream, stream_kernels.hip)
from the FWS_STREAM_TRACE build (make -C flashws_amd/csrc prof ->
flashws_amd/lib/libfws_gpu_prof.so): scan, hand-off to the unmasker, guess +
C publish, verify, look-back, frames + unmask, look-back window; start-time
spread by ticket; kernel time per call by HIP events.

usage: python tools/prof_stream.py [c2|c3|dense64|c5_256m] [calls]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from flashws_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "flashws_amd", "lib", "libfws_gpu_prof.so")
from flashws_amd import gpu  # noqa: E402

W = 10   # stream_kernels.hip kXTraceW
NAMES = ["scan", "scan_to_P", "P_to_unmasker", "guess+C", "verify", "lookback", "frames+unmask"]


def stats(v):
    v = np.asarray(v, dtype=np.float64)
    if v.size == 0:
        return None
    return {"med": round(float(np.median(v)), 2), "p90": round(float(np.percentile(v, 90)), 2),
            "max": round(float(v.max()), 2)}


def run(which, calls):
    L = _lib.lib()
    L.fws_internal_fused_trace_read.restype = C.c_longlong
    mk = {"c2": gpu.config_c2, "c3": gpu.config_c3,
          "dense64": lambda: gpu.config_c2(n_frames=200_000, payload=64),
          "c5_256m": lambda: gpu.config_c5(n_frames=16384)}[which]
    wire, descs, _ = mk()
    dev = torch.device("cuda:0")
    ctx = gpu.Ctx(0, max_frames=len(descs) + 64, max_stream_bytes=len(wire))
    bufs = [torch.from_numpy(wire).to(dev) for _ in range(4)]
    cap = len(descs) + 64
    old = L.fws_internal_set_fused(1)
    L.fws_internal_fused_trace(1)
    rec = {"calls": []}
    for c in range(calls):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc, _, res, _ = gpu.decode_stream(ctx, bufs[c % 4], cap=cap)
        e1.record()
        torch.cuda.synchronize()
        r = gpu.read_result(res)
        cn = (C.c_uint32 * 32)()
        L.fws_internal_decode_counters(ctx.h, cn, 32)
        rec["calls"].append({"us": round(e0.elapsed_time(e1) * 1e3, 1), "rc": rc, "status": int(r["status"]),
                             "frames_ok": int(r["n_frames"]) == len(descs), "fmode": cn[13],
                             "first_failed_st": ((~cn[14]) & 0xFFFFFFFF) if cn[14] else None,
                             "timeouts": cn[17]})
    n_st = (len(wire) + 32767) // 32768
    out = np.zeros(n_st * W, dtype=np.uint64)
    got = L.fws_internal_fused_trace_read(out.ctypes.data_as(C.POINTER(C.c_uint64)), n_st)
    L.fws_internal_fused_trace(0)
    L.fws_internal_set_fused(old)
    t = out.reshape(-1, W)[:got].astype(np.float64)
    ok = t[:, 7] > 0
    rec["super_tiles"] = int(got)
    rec["committed"] = int(ok.sum())
    t = t[ok] / 100.0   # us
    if len(t):
        base = t[:, 0].min()
        rec["span_us"] = round(float(t[:, 7].max() - base), 1)
        for i, name in enumerate(NAMES):
            rec[name + "_us"] = stats(t[:, i + 1] - t[:, i])
        rec["lookback_window"] = stats(t[:, 8] * 100.0)
        q = np.linspace(0, len(t) - 1, 9).astype(int)
        rec["scan_start_by_ticket_us"] = [round(float(t[i, 0] - base), 1) for i in q]
        rec["done_by_ticket_us"] = [round(float(t[i, 7] - base), 1) for i in q]
    ctx.close()
    return rec


def main():
    which = sys.argv[1:2] or ["c3"]
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    cfgs = which if which != ["all"] else ["c2", "c3", "dense64"]
    print(json.dumps({w: run(w, calls) for w in cfgs}, indent=1))


if __name__ == "__main__":
    main()
