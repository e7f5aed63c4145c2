#!/usr/bin/env python3
"""Per-workgroup timelines of k_merge / k_link / k_emit from the FWS_SCAN_PROF
build (make -C flashws_amd/csrc prof): for the last of a few C2/C3 decodes,
each kernel's workgroup start spread and per-phase durations (us; median,
p90, max over workgroups), plus the last k_link workgroup's resolve phases."""
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

KW = 1024


def n_super_tiles(nbytes):
    """merge_kernels.hip st_tiles_for: 512 KiB super tiles, halved (to 64 KiB)
    while a stream gives fewer than 512 of them"""
    tiles = (nbytes + 2047) // 2048
    t = 256
    while t > 32 and tiles < t * 512:
        t //= 2
    return (tiles + t - 1) // t


def stats(v):
    v = np.asarray(v, dtype=np.float64)
    if v.size == 0:
        return None
    return {"med": round(float(np.median(v)), 2), "p90": round(float(np.percentile(v, 90)), 2),
            "max": round(float(v.max()), 2)}


def main():
    dev = torch.device("cuda:0")
    L = _lib.lib()
    tr = L.fws_internal_merge_trace
    tr.argtypes = [C.POINTER(C.c_ulonglong)]
    out = {}
    cfgs = (("C2", gpu.config_c2), ("C3", gpu.config_c3),
            ("dense64", lambda: gpu.config_c2(n_frames=200_000, payload=64)))
    for name, mk in cfgs:
        wire, descs, _ = mk()
        n = len(descs)
        ctx = gpu.Ctx(0, max_frames=n + 16, max_stream_bytes=len(wire))
        w = torch.from_numpy(wire).to(dev)
        n_st = n_super_tiles(len(wire))
        for _ in range(4):
            gpu.decode_stream(ctx, w, cap=n + 16)
        torch.cuda.synchronize()
        arr = (C.c_ulonglong * (KW * 32))()
        tr(arr)
        t = np.frombuffer(arr, dtype=np.uint64).reshape(KW, 32).astype(np.float64) / 100.0   # us
        r = {}
        m = t[:n_st]
        t0 = m[:, 30].min()
        r["k_merge_start_spread_us"] = stats(m[:, 30] - t0)
        prev = m[:, 30]
        for k, lab in enumerate(["counts", "records", "next+table", "jump", "tails"]):
            r[f"k_merge_{lab}"] = stats(m[:, k] - prev)
            prev = m[:, k]
        r["k_merge_end_us"] = stats(m[:, 4] - t0)
        end = m[:, 4] - t0
        slow = np.argsort(end)[-5:][::-1]
        r["k_merge_rows"] = {str(int(i)): [round(float(m[i, k] - m[i, 30]), 2) for k in (0, 1, 2, 3, 4)]
                             + [int(m[i, 22] * 100), int(m[i, 23] * 100)]
                             for i in (0, 1, n_st // 2, n_st - 2, n_st - 1)}
        r["k_merge_slowest"] = [{"st": int(i), "end_us": round(float(end[i]), 2),
                                 "records_us": round(float(m[i, 1] - m[i, 0]), 2),
                                 "counts_us": round(float(m[i, 0] - m[i, 30]), 2)} for i in slow]
        big = m[:, 21] > m[:, 30]
        if big.any():
            prev = m[big, 0]
            for k, lab in zip((18, 19, 20, 21), ["offsets", "next", "jump", "results"]):
                r[f"merge_mid_{lab}"] = stats(m[big, k] - prev)
                prev = m[big, k]
        e = t[:n_st]
        t0e = e[:, 28].min()
        ok = e[:, 26] > e[:, 28]
        r["k_emit_start_spread_us"] = stats(e[:, 28] - t0e)
        prev = e[:, 28]
        for k, lab in zip((24, 25, 26), ["load", "mark", "write"]):
            r[f"k_emit_{lab}"] = stats((e[:, k] - prev)[ok])
            prev = e[:, k]
        r["k_emit_end_us"] = stats(e[ok, 26] - t0e)
        r["gap_merge_end_to_emit_start_us"] = round(float(t0e - m[:, 4].max()), 2)
        # the last k_link workgroup's resolve phases (marks 10..17 in its row)
        lk = t[:, 17]
        row = int(np.argmax(lk))
        if lk[row] > 0:
            names = ["root+init", "compact", "cnx", "prune", "entries", "st_scan", "-", "terminal"]
            prev = t[row, 29]
            ph = {}
            for k in range(10, 18):
                if k == 16:
                    continue
                ph[names[k - 10]] = round(float(t[row, k] - prev), 2)
                prev = t[row, k]
            r["k_link_last_wg_phases_us"] = ph
            r["k_link_last_wg_start_after_link_start_us"] = round(float(t[row, 29] - t[:, 29][t[:, 29] > 0].min()), 2)
        r["counters"] = gpu.decode_counters(ctx)
        import ctypes as CT
        raw = (CT.c_uint32 * 16)()
        L.fws_internal_decode_counters(ctx.h, raw, 16)
        r["counters_raw"] = list(raw)
        out[name] = r
        ctx.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
