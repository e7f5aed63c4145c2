#!/usr/bin/env python3
"""Where a multi-launch step's time goes: from a rocprofv3 kernel-trace CSV,
cut the kernel sequence into steps at every launch of `first` (a kernel-name
prefix), then print the median over steps of each kernel's duration, of the
gap before it (end of the previous kernel -> its start: the launch boundary
the GPU sees), and of the whole span (first start -> last end). Steps whose
launches were queued ahead (back-to-back calls) show the device-side cost.

usage: python tools/step_gaps.py kernel_trace.csv first_kernel_prefix [--skip N]"""
import argparse
import csv
import json

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("first")
    ap.add_argument("--skip", type=int, default=3, help="steps dropped at the start (warm-up)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], None
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fwsk::", "")
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if name.startswith(a.first):
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append((name, t0, t1))
    steps = steps[a.skip:-1] if len(steps) > a.skip + 1 else steps
    shape = [k[0] for k in steps[0]]
    steps = [s for s in steps if [k[0] for k in s] == shape]
    out = {"steps": len(steps), "kernels": []}
    for i, name in enumerate(shape):
        dur = [ (s[i][2] - s[i][1]) / 1e3 for s in steps]
        gap = [ (s[i][1] - s[i - 1][2]) / 1e3 for s in steps] if i else [0.0]
        out["kernels"].append({"kernel": name[:48], "us": round(float(np.median(dur)), 2),
                               "gap_before_us": round(float(np.median(gap)), 2)})
    span = [(s[-1][2] - s[0][1]) / 1e3 for s in steps]
    nxt = [(steps[j + 1][0][1] - steps[j][-1][2]) / 1e3 for j in range(len(steps) - 1)]
    out["span_us"] = round(float(np.median(span)), 2)
    out["gap_to_next_step_us"] = round(float(np.median(nxt)), 2) if nxt else None
    out["step_period_us"] = round(float(np.median([(steps[j + 1][0][1] - steps[j][0][1]) / 1e3
                                                    for j in range(len(steps) - 1)])), 2) if nxt else None
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
