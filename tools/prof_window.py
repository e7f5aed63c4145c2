#!/usr/bin/env python3
"""Kernel stats over the timed window of a bench.py config run under rocprofv3
(--kernel-trace): per kernel name, the last K dispatches (a config's timed
calls come after its warm-up calls; run bench.py --only CFG --no-pipelined so
nothing else follows them). Writes rocprofv3's stats columns for the window,
plus the run's whole-run stats beside it, and prints a JSON summary.

usage: python tools/prof_window.py TRACE_CSV --last K --out OUT.csv [--json OUT.json] [--bench BENCH_LINE.json]"""
import argparse
import csv
import json
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--json")
    ap.add_argument("--bench", help="the bench.py JSON line of the same run (its ms_per_step per config)")
    a = ap.parse_args()
    runs = defaultdict(list)
    for row in csv.DictReader(open(a.trace)):
        if row.get("Kind", "KERNEL_DISPATCH") != "KERNEL_DISPATCH":
            continue
        runs[row["Kernel_Name"]].append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    rows, summary = [], {}
    for name, v in runs.items():
        v.sort()
        w = [e - s for s, e in v[-a.last:]]
        allw = [e - s for s, e in v]
        rows.append((name, len(w), sum(w), sum(w) / len(w), min(w), max(w), statistics.pstdev(w) if len(w) > 1 else 0.0))
        summary[name.split("(")[0].replace("void ", "")] = {
            "window_calls": len(w), "window_avg_us": round(sum(w) / len(w) / 1e3, 3),
            "window_min_us": round(min(w) / 1e3, 3), "window_max_us": round(max(w) / 1e3, 3),
            "all_calls": len(allw), "all_avg_us": round(sum(allw) / len(allw) / 1e3, 3)}
    tot = sum(r[2] for r in rows) or 1
    rows.sort(key=lambda r: -r[2])
    with open(a.out, "w", newline="") as f:
        wr = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        wr.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for name, n, t, avg, mn, mx, sd in rows:
            wr.writerow([name, n, t, round(avg, 6), round(100.0 * t / tot, 2), mn, mx, round(sd, 6)])
    out = {"window_last": a.last, "kernels": summary}
    if a.bench:
        line = json.loads(open(a.bench).read().strip().splitlines()[-1])
        out["bench_ms_per_step"] = {k: v.get("ms_per_step") for k, v in line.get("extra", {}).items()
                                    if isinstance(v, dict) and "ms_per_step" in v}
    s = json.dumps(out, indent=1)
    if a.json:
        open(a.json, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
