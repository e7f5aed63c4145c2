#!/usr/bin/env python3
"""Per-dispatch SQ counters (median over dispatches) per kernel from rocprofv3
--pmc CSV directories (tools/gpu_pmc_scan.sh), merged into one JSON.

usage: python tools/sq_summary.py DIR [DIR ...] --note TEXT --out profiles/rNN/x.json"""
import argparse
import csv
import glob
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--note", default="")
    ap.add_argument("--out")
    a = ap.parse_args()
    per = {}
    for d in a.dirs:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                k = row["Kernel_Name"].split("(")[0].replace("void ", "")
                key = (f, row["Dispatch_Id"])
                per.setdefault(k, {}).setdefault(row["Counter_Name"], {}).setdefault(key, 0.0)
                per[k][row["Counter_Name"]][key] += float(row["Counter_Value"])
    out = {"note": a.note, "per_dispatch": {}}
    for k, cs in sorted(per.items()):
        out["per_dispatch"][k] = {c: round(statistics.median(v.values())) for c, v in sorted(cs.items())}
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
