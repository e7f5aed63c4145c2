#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter CSVs (one value per counter
per dispatch, averaged over a kernel's dispatches after the first `skip`).
usage: python tools/pmc_kernel_avg.py DIR [DIR ...] [--kernel SUBSTR] [--skip N]"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--skip", type=int, default=4)
    a = ap.parse_args()
    for d in a.dirs:
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        for f in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = r["Kernel_Name"]
                    if a.kernel and a.kernel not in k:
                        continue
                    vals[k][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"]),
                                                       int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
        for k, cs in vals.items():
            out = {}
            for c, v in cs.items():
                v.sort()
                v = v[a.skip:] if len(v) > a.skip else v
                out[c] = sum(x[1] for x in v) / len(v)
                out["_us"] = sum(x[2] for x in v) / len(v) / 1e3
                out["_n"] = len(v)
            print(d, k[:60], {c: round(x, 3) for c, x in sorted(out.items())})


if __name__ == "__main__":
    main()
