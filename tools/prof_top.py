#!/usr/bin/env python3
"""Per-kernel summary (calls, total/avg us, %) from a rocprofv3 results database.

usage: python tools/prof_top.py gpurun_out/<dir> [--csv out.csv]
"""
import argparse
import glob
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--csv")
    a = ap.parse_args()
    dbs = glob.glob(a.path + "/**/*.db", recursive=True) if not a.path.endswith(".db") else [a.path]
    if not dbs:
        sys.exit("no .db under " + a.path)
    rows = []
    for db in dbs:
        c = sqlite3.connect(db)
        rows += list(c.execute("select name, count(*), sum(duration)/1000.0, avg(duration)/1000.0 "
                               "from kernels group by name"))
    tot = sum(r[2] for r in rows) or 1.0
    rows.sort(key=lambda r: -r[2])
    lines = ["name,calls,total_us,avg_us,percent"]
    for n, k, t, av in rows:
        short = n.split("(")[0].replace("void ", "")
        lines.append(f'"{short}",{k},{t:.3f},{av:.3f},{100 * t / tot:.2f}')
    out = "\n".join(lines) + "\n"
    if a.csv:
        open(a.csv, "w").write(out)
    print(out, end="")


if __name__ == "__main__":
    main()
