#!/usr/bin/env python3
"""Per-dispatch timeline of the last decode call(s) in a rocprofv3 kernel trace
(--kernel-trace -f csv): start / end in microseconds from the first dispatch
shown, duration, queue and stream ids, kernel name. Shows whether the decode
segments' kernels overlap.

usage: python tools/kernel_timeline.py RUN_kernel_trace.csv [last_n_dispatches]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    t0 = int(rows[0]["Start_Timestamp"])
    for r in rows:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print(f"{s / 1e3:9.2f} {e / 1e3:9.2f} {(e - s) / 1e3:8.2f}  q{r.get('Queue_Id', '?'):>3} "
              f"s{r.get('Stream_Id', '?'):>3}  {r['Kernel_Name'][:60]}")


if __name__ == "__main__":
    main()
