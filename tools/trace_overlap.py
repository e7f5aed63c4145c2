#!/usr/bin/env python3
"""Timeline of the last N kernel dispatches of a rocprofv3 --kernel-trace CSV
(start/end relative to the first shown, stream/queue id), and the busy time of
the union of their intervals -- how much two streams' kernels overlap.

usage: python tools/trace_overlap.py DIR [N]"""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    t0 = int(rows[0]["Start_Timestamp"])
    ivs = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        ivs.append((s, e))
        q = r.get("Stream_Id") or r.get("Queue_Id")
        print(f'{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:7.1f}  q{q}  {r["Kernel_Name"].split("(")[0][:50]}')
    busy, cur = 0, None
    for s, e in sorted(ivs):
        if cur is None or s > cur[1]:
            if cur:
                busy += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    busy += cur[1] - cur[0]
    span = max(e for _, e in ivs) - min(s for s, _ in ivs)
    print(f"span {span / 1e3:.1f} us, busy (union) {busy / 1e3:.1f} us, sum {sum(e - s for s, e in ivs) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
