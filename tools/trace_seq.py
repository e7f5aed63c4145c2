#!/usr/bin/env python3
"""Print a rocprofv3 kernel-trace CSV as runs of (kernel, count, median us)."""
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
runs = []
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if runs and runs[-1][0] == name:
        runs[-1][1].append(dur)
    else:
        runs.append((name, [dur]))
for name, ds in runs:
    print(f"{name:42s} x{len(ds):4d}  median {np.median(ds):8.2f} us  min {min(ds):8.2f}")
