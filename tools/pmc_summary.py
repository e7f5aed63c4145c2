#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from rocprofv3 PMC passes.

rocprofv3 cannot collect FETCH_SIZE (3 TCC slots) and WRITE_SIZE (2) in one
pass on gfx950, so they come from two runs of the same command:

  rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/pmc_fetch -- python3 bench.py ...
  rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/pmc_write -- python3 bench.py ...

Both counters are in KiB. Per MI355X_MICROARCH.md (HBM section), FETCH_SIZE
reports exactly half the bytes of a 16-B-per-lane streaming read on gfx950,
so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.

r06: with --rdreq DIR (a third pass, --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum) the read bytes are counted per
request size instead: 32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B.
FETCH_SIZE's expression counts every request that is not 32 B as 64 B
(its 128-B term is TCC_BUBBLE, zero on gfx950), which is where the "half" of a
streaming read comes from; the doubling then also doubles the 64-B requests
(scalar descriptor loads). Calibration (profiles/r06/pmc_rq_calibration.json):
on the plain in-place XOR probe the sized count is the wire's 268,959,744 B
plus 12 KiB.

usage: python tools/pmc_summary.py --fetch DIR --write DIR --kernel k_unmask_fast \
           --alg-bytes 537395200 --out profiles/pmc_unmask.json
"""
import argparse
import csv
import glob
import json
import statistics


def per_dispatch(d, counter, kernel):
    vals = {}
    files = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter or kernel not in row.get("Kernel_Name", ""):
                    continue
                key = (f, row.get("Dispatch_Id"))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} under {d}")
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--rdreq", default="", help="a pass of the four TCC_EA0_RDREQ*_sum counters: sized read bytes")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--alg-bytes", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--source", default="flashws_amd/csrc/unmask_kernels.hip",
                    help="the kernel's source file; its sha256 is recorded so bench.py can tell a stale summary")
    a = ap.parse_args()
    import datetime
    import hashlib
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, a.source), "rb") as fh:
        src_sha = hashlib.sha256(fh.read()).hexdigest()[:16]
    try:
        commit = subprocess.run(["git", "-C", root, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                text=True).stdout.strip() or None
    except OSError:
        commit = None
    f = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    w = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    fk, wk = statistics.median(f), statistics.median(w)
    read_b = 2.0 * fk * 1024.0          # gfx950: FETCH_SIZE counts half of a wide streaming read
    write_b = wk * 1024.0
    sized = None
    if a.rdreq:
        n32 = statistics.median(per_dispatch(a.rdreq, "TCC_EA0_RDREQ_32B_sum", a.kernel))
        n64 = statistics.median(per_dispatch(a.rdreq, "TCC_EA0_RDREQ_64B_sum", a.kernel))
        n128 = statistics.median(per_dispatch(a.rdreq, "TCC_EA0_RDREQ_128B_sum", a.kernel))
        nall = statistics.median(per_dispatch(a.rdreq, "TCC_EA0_RDREQ_sum", a.kernel))
        sized = {"RDREQ": nall, "RDREQ_32B": n32, "RDREQ_64B": n64, "RDREQ_128B": n128,
                 "read_bytes": round(32 * n32 + 64 * n64 + 128 * n128),
                 "fetch_x2_read_bytes": round(read_b)}
        read_b = float(sized["read_bytes"])
    out = {
        "kernel": a.kernel,
        "dispatches": {"fetch_pass": len(f), "write_pass": len(w)},
        "FETCH_SIZE_KiB_median": fk,
        "WRITE_SIZE_KiB_median": wk,
        "read_bytes_per_launch": round(read_b),
        "write_bytes_per_launch": round(write_b),
        "hbm_bytes_per_launch": round(read_b + write_b),
        "alg_bytes_per_launch": a.alg_bytes,
        "traffic_over_alg": round((read_b + write_b) / a.alg_bytes, 4),
        "correction": ("read = 32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B (sized requests; "
                       "2 x FETCH_SIZE kept as fetch_x2_read_bytes)" if sized else
                       "read = 2 x FETCH_SIZE (gfx950 half-count of 16-B/lane streaming reads, "
                       "MI355X_MICROARCH.md HBM)") + "; write = WRITE_SIZE; KiB = 1024 B",
        "sized_reads": sized,
        "kernel_source": a.source,
        "kernel_source_sha16": src_sha,
        "commit": commit,
        "measured": datetime.date.today().isoformat(),
    }
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
