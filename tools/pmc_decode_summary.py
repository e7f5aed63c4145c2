#!/usr/bin/env python3
"""Per-kernel and per-decode HBM traffic and SQ counters of one stream-decode
config from rocprofv3 PMC passes (tools/gpu_round.sh pmc_decode / sq_decode:
`rocprofv3 --pmc FETCH_SIZE`, `--pmc WRITE_SIZE`, `--pmc SQ_...` of
tools/run_decode.py c3).

Traffic per dispatch = 2 x FETCH_SIZE + WRITE_SIZE (KiB; the gfx950 half-count
of 16-B-per-lane streaming reads, MI355X_MICROARCH.md HBM section), median over
dispatches; a decode is one dispatch of each k_* kernel. SQ counters are summed
per dispatch (every SE / XCD instance), median over dispatches.

usage: python tools/pmc_decode_summary.py --fetch DIR --write DIR --sq DIR \
           --alg-bytes 537147460 --tiles 131196 --out profiles/r05/pmc_decode_c3.json
"""
import argparse
import csv
import glob
import json
import statistics


def per_kernel(d, counters):
    """{kernel: {counter: [per-dispatch values]}} from counter_collection CSVs under d"""
    acc = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                c = row.get("Counter_Name")
                if c not in counters:
                    continue
                k = row.get("Kernel_Name", "")
                if "fwsk::" not in k:
                    continue
                name = k.split("(")[0].replace("void ", "").strip()
                key = (f, row.get("Dispatch_Id"))
                acc.setdefault(name, {}).setdefault(c, {})
                acc[name][c][key] = acc[name][c].get(key, 0.0) + float(row["Counter_Value"])
    return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--sq")
    ap.add_argument("--alg-bytes", type=int, required=True)
    ap.add_argument("--tiles", type=int, default=0)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch = per_kernel(a.fetch, {"FETCH_SIZE"})
    write = per_kernel(a.write, {"WRITE_SIZE"})
    kernels = {}
    total = 0.0
    for k in sorted(set(fetch) | set(write)):
        fr = statistics.median(fetch.get(k, {}).get("FETCH_SIZE", [0.0])) * 1024 * 2
        wr = statistics.median(write.get(k, {}).get("WRITE_SIZE", [0.0])) * 1024
        kernels[k] = {"read_bytes": int(fr), "write_bytes": int(wr), "hbm_bytes": int(fr + wr),
                      "dispatches": len(fetch.get(k, {}).get("FETCH_SIZE", []))}
        total += fr + wr
    out = {"kernels": kernels, "hbm_bytes_per_decode": int(total), "alg_bytes_per_decode": a.alg_bytes,
           "traffic_over_alg": round(total / a.alg_bytes, 4),
           "correction": "read = 2 x FETCH_SIZE (gfx950 half-count, MI355X_MICROARCH.md HBM); write = WRITE_SIZE"}
    if a.sq:
        names = {"SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
                 "SQ_WAIT_INST_ANY", "SQ_INSTS_VMEM"}
        sq = per_kernel(a.sq, names)
        out["sq"] = {}
        for k, cs in sorted(sq.items()):
            m = {c: statistics.median(v) for c, v in cs.items()}
            rec = {c: int(v) for c, v in m.items()}
            if m.get("SQ_WAVE_CYCLES"):
                rec["wait_inst_any_over_wave_cycles"] = round(m.get("SQ_WAIT_INST_ANY", 0) / m["SQ_WAVE_CYCLES"], 3)
            if a.tiles and "k_scan" in k:
                rec["valu_per_tile"] = round(m.get("SQ_INSTS_VALU", 0) / a.tiles, 1)
                rec["salu_per_tile"] = round(m.get("SQ_INSTS_SALU", 0) / a.tiles, 1)
            out["sq"][k] = rec
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({"hbm_bytes_per_decode": out["hbm_bytes_per_decode"], "traffic_over_alg": out["traffic_over_alg"],
                      "k_scan_sq": {k: v for k, v in out.get("sq", {}).items() if "k_scan" in k}}))


if __name__ == "__main__":
    main()
