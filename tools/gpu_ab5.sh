#!/bin/bash
# r06: sorted unmask workgroup order (plain vs XCD runs): parity, interleaved timing, sized read requests
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python -u -m pytest tests/test_gpu_unmask.py -x -q --timeout 120 --timeout-method thread -k "sorted" > $O/t_sorted5.log 2>&1 || { tail -30 $O/t_sorted5.log; exit 1; }
tail -1 $O/t_sorted5.log
timeout -k 10 300 python -u tools/ab_sorted.py 9 200 0,3 > $O/ab_sorted5.jsonl 2>&1 || { tail -20 $O/ab_sorted5.jsonl; exit 1; }
tail -2 $O/ab_sorted5.jsonl
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
(cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc $C -f csv -d $R/$O/pmc5_rq -o run -- python3 $R/tools/ab_sorted.py 1 20 0,3) > $O/pmc5_rq.log 2>&1 || { tail -5 $O/pmc5_rq.log; exit 1; }
(cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/$O/pmc5_wr -o run -- python3 $R/tools/ab_sorted.py 1 20 0,3) > $O/pmc5_wr.log 2>&1 || { tail -5 $O/pmc5_wr.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, statistics
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in ("gpurun_out/r06/pmc5_rq", "gpurun_out/r06/pmc5_wr"):
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_unmask_sorted" in r["Kernel_Name"]:
                agg[r["Kernel_Name"][:50]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    m = {c: statistics.median(x) for c, x in v.items()}
    rd = 32 * m.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * m.get("TCC_EA0_RDREQ_64B_sum", 0) + 128 * m.get("TCC_EA0_RDREQ_128B_sum", 0)
    wr = m.get("WRITE_SIZE", 0) * 1024
    print(k, {c: m[c] for c in m}, "read", rd, "write", wr, "traffic/alg", round((rd + wr) / 537395200, 5))
PY
