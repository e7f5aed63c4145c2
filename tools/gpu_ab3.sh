#!/bin/bash
# r06: probe3 (units per wave, store cache policies), calibrated read-request counters
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 180 tools/bin/bw_probe3 > $O/bw_probe3.txt 2>&1 || { cat $O/bw_probe3.txt; exit 1; }
cat $O/bw_probe3.txt
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
(cd /tmp && TMPDIR=/tmp timeout -s KILL 90 rocprofv3 --pmc $C -f csv -d $R/$O/pmc_rq_probe -o run -- $R/tools/bin/bw_probe3 quick) > $O/pmc_rq_probe.log 2>&1 || { tail -5 $O/pmc_rq_probe.log; exit 1; }
(cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc $C -f csv -d $R/$O/pmc_rq_main -o run -- python3 $R/bench.py --no-extra --no-cpu --no-batch-extra --steps 10 --warmup 2) > $O/pmc_rq_main.log 2>&1 || { tail -5 $O/pmc_rq_main.log; exit 1; }
find $O/pmc_rq_probe $O/pmc_rq_main -name "*counter_collection.csv" | head
