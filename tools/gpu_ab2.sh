#!/bin/bash
# r06: service queue modes, probe3, the box's TCC request counters
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 120 tools/bin/bw_probe3 > $O/bw_probe3.txt 2>&1 || { cat $O/bw_probe3.txt; exit 1; }
cat $O/bw_probe3.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_service.py -v -s --timeout 120 --timeout-method thread -k "beside or persistent_off" > $O/t_service2.log 2>&1; rc=$?
grep "queue=\|PASSED\|FAILED" $O/t_service2.log; tail -2 $O/t_service2.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
(cd /tmp && timeout -k 10 60 rocprofv3 --list-avail) > $O/counters.txt 2>&1 || true
grep -o "TCC_EA0_RD[A-Z0-9_]*\|TCC_EA_RD[A-Z0-9_]*\|TCC_BUBBLE[A-Z0-9_]*\|TCC_EA0_WR[A-Z0-9_]*" $O/counters.txt | sort -u | head -40
