#!/bin/bash
# r06 A/B: sorted unmask kernels (parity first, then interleaved timing + the XOR probe),
# then the service queue / mux tests
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_unmask.py -x -q --timeout 120 --timeout-method thread -k "sorted" > $O/t_sorted.log 2>&1 || { tail -30 $O/t_sorted.log; exit 1; }
tail -2 $O/t_sorted.log
timeout -k 10 300 python -u tools/ab_sorted.py 9 200 0,2 > $O/ab_sorted.jsonl 2>&1 || { tail -20 $O/ab_sorted.jsonl; exit 1; }
tail -2 $O/ab_sorted.jsonl
timeout -k 10 120 tools/bin/bw_probe2 > $O/bw_probe2.txt 2>&1 || exit 1
head -3 $O/bw_probe2.txt
timeout -k 10 120 tools/bin/bw_probe3 > $O/bw_probe3.txt 2>&1 || exit 1
cat $O/bw_probe3.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_service.py -x -v -s --timeout 120 --timeout-method thread > $O/t_service.log 2>&1 || { tail -30 $O/t_service.log; exit 1; }
grep "queue=" $O/t_service.log; tail -2 $O/t_service.log
