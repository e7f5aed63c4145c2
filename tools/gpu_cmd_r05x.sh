set -o pipefail
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 500 python tools/ab_rtt1.py ab_nopf 2 > $O/ab_rtt1_pf.jsonl 2> $O/ab_rtt1.err || { tail -5 $O/ab_rtt1.err; exit 1; }
cat $O/ab_rtt1_pf.jsonl
