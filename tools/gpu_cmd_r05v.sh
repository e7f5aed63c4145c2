set -o pipefail
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python tools/echo_prof.py 2 3000 > $O/echo_prof.jsonl 2> $O/echo_prof.err || { tail -5 $O/echo_prof.err; exit 1; }
cut -c1-700 $O/echo_prof.jsonl
