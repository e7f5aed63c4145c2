set -o pipefail
O=gpurun_out/r05; mkdir -p $O
bash tools/gpu_round.sh utf8tests || exit 1
timeout -k 10 200 python tools/ab_c5d.py > $O/ab_c5d_b.jsonl 2>> $O/ab_c5d.err || exit 1
cat $O/ab_c5d_b.jsonl
