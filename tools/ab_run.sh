# ad-hoc pass (overwritten per experiment)
set -o pipefail
O=gpurun_out/ab10; mkdir -p $O
for r in 1 2; do
for l in gpu tx2 tx1; do
L=flashws_amd/lib/libfws_gpu_$l.so; [ $l = gpu ] && L=flashws_amd/lib/libfws_gpu.so
timeout -k 10 200 python tools/tune_tx.py --lib $L >> $O/tx.txt 2>&1 || exit 1
done; done
grep -h '^{' $O/tx.txt
ROUND=r03s3 bash tools/gpu_round.sh pmc pmc_decode
