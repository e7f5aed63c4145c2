# ad-hoc pass (overwritten per experiment)
set -o pipefail
O=gpurun_out/ab14; mkdir -p $O
for r in 1 2 3; do
for l in gpu g8; do
L=flashws_amd/lib/libfws_gpu_$l.so; [ $l = gpu ] && L=flashws_amd/lib/libfws_gpu.so
timeout -k 10 200 python tools/time_c4.py --lib $L >> $O/c4.txt 2>&1 || exit 1
done; done
grep -h '^{' $O/c4.txt
