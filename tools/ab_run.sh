# ad-hoc pass (overwritten per experiment)
set -o pipefail
O=gpurun_out/ab5; mkdir -p $O
for r in 1 2 3; do
for l in gpu raw; do
L=flashws_amd/lib/libfws_gpu_$l.so; [ $l = gpu ] && L=flashws_amd/lib/libfws_gpu.so
timeout -k 10 120 python tools/scan_ablation.py --lib $L 50 >> $O/scan.txt 2>&1 || exit 1
timeout -k 10 200 python tools/time_decode.py 40 --lib $L >> $O/dec.txt 2>&1 || exit 1
done; done
grep '^{' $O/scan.txt; grep '^{' $O/dec.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
