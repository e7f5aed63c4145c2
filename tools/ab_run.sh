# ad-hoc pass (overwritten per experiment)
set -o pipefail
O=gpurun_out/ab9; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
for l in gpu base; do
L=flashws_amd/lib/libfws_gpu_$l.so; [ $l = gpu ] && L=flashws_amd/lib/libfws_gpu.so
timeout -k 10 120 python tools/scan_ablation.py --lib $L 50 >> $O/scan_$l.txt 2>&1 || exit 1
timeout -k 10 200 python tools/time_decode.py 40 --lib $L >> $O/dec_$l.txt 2>&1 || exit 1
done; done
grep -h '^{' $O/scan_gpu.txt $O/scan_base.txt $O/dec_gpu.txt $O/dec_base.txt | cut -c1-200
