# ad-hoc pass (overwritten per experiment)
set -o pipefail
O=gpurun_out/ab13; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread > $O/tx_tests.log 2>&1 || { tail -30 $O/tx_tests.log; exit 1; }
tail -1 $O/tx_tests.log
for r in 1 2 3; do
for l in gpu sw6; do
L=flashws_amd/lib/libfws_gpu_$l.so; [ $l = gpu ] && L=flashws_amd/lib/libfws_gpu.so
timeout -k 10 200 python tools/time_decode.py 40 --lib $L >> $O/dec_$l.txt 2>&1 || exit 1
done; done
grep -h '^{' $O/dec_gpu.txt $O/dec_sw6.txt | cut -c1-230
