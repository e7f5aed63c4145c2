# fused decode iteration: fused-mode decode tests, then phase clocks (C2, C3)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py -k "fused" -x -q --timeout 120 --timeout-method thread > gpurun_out/fused_tests.log 2>&1
rc=$?
tail -3 gpurun_out/fused_tests.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/prof_fused.txt
for c in c2 c3 dense64; do
  timeout -k 10 120 python -u tools/prof_fused.py $c 2 >> gpurun_out/prof_fused.txt 2>&1 || { echo "FAIL $c $?" >> gpurun_out/prof_fused.txt; break; }
done
cat gpurun_out/prof_fused.txt
