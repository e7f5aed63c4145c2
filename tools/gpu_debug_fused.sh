mkdir -p gpurun_out
rm -f gpurun_out/debug_fused.txt
for i in 1 2 3 4; do
  echo "== process $i" >> gpurun_out/debug_fused.txt
  timeout -k 5 50 python -u tools/debug_fused.py c3 2 >> gpurun_out/debug_fused.txt 2>&1
  rc=$?
  echo "rc=$rc" >> gpurun_out/debug_fused.txt
  [ $rc -eq 0 ] || break
done
cat gpurun_out/debug_fused.txt
