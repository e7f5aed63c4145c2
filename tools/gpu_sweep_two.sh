mkdir -p gpurun_out
rm -f gpurun_out/sweep_two.txt
for c in c3 c2; do
  timeout -k 10 240 python -u tools/sweep_two.py $c 30 >> gpurun_out/sweep_two.txt 2>&1 || { echo "FAIL $c $?" >> gpurun_out/sweep_two.txt; break; }
done
cat gpurun_out/sweep_two.txt
