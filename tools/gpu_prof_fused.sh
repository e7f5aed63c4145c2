# k_fused phase clocks per super tile (tools/prof_fused.py)
mkdir -p gpurun_out
for c in c2 c3; do
  timeout -k 10 120 python -u tools/prof_fused.py $c 2 >> gpurun_out/prof_fused.txt 2>&1 || { echo "FAIL $c $?" >> gpurun_out/prof_fused.txt; break; }
done
cat gpurun_out/prof_fused.txt
