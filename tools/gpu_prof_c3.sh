mkdir -p gpurun_out
timeout -k 10 100 python -u tools/prof_fused.py c3 1 > gpurun_out/prof_c3.txt 2>&1; echo "rc=$?" >> gpurun_out/prof_c3.txt
cat gpurun_out/prof_c3.txt
