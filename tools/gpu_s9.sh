set -e
mkdir -p gpurun_out/s9
timeout -k 10 300 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_onelaunch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s9/tests.log 2>&1
timeout -k 10 400 python -u tools/ab_tx.py 40 plan,so5,so8,sod5,sod6 > gpurun_out/s9/ab_tx.jsonl 2>gpurun_out/s9/ab_tx.err
timeout -k 10 300 python -u tools/ab_c4.py 5 50 -1:512:4,-2:512:4,2:512:4 > gpurun_out/s9/ab_c4.jsonl 2>gpurun_out/s9/ab_c4.err
echo done
