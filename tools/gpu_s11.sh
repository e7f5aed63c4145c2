set -e
mkdir -p gpurun_out/s11
FWS_TEST_TX_SR=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_tx.py -x -q -k "plan_sr" --timeout 120 --timeout-method thread > gpurun_out/s11/tx_sr_tests.log 2>&1
timeout -k 10 300 python -u tools/ab_tx.py 40 plan,sr5,sr8 > gpurun_out/s11/ab_tx.jsonl 2>gpurun_out/s11/ab_tx.err
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py -x -v --timeout 120 --timeout-method thread > gpurun_out/s11/dropin.log 2>&1
timeout -k 10 300 python -u bench.py --only c1 --no-cpu --no-batch-extra --steps 20 --warmup 5 > gpurun_out/s11/bench_c1.json 2> gpurun_out/s11/bench_c1.err
echo done
