# round-4 A/B pass: decode + one-launch parity on the product build, then the
# landing-lookup A/B (tools/time_decode.py, product vs libfws_gpu_land0.so)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_onelaunch.py tests/test_gpu_engine.py > gpurun_out/p4_tests.log 2>&1 &&
timeout -k 10 150 python -u tools/time_decode.py 20 > gpurun_out/td4.jsonl 2>&1 &&
timeout -k 10 150 python -u tools/time_decode.py 20 --lib flashws_amd/lib/libfws_gpu_land0.so >> gpurun_out/td4.jsonl 2>&1 &&
timeout -k 10 150 python -u tools/time_decode.py 20 >> gpurun_out/td4.jsonl 2>&1 &&
timeout -k 10 150 python -u tools/time_decode.py 20 --lib flashws_amd/lib/libfws_gpu_land0.so >> gpurun_out/td4.jsonl 2>&1 &&
timeout -k 10 150 python -u tools/ab_gather.py 30 > gpurun_out/ab_gather4.jsonl 2>&1
