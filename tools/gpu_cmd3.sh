mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_onelaunch.py tests/test_gpu_engine.py > gpurun_out/ol.log 2>&1 &&
FWS_LIB_VARIANT=sel timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode.py > gpurun_out/sel_tests.log 2>&1 &&
timeout -k 10 150 python -u tools/time_decode.py 20 > gpurun_out/td.jsonl 2>&1 &&
timeout -k 10 150 python -u tools/time_decode.py 20 --lib flashws_amd/lib/libfws_gpu_sel.so >> gpurun_out/td.jsonl 2>&1 &&
timeout -k 10 150 python -u tools/time_decode.py 20 >> gpurun_out/td.jsonl 2>&1 &&
timeout -k 10 150 python -u tools/time_decode.py 20 --lib flashws_amd/lib/libfws_gpu_sel.so >> gpurun_out/td.jsonl 2>&1 &&
timeout -k 10 150 python -u tools/ab_gather.py 30 > gpurun_out/ab_gather.jsonl 2>&1 &&
timeout -k 10 150 python -u tools/ab_gather.py 30 --lib flashws_amd/lib/libfws_gpu_w6.so >> gpurun_out/ab_gather.jsonl 2>&1 &&
timeout -k 10 150 python -u tools/ab_gather.py 30 >> gpurun_out/ab_gather.jsonl 2>&1 &&
timeout -k 10 200 python -u tools/prof_merge_trace.py > gpurun_out/merge_trace.json 2> gpurun_out/merge_trace.err
