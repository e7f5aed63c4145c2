# round-4 GPU pass 1: correctness of this round's changes (decode, one-launch
# gather, in-place host reads, host-polled completion flags, drop-in), the RTT
# probe (every step under its own limit)
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests && timeout -k 10 900 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_onelaunch.py tests/test_gpu_inplace.py tests/test_gpu_session.py tests/test_gpu_mux.py tests/test_gpu_echo.py tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread > $O/tests_p1.log 2>&1 && tail -2 $O/tests_p1.log && \
step rtt && timeout -k 10 100 tools/bin/rtt_probe default > $O/rtt_flag.jsonl 2>&1 && cat $O/rtt_flag.jsonl && echo done1
