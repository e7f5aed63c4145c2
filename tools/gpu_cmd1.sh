# round-4 GPU pass 1: RTT probes, decode + one-launch tests, A/B of the lean
# k_scan node parse, drop-in tests, bench (every step under its own limit)
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step rtt && timeout -k 10 120 tools/bin/rtt_probe default > $O/rtt_default.jsonl 2>&1 && \
timeout -k 10 120 tools/bin/rtt_probe spin > $O/rtt_spin.jsonl 2>&1 && \
step tests && timeout -k 10 700 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_onelaunch.py tests/test_gpu_inplace.py tests/test_gpu_session.py tests/test_gpu_mux.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $O/dec_tests.log 2>&1 && tail -2 $O/dec_tests.log && \
step ab && for i in 1 2; do
  timeout -k 10 120 python tools/scan_ablation.py --lib flashws_amd/lib/libfws_gpu_nolean.so 50 >> $O/scan_ab.jsonl 2>/dev/null &&
  timeout -k 10 120 python tools/scan_ablation.py --lib flashws_amd/lib/libfws_gpu.so 50 >> $O/scan_ab.jsonl 2>/dev/null &&
  timeout -k 10 120 python tools/time_decode.py 20 --lib flashws_amd/lib/libfws_gpu_nolean.so >> $O/dec_ab.jsonl 2>/dev/null &&
  timeout -k 10 120 python tools/time_decode.py 20 --lib flashws_amd/lib/libfws_gpu.so >> $O/dec_ab.jsonl 2>/dev/null || exit 1
done && cat $O/scan_ab.jsonl $O/dec_ab.jsonl && \
step emit_ab && timeout -k 10 200 python tools/ab_emit_path.py 20 > $O/emit_path_ab.jsonl 2>&1 && cat $O/emit_path_ab.jsonl && \
ROUND=r04 bash tools/gpu_round.sh dropin bench
