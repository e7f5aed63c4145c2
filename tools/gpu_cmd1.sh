# round-4 GPU pass 1: correctness of this round's changes (decode incl. the fused
# path resolve, one-launch gather, in-place host reads), RTT probes, A/B of the
# lean k_scan node parse and of k_emit_path (every step under its own limit)
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests && timeout -k 10 840 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_onelaunch.py tests/test_gpu_inplace.py tests/test_gpu_session.py tests/test_gpu_mux.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $O/dec_tests.log 2>&1 && tail -2 $O/dec_tests.log && \
step rtt && timeout -k 10 100 tools/bin/rtt_probe default > $O/rtt_default.jsonl 2>&1 && \
timeout -k 10 100 tools/bin/rtt_probe spin > $O/rtt_spin.jsonl 2>&1 && \
step emit_ab && timeout -k 10 150 python tools/ab_emit_path.py 20 > $O/emit_path_ab.jsonl 2>&1 && \
step scan_ab && for i in 1 2; do
  timeout -k 10 60 python tools/scan_ablation.py --lib flashws_amd/lib/libfws_gpu_nolean.so 50 >> $O/scan_ab.jsonl 2>/dev/null &&
  timeout -k 10 60 python tools/scan_ablation.py --lib flashws_amd/lib/libfws_gpu.so 50 >> $O/scan_ab.jsonl 2>/dev/null || exit 1
done && echo done1
