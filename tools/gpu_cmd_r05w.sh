set -o pipefail
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mux.py tests/test_gpu_service.py tests/test_gpu_dropin.py > $O/t_mux_dropin.log 2>&1 || { tail -30 $O/t_mux_dropin.log; exit 1; }
tail -3 $O/t_mux_dropin.log
timeout -k 10 400 python tools/echo_prof.py 2 3000 > $O/echo_prof_chunk.jsonl 2> $O/echo_prof.err || { tail -5 $O/echo_prof.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r05/echo_prof_chunk.jsonl"):
    d=json.loads(l); print(d["mode"], d["clients"], d.get("chunk"), d["goodput_rx_tx_mbps"], d["rtt_us"]["p50"], d.get("per_step_us"), d.get("reads_per_flush"), d["server_cpu_per_wall"])
PY
