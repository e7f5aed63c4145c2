set -o pipefail
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 500 python tools/echo_prof.py 3 3000 prefetch > $O/echo_prof_prefetch.jsonl 2> $O/echo_prof.err || { tail -5 $O/echo_prof.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r05/echo_prof_prefetch.jsonl"):
    d=json.loads(l); print(d["mode"], d["clients"], d.get("env"), d["goodput_rx_tx_mbps"], d["rtt_us"]["p50"], d.get("per_step_us"), d.get("reads_per_flush"))
PY
