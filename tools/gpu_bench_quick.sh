# default bench line without the CPU baseline legs, and the decode two-in-flight records
timeout -k 10 400 python bench.py --no-cpu --no-batch-extra > gpurun_out/bench_nocpu.json 2> gpurun_out/bench_nocpu.err || { tail -5 gpurun_out/bench_nocpu.err; exit 1; }
python3 - <<'PY'
import json
b = json.loads(open("gpurun_out/bench_nocpu.json").read().strip().splitlines()[-1])
print(b["value"], b["roofline"]["frac"])
for k in ("C2_stream_decode", "C3_mixed_stream_decode"):
    print(k, b["extra"][k]["ms_per_step"], b["extra"][k]["two_in_flight"])
PY
