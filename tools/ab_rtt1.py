#!/usr/bin/env python3
"""A/B of the per-read host path between two builds of libfws_gpu.so: the
product library and a variant placed as flashws_amd/lib/<dir>/libfws_gpu.so
(the tools' RUNPATH yields to LD_LIBRARY_PATH). Per variant, order
alternated: tools/bin/lat_feed's session reads (4 KiB, resident decode, p50)
and the drop-in echo with one client (oracle/_ref/ws_dropin, 20,000 4 KiB
messages, RTT p50). One JSON line per run.

usage: python tools/ab_rtt1.py VARIANT_DIR [reps]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "oracle", "_ref", "ws_dropin")
LAT = os.path.join(ROOT, "tools", "bin", "lat_feed")


def env_for(variant):
    env = dict(os.environ)
    if variant:
        env["LD_LIBRARY_PATH"] = os.path.join(ROOT, "flashws_amd", "lib", variant) + ":" + env.get("LD_LIBRARY_PATH", "")
    return env


def lat(variant):
    r = subprocess.run([LAT, "3000"], capture_output=True, text=True, timeout=200, env=env_for(variant))
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-500:])
    out = {}
    for ln in r.stdout.splitlines():
        if not ln.startswith("{"):
            continue
        d = json.loads(ln)
        if d.get("workers") == 16 and not d.get("mux") and d.get("payload") in (0, 4096):
            out[f"{d['buffer']}_{d['payload']}"] = d["p50_us"]
    return out


def echo1(variant):
    env = env_for(variant)
    srv = subprocess.Popen([DROPIN, "server", "--port", "0", "--conns", "1", "--max-seconds", "60", "--gpu",
                            "--device", "0"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    line = srv.stdout.readline()
    if not line.startswith("listening"):
        srv.kill()
        raise RuntimeError(f"server did not start: {line!r}")
    port = int(line.split()[1])
    r = subprocess.run([DROPIN, "client", "--port", str(port), "--clients", "1", "--msgs", "20000", "--warmup", "500",
                        "--msg-len", "4096", "--max-seconds", "60"], capture_output=True, text=True, timeout=120)
    srv.communicate(timeout=60)
    c = json.loads(r.stdout.strip().splitlines()[-1])
    assert c.get("verified"), c
    return {"rtt_p50_us": c["rtt_us"]["p50"], "goodput_mbps": c["goodput_rx_tx_mbps"]}


def main():
    variant = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    for rep in range(reps):
        for v in ((None, variant) if rep % 2 == 0 else (variant, None)):
            rec = {"variant": v or "product", "rep": rep}
            rec.update(lat(v))
            rec.update(echo1(v))
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
