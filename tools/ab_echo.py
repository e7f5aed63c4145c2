#!/usr/bin/env python3
"""A/B of the drop-in echo server (oracle/_ref/ws_dropin: the reference's FLoop
+ WSServerSocket<false> with fws_amd::GpuRxHook) with the per-read launch path
and with the persistent receive decode (--persistent N: fws_gpu_ctx_set_rx_persistent),
4 KiB masked BIN frames, window 1, every byte checked by the client; one JSON
line per (mode, clients, repetition): goodput rx+tx Mbit/s, RTT p50/p99, GPU
reads and batches, the server's zero-copy slots.

usage: python tools/ab_echo.py [reps]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "oracle", "_ref", "ws_dropin")


def run(mode, clients, msgs, persistent):
    args = [DROPIN, "server", "--port", "0", "--conns", str(clients), "--max-seconds", "60"]
    if mode != "reference":
        args += ["--gpu-batch" if mode == "batched" else "--gpu", "--device", "0"]
        args += ["--persistent", str(persistent)]        # (0: a launch per read)
    p = subprocess.Popen(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    if not line.startswith("listening"):
        p.kill()
        raise RuntimeError(f"server did not start: {line!r} {p.stderr.read()[-500:]}")
    port = int(line.split()[1])
    r = subprocess.run([DROPIN, "client", "--port", str(port), "--clients", str(clients), "--msgs", str(msgs),
                        "--warmup", "200", "--msg-len", "4096", "--max-seconds", "60"],
                       capture_output=True, text=True, timeout=120)
    out, err = p.communicate(timeout=60)
    if p.returncode != 0 or r.returncode != 0:
        raise RuntimeError(f"rc server {p.returncode} client {r.returncode}: {err[-400:]} {r.stderr[-400:]}")
    st = json.loads(out.strip().splitlines()[-1])
    cli = json.loads(r.stdout.strip().splitlines()[-1])
    assert cli.get("verified"), cli
    return {"goodput_rx_tx_mbps": cli.get("goodput_rx_tx_mbps"), "rtt_us": cli.get("rtt_us"),
            "gpu_reads": st.get("gpu_reads"), "gpu_batches": st.get("gpu_batches"), "zc_slots": st.get("zc_slots")}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    cases = [("reference", 1, 20000, 0), ("per_read", 1, 20000, 0), ("per_read", 1, 20000, 4),
             ("per_read", 1, 20000, 16), ("reference", 64, 500, 0), ("batched", 64, 500, 0),
             ("batched", 64, 500, 32), ("batched", 64, 500, 64), ("reference", 8, 4000, 0),
             ("batched", 8, 4000, 0), ("batched", 8, 4000, 16)]
    for rep in range(reps):
        for mode, clients, msgs, pers in (cases if rep % 2 == 0 else cases[::-1]):
            rec = run(mode, clients, msgs, pers)
            rec.update({"mode": mode, "clients": clients, "persistent": pers, "rep": rep})
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
