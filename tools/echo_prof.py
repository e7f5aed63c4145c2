#!/usr/bin/env python3
"""Where a step of the batched drop-in echo server goes (oracle/_ref/ws_dropin
with GpuRxHook::EnableBatched, FWS_HOOK_PROF=1): per case one JSON line with
the client's goodput and RTT, each process's CPU time against the wall time
(os.wait4 rusage: a process near 1.0 CPU-s per wall-s is the bottleneck of the
closed loop), and the server hook's step profile (FWS_HOOK_CHUNK: reads per submitted chunk) -- steps, flushes, reads,
the loop's own part of the steps (epoll + recv), the mux rounds and the event
dispatch (application callbacks: the echo sends), per step.

usage: python tools/echo_prof.py [reps] [msgs_per_client] [chunk|prefetch]"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "oracle", "_ref", "ws_dropin")


def wait_rusage(p):
    _, status, ru = os.wait4(p.pid, 0)
    p.returncode = os.waitstatus_to_exitcode(status)
    return ru.ru_utime + ru.ru_stime


def run(mode, clients, msgs, persistent, chunk=None, extra_env=None):
    env = dict(os.environ, FWS_HOOK_PROF="1", **(extra_env or {}))
    if chunk is not None:
        env["FWS_HOOK_CHUNK"] = str(chunk)       # reads per submitted chunk (0: one batch per step)
    args = [DROPIN, "server", "--port", "0", "--conns", str(clients), "--max-seconds", "60"]
    if mode != "reference":
        args += ["--gpu-batch" if mode == "batched" else "--gpu", "--device", "0", "--persistent", str(persistent)]
    srv = subprocess.Popen(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    line = srv.stdout.readline()
    if not line.startswith("listening"):
        srv.kill()
        raise RuntimeError(f"server did not start: {line!r}")
    port = int(line.split()[1])
    t0 = time.monotonic()
    cli = subprocess.Popen([DROPIN, "client", "--port", str(port), "--clients", str(clients), "--msgs", str(msgs),
                            "--warmup", "200", "--msg-len", "4096", "--max-seconds", "60"],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    cout = cli.stdout.read()
    ccpu = wait_rusage(cli)
    wall = time.monotonic() - t0
    sout = srv.stdout.read()
    scpu = wait_rusage(srv)
    if srv.returncode != 0 or cli.returncode != 0:
        raise RuntimeError(f"rc server {srv.returncode} client {cli.returncode}: {srv.stderr.read()[-300:]}")
    c = json.loads(cout.strip().splitlines()[-1])
    assert c.get("verified"), c
    rec = {"mode": mode, "clients": clients, "persistent": persistent, "chunk": chunk, "msgs_per_client": msgs,
           "goodput_rx_tx_mbps": c.get("goodput_rx_tx_mbps"), "rtt_us": c.get("rtt_us"),
           "wall_s": round(wall, 3), "client_cpu_per_wall": round(ccpu / wall, 3),
           "server_cpu_per_wall": round(scpu / wall, 3)}
    for ln in sout.strip().splitlines():
        if ln.startswith('{"hook_prof"'):
            hp = json.loads(ln)["hook_prof"]
            st = max(hp["steps"], 1)
            rec["hook_prof"] = hp
            rec["per_step_us"] = {k: round(hp[k] / st, 2) for k in ("loop_us", "mux_us", "dispatch_us", "step_end_us")}
            rec["reads_per_flush"] = round(hp["reads"] / max(hp["flushes"], 1), 1)
    return rec


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    msgs = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
    which = sys.argv[3] if len(sys.argv) > 3 else "chunk"
    if which == "prefetch":      # the dispatch's prefetch of the next read (FWS_HOOK_PREFETCH)
        cases = [("reference", 64, 0, None, None)] + \
                [("batched", c, 16, 16, {"FWS_HOOK_PREFETCH": p}) for c in (64, 8) for p in ("1", "0")]
    else:
        cases = [("reference", 64, 0, None, None)] + [("batched", 64, 16, c, None) for c in (0, 8, 16, 32)] + \
                [("reference", 8, 0, None, None), ("batched", 8, 16, 0, None), ("batched", 8, 16, 4, None)]
    for rep in range(reps):
        for mode, clients, pers, chunk, env in (cases if rep % 2 == 0 else cases[::-1]):
            rec = run(mode, clients, msgs if clients > 8 else 4 * msgs, pers, chunk, env)
            rec["rep"] = rep
            if env:
                rec["env"] = env
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
