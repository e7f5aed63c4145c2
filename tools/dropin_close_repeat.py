#!/usr/bin/env python3
"""Repeat one drop-in load case (tests/test_gpu_dropin.py::test_dropin_reference_client_load)
N times, sequentially, and report every server close log that is not [1000, "bye"] per
connection, with the server's counters. One server + one client process at a time.

usage: python tools/dropin_close_repeat.py N clients msg_len tls(0|1) chunk(none|flush|K)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "oracle", "_ref", "ws_dropin")
TLS_ARGS = ["--tls", "--cert", os.path.join(ROOT, "tests", "tls", "server.crt"),
            "--key", os.path.join(ROOT, "tests", "tls", "server.key")]


def one(clients, msg_len, tls, env):
    args = [DROPIN, "server", "--conns", str(clients), "--max-seconds", "60", "--gpu-batch"] + (TLS_ARGS if tls else [])
    p = subprocess.Popen(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    port = int(p.stdout.readline().split()[1])
    r = subprocess.run([DROPIN, "client", "--port", str(port), "--clients", str(clients), "--msgs", "600",
                        "--warmup", "20", "--msg-len", str(msg_len), "--ping-every", "50", "--max-seconds", "60"]
                       + (["--tls"] if tls else []), capture_output=True, text=True, timeout=90)
    out, err = p.communicate(timeout=60)
    st = json.loads(out.strip().splitlines()[-1])
    cli = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {"rc": r.returncode}
    return st, cli


def main():
    n, clients, msg_len, tls, chunk = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4] == "1", sys.argv[5]
    env = dict(os.environ)
    if chunk == "flush":
        env["FWS_HOOK_DEFER"] = "0"
    elif chunk != "none":
        env["FWS_HOOK_CHUNK"] = chunk
    bad = 0
    for i in range(n):
        st, cli = one(clients, msg_len, tls, env)
        ok = all(c == [1000, b"bye".hex()] for c in st["close_log_hex"][:clients]) and cli.get("verified") is True
        if not ok:
            bad += 1
            print(json.dumps({"run": i, "server": st, "client": cli}), flush=True)
    print(json.dumps({"runs": n, "bad": bad, "clients": clients, "msg_len": msg_len, "tls": tls, "chunk": chunk}),
          flush=True)


if __name__ == "__main__":
    main()
