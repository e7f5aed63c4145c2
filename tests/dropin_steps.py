"""Two-connection scenarios whose reads must land in ONE FLoop::OneStep of the
drop-in server (tools/dropin/ws_dropin.cpp --commands), for comparing the
batched GPU hook with the reference server (test helper, no GPU by itself).

Connection A sends "cmd:sleep:<ms>": the server echoes it and its end-of-step
callback then sleeps, so whatever both clients send in the meantime is read in
the next step, A's read first (A's socket is readable first).

* "close_peers": A sends "cmd:close-peers" (the server echoes it and closes B
  with 1000 "peer" from A's on_read), B sends a data frame. In the reference,
  B's read arrives at a closing socket: the readable callback closes the TCP
  socket (ws_server_socket.h:187-194).
* "eof_with_data": B first sends "cmd:shutwr" (the server shuts its TCP write
  side), then -- inside the sleep -- a "cmd:noecho..." frame and its FIN, so the
  next step reads B's data and sees EPOLLHUP in the same event (floop.h:715-730:
  DeleteFd(true) -> on_close). The reference delivers the read before on_close.

Each scenario returns what both clients received and the server's JSON line.
"""
import socket
import subprocess
import time

import wsraw
from wsframes import frame


def _read_until(s, pred, timeout=10.0):
    s.settimeout(timeout)
    got = b""
    t0 = time.time()
    while not pred(got):
        if time.time() - t0 > timeout:
            raise TimeoutError(f"waited for {pred}, got {got[:64]!r}")
        b = s.recv(1 << 16)
        if not b:
            return got, True
        got += b
    return got, False


def _drain(s, timeout=10.0):
    s.settimeout(timeout)
    got = b""
    try:
        while True:
            b = s.recv(1 << 16)
            if not b:
                break
            got += b
    except (ConnectionResetError, socket.timeout):
        pass
    return got


def run_scenario(dropin, mode, scenario, sleep_ms=300):
    """mode: "reference", "gpu" (per read) or "gpu_batch"."""
    args = [dropin, "server", "--conns", "2", "--max-seconds", "60", "--commands"]
    if mode == "gpu":
        args.append("--gpu")
    elif mode == "gpu_batch":
        args.append("--gpu-batch")
    p = subprocess.Popen(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    assert line.startswith("listening"), (line, p.stderr.read()[-2000:] if p.poll() is not None else "")
    port = int(line.split()[1])
    a, _, ra = wsraw.connect(port)
    b, _, rb = wsraw.connect(port)
    out = {}
    if scenario == "eof_with_data":
        b.sendall(frame(2, b"cmd:shutwr", key=0x01020304))
        got, eof = _read_until(b, lambda g: False)           # the server's FIN
        assert eof, got
        rb += got
    sleep_msg = f"cmd:sleep:{sleep_ms}".encode()
    a.sendall(frame(2, sleep_msg, key=0x0A0B0C0D))
    got, _ = _read_until(a, lambda g: len(wsraw.parse_server_frames(g)) >= 1)
    ra += got
    # the server now sleeps at the end of this step: both sends land in the next one
    if scenario == "close_peers":
        a.sendall(frame(2, b"cmd:close-peers", key=0x11121314))
        b.sendall(frame(2, b"data from b, sent while the server sleeps", key=0x21222324))
        rb += _drain(b)                                       # CLOSE 1000 "peer", then EOF
        got, _ = _read_until(a, lambda g: len(wsraw.parse_server_frames(g)) >= 1)
        ra += got
    elif scenario == "eof_with_data":
        b.sendall(frame(2, b"cmd:noecho, then FIN in the same step", key=0x31323334))
        b.shutdown(socket.SHUT_WR)
        rb += _drain(b)                                       # (the server's FIN came earlier)
        time.sleep(sleep_ms / 1000.0 + 0.2)                   # A's CLOSE in a later step
    else:
        raise ValueError(scenario)
    b.close()
    a.sendall(wsraw.close_frame(1000, b"a done"))
    ra += _drain(a)
    a.close()
    o, e = p.communicate(timeout=60)
    assert p.returncode == 0, e[-2000:]
    import json
    out["server"] = json.loads(o.strip().splitlines()[-1])
    out["a_frames"] = wsraw.parse_server_frames(ra)
    out["b_frames"] = wsraw.parse_server_frames(rb)
    return out
