"""GPU: the north star's drop-in -- a flashws echo server on the reference's
own FLoop + WSServerSocket<false> (compiled from the reference headers,
oracle/_ref/ws_dropin, source tools/dropin/ws_dropin.cpp) whose receive decode
is moved to the MI355X by ONE added call, fws_amd::GpuRxHook::Enable
(include/flashws_amd/gpu_floop.hpp). No reference file is changed.

* scripted parity: the same byte scripts (fragmented messages, interleaved
  PINGs, every length form, random read splits, CLOSE with code and reason,
  protocol errors) are sent by a raw client to the reference's own server and
  to the same server with the GPU hook; everything the client receives back
  (echo frames, PONGs, the CLOSE echo or the 1006 error close with the
  reference's error text) and the server's on_close log must be identical;
* load: the reference's WSClientSocket with many connections, every echoed
  byte checked, PINGs answered, clean CLOSE handshakes, through the GPU hook;
* batched (ws:// and wss://): the same scripted parity, load runs and the
  reference's echo client with GpuRxHook::EnableBatched, which decodes the
  reads of all connections of one FLoop step in one GPU round trip
  (fws_rx_mux) at the end of the step;
* wss:// (SURVEY §8f rank 4): the same scripted parity and a load run over
  the reference's TLSSocket (WSServerSocket<true> + fws_amd::GpuRxHookTls):
  OpenSSL decrypts on the CPU, the GPU decodes the plaintext reads. The
  certificate is the test-only self-signed one in tests/tls/.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import wsraw
from wsframes import frame

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "oracle", "_ref", "ws_dropin")
TLS_ARGS = ["--tls", "--cert", os.path.join(ROOT, "tests", "tls", "server.crt"),
            "--key", os.path.join(ROOT, "tests", "tls", "server.key")]


class Server:
    def __init__(self, gpu, conns, max_seconds=90, tls=False, batch=False):
        if not os.path.exists(DROPIN):
            pytest.fail("oracle/_ref/ws_dropin not built (make -C oracle ref in the build container; "
                        "__graft_entry__.build() produces it)", pytrace=False)
        args = [DROPIN, "server", "--conns", str(conns), "--max-seconds", str(max_seconds)]
        if gpu:
            args.append("--gpu-batch" if batch else "--gpu")
        if tls:
            args += TLS_ARGS
        self.p = subprocess.Popen(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        line = self.p.stdout.readline()
        assert line.startswith("listening"), (line, self.p.stderr.read()[-2000:] if self.p.poll() is not None else "")
        self.port = int(line.split()[1])

    def finish(self, timeout=60):
        out, err = self.p.communicate(timeout=timeout)
        assert self.p.returncode == 0, err[-2000:]
        return json.loads(out.strip().splitlines()[-1])


def _chunks(atoms, rng, max_chunk):
    """Send sizes for the concatenated atoms: random cut points, but never
    inside or right after a control frame's header -- the reference server
    dereferences a null control buffer when a read ends there (SURVEY
    Appendix A.5), so such splits are kept out of the comparison."""
    stream = b"".join(a for a, _ in atoms)
    banned, pos = set(), 0
    for a, ctl in atoms:
        if ctl:
            banned.update(range(pos + 1, pos + len(a)))
        pos += len(a)
    cuts, p = [], 0
    while True:
        p += int(rng.integers(1, max_chunk + 1))
        if p >= len(stream):
            break
        if p not in banned:
            cuts.append(p)
    bounds = [0] + cuts + [len(stream)]
    return stream, [b - a for a, b in zip(bounds, bounds[1:])]


def _scripts():
    rng = np.random.default_rng(2026)

    def key():
        return int(rng.integers(0, 2**32))

    def msg(op, payload, pieces=1, ping_after=None):
        atoms, n = [], len(payload)
        cuts = sorted(set(int(x) for x in rng.integers(0, n + 1, pieces - 1))) if pieces > 1 else []
        bounds = [0] + cuts + [n]
        for k in range(len(bounds) - 1):
            first, last = k == 0, k == len(bounds) - 2
            atoms.append((frame(op if first else 0, payload[bounds[k]:bounds[k + 1]], fin=int(last), key=key()),
                          False))
            if ping_after == k:
                atoms.append((frame(9, b"mid-message ping", key=key()), True))
        return atoms

    def rand_payload(n):
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()

    mixed = []
    for i in range(60):
        n = int(rng.choice([0, 1, 5, 125, 126, 127, 1000, 4096, 65535, 65536, 70000, int(rng.integers(0, 20000))]))
        op = int(rng.choice([1, 2]))
        pl = rand_payload(n) if op == 2 else bytes(rng.integers(32, 127, n, dtype=np.uint8))
        pieces = int(rng.choice([1, 1, 2, 3]))
        mixed += msg(op, pl, pieces, ping_after=0 if (pieces > 1 and i % 3 == 0) else None)
        if i % 7 == 0:
            mixed.append((frame(9, rand_payload(int(rng.integers(0, 126))), key=key()), True))
    good = [(frame(2, b"some data before the error"), False)]
    byte_wise = [(frame(2, rand_payload(300 + k)), False) for k in range(5)]
    s_byte, c_byte = _chunks(byte_wise, rng, 1)
    close = wsraw.close_frame(1000)
    return {
        "mixed_then_close": _chunks(mixed + [(wsraw.close_frame(1000, b"done"), True)], rng, 9000),
        "close_code_only": _chunks([(frame(2, b"x" * 300), False), (wsraw.close_frame(1001), True)], rng, 11),
        "ping_125_then_close": _chunks([(frame(9, bytes(range(125))), True), (frame(1, b"hello"), False),
                                        (wsraw.close_frame(1000, b"ok"), True)], rng, 200),
        "err_rsv1": _chunks(good + [(bytes([0xC2, 0x80]) + b"\0" * 8, False)], rng, 9),
        "err_opcode3": _chunks(good + [(bytes([0x83, 0x85, 1, 2, 3, 4]) + b"abcde", False)], rng, 40),
        "err_len_2p32p1": _chunks(good + [(bytes([0x82, 0xFF]) + (2**32 + 1).to_bytes(8, "big") + b"\0" * 4, False)],
                                  rng, 4),
        "split_header_every_byte": (s_byte + close, c_byte + [len(close)]),
    }


SCRIPTS = _scripts()


def _run_all(gpu, tls=False, batch=False):
    srv = Server(gpu, conns=len(SCRIPTS), tls=tls, batch=batch)
    got = {}
    for name, (stream, chunks) in SCRIPTS.items():
        head, data = wsraw.run_script(srv.port, stream, chunks, tls=tls)
        got[name] = (head, data)
    return got, srv.finish()


def _hook_env(chunk, monkeypatch):
    """chunk: None (default chunks; the step's last chunk deferred to the next
    step while the loop has events waiting, SetDeferLastChunk's default), an int
    (FWS_HOOK_CHUNK: the batched hook's reads go to the GPU in chunks of this
    many) or "flush" (FWS_HOOK_DEFER=0: every step's chunks dispatched at its
    end, the r05 hook)"""
    if chunk == "flush":
        monkeypatch.setenv("FWS_HOOK_DEFER", "0")
    elif chunk is not None:
        monkeypatch.setenv("FWS_HOOK_CHUNK", str(chunk))


@pytest.mark.parametrize("tls,batch,chunk", [(False, False, None), (True, False, None), (False, True, None),
                                             (True, True, None), (False, True, 1), (True, True, 2),
                                             (False, True, "flush"), (True, True, "flush")],
                         ids=["ws", "wss", "ws_batched", "wss_batched", "ws_batched_chunk1", "wss_batched_chunk2",
                              "ws_batched_flush", "wss_batched_flush"])
def test_dropin_scripted_parity_with_reference_server(cuda, tls, batch, chunk, monkeypatch):
    """Scripted sessions (split reads, PING, fragmented messages, protocol
    errors, CLOSE) against the reference server and the hooked one, per read
    and batched per loop step (GpuRxHook::EnableBatched): handshake replies,
    every echoed / control / close frame byte and the close log are equal."""
    _hook_env(chunk, monkeypatch)
    ref, ref_srv = _run_all(gpu=False, tls=tls)
    gpu, gpu_srv = _run_all(gpu=True, tls=tls, batch=batch)
    assert gpu_srv["gpu_reads"] > 0 and ref_srv["gpu_reads"] == 0
    assert (gpu_srv["gpu_batches"] > 0) == batch
    for name in SCRIPTS:
        assert gpu[name][0] == ref[name][0], name                     # handshake reply
        assert gpu[name][1] == ref[name][1], (name, wsraw.parse_server_frames(ref[name][1])[-2:],
                                              wsraw.parse_server_frames(gpu[name][1])[-2:])
    assert gpu_srv["msgs"] == ref_srv["msgs"] and gpu_srv["bytes"] == ref_srv["bytes"]
    assert gpu_srv["close_log_hex"] == ref_srv["close_log_hex"]
    # what the scripts must have produced (not only equal, also right)
    fr = wsraw.parse_server_frames(gpu["err_rsv1"][1])
    assert fr[0][1] == 2 and fr[-1][1] == 8
    assert fr[-1][2][:2] == (1006).to_bytes(2, "big") and fr[-1][2][2:] == b"rev bits are not zero"
    fr = wsraw.parse_server_frames(gpu["err_opcode3"][1])
    assert fr[-1][2][2:] == b"Opcode 3 is not valid"
    fr = wsraw.parse_server_frames(gpu["mixed_then_close"][1])
    assert fr[-1] == (1, 8, (1000).to_bytes(2, "big") + b"done")
    assert sum(1 for f in fr if f[1] == 10) > 0                       # PONGs


@pytest.mark.parametrize("clients,msg_len,tls,batch,chunk", [
    (1, 4096, False, False, None), (8, 4096, False, False, None), (4, 70000, False, False, None),
    (16, 512, False, False, None), (8, 4096, True, False, None), (2, 70000, True, False, None),
    (8, 4096, False, True, None), (4, 70000, False, True, None), (16, 512, False, True, None),
    (8, 4096, True, True, None), (16, 512, False, True, 3), (8, 70000, False, True, 2), (8, 4096, True, True, 2),
    (8, 4096, False, True, "flush"), (16, 512, False, True, "flush"), (4, 70000, False, True, "flush"),
    (8, 4096, True, True, "flush")])
def test_dropin_reference_client_load(cuda, clients, msg_len, tls, batch, chunk, monkeypatch):
    _hook_env(chunk, monkeypatch)
    srv = Server(True, conns=clients, tls=tls, batch=batch)
    r = subprocess.run([DROPIN, "client", "--port", str(srv.port), "--clients", str(clients), "--msgs", "600",
                        "--warmup", "20", "--msg-len", str(msg_len), "--ping-every", "50", "--max-seconds", "60"]
                       + (["--tls"] if tls else []), capture_output=True, text=True, timeout=90)
    assert r.returncode == 0, (r.stdout, r.stderr[-2000:])
    cli = json.loads(r.stdout.strip().splitlines()[-1])
    st = srv.finish()
    assert cli["verified"] is True and cli["pongs"] == clients * (620 // 50)
    assert st["gpu_reads"] > 0 and st["msgs"] == clients * 620
    if not tls:                     # the loop's MemPool read slots, proven by the pool's own records
        assert st["zc_slots"] > 0
    assert all(c == [1000, b"bye".hex()] for c in st["close_log_hex"][:clients]), st
    if batch:                       # the step's reads went to the GPU together
        assert 0 < st["gpu_batches"] <= st["gpu_reads"]
    if chunk == "flush":            # SetDeferLastChunk(false): no step end leaves a chunk in flight
        assert st["deferred_chunks"] == 0


REF_CLIENTS = {n: os.path.join(ROOT, "oracle", "_ref", f"ws_ref_client_{n}") for n in (1, 8)}
REF_CLIENT_PORT = 58600        # oracle/refclient/test_def.h (compile-time in the reference client)


def run_reference_client(n_clients, gpu, tmp_path, batch=False):
    """The reference's unchanged tests/new-ws-echo/test_ws_client.cpp (built by
    oracle/Makefile `refclient` with our loopback test_def.h: 4 KiB BIN
    messages, 40,000 in total) against the drop-in server. Returns the client's
    stdout and the server's JSON line."""
    exe = REF_CLIENTS[n_clients]
    if not os.path.exists(exe):
        pytest.fail(f"{exe} not built (make -C oracle refclient in the build container)", pytrace=False)
    args = [DROPIN, "server", "--port", str(REF_CLIENT_PORT), "--conns", str(n_clients), "--max-seconds", "90"]
    if gpu:
        args.append("--gpu-batch" if batch else "--gpu")
    p = subprocess.Popen(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    assert line.startswith("listening"), (line, p.stderr.read()[-2000:] if p.poll() is not None else "")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, cwd=str(tmp_path))
    out, err = p.communicate(timeout=60)
    assert p.returncode == 0, err[-2000:]
    return r, json.loads(out.strip().splitlines()[-1])


@pytest.mark.parametrize("n_clients,batch", [(1, False), (8, False), (8, True)], ids=["1", "8", "8_batched"])
def test_reference_echo_client_through_gpu_hook(cuda, n_clients, batch, tmp_path):
    """C1 through the reference's own echo client: every message the client gets
    back was unmasked by the MI355X (GpuRxHook), its FWS_ASSERT(size ==
    MAX_DATA_LEN) holds for each one (test_ws_client.cpp:217) and its HashArr
    of the echoed payload equals the hash of what it sent at every 16,384th
    message (test_ws_client.cpp:260-277; a mismatch aborts the client)."""
    r, st = run_reference_client(n_clients, True, tmp_path, batch=batch)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    data_hash = [ln.split(":")[1].strip() for ln in r.stdout.splitlines() if ln.startswith("data hash:")]
    checks = [ln.rsplit("hash value:", 1)[1].split(",")[0].strip() for ln in r.stdout.splitlines()
              if "hash value:" in ln]
    assert len(data_hash) == 1 and len(checks) == 40000 // 16384, r.stdout[-3000:]
    assert all(c == data_hash[0] for c in checks)
    assert "avg (rx+tx) goodput" in r.stdout
    assert st["gpu"] is True and st["gpu_reads"] > 0 and st["msgs"] == 40000


REF_SERVER_GPU = os.path.join(ROOT, "oracle", "_ref", "ws_ref_server_gpu")


@pytest.mark.parametrize("n_clients", [1, 8])
def test_reference_echo_server_unchanged_with_gpu_hook(cuda, n_clients, tmp_path):
    """Both ends of C1 are the reference's own code: tests/new-ws-echo/
    test_ws_server.cpp and test_ws_client.cpp, compiled unchanged from their
    place (oracle/Makefile `refserver` / `refclient`). The server's one hook line
    (GpuRxHook::Enable on its listening socket) comes from our test_def.h, so
    every read the server decodes goes through the MI355X; the client's HashArr
    checks of the echo (test_ws_client.cpp:260-277) pass, and the hook's GPU
    read count, printed at SIGTERM, is non-zero."""
    if not os.path.exists(REF_SERVER_GPU):
        pytest.fail(f"{REF_SERVER_GPU} not built (make -C oracle refserver in the build container)", pytrace=False)
    exe = REF_CLIENTS[n_clients]
    p = subprocess.Popen([REF_SERVER_GPU], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         cwd=str(tmp_path))
    try:
        seen = []
        for line in p.stdout:
            seen.append(line)
            if line.startswith("gpu hook enabled"):
                break
        assert seen and seen[-1].startswith("gpu hook enabled"), ("".join(seen)[-2000:], p.poll())
        r = subprocess.run([exe], capture_output=True, text=True, timeout=120, cwd=str(tmp_path))
    finally:
        p.terminate()
        out, err = p.communicate(timeout=30)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    data_hash = [ln.split(":")[1].strip() for ln in r.stdout.splitlines() if ln.startswith("data hash:")]
    checks = [ln.rsplit("hash value:", 1)[1].split(",")[0].strip() for ln in r.stdout.splitlines()
              if "hash value:" in ln]
    assert len(data_hash) == 1 and len(checks) == 40000 // 16384, r.stdout[-3000:]
    assert all(c == data_hash[0] for c in checks)
    reads = [int(ln.split()[1]) for ln in out.splitlines() if ln.startswith("gpu_reads ")]
    assert reads and reads[0] > 0, (out[-2000:], err[-2000:])


@pytest.mark.parametrize("scenario", ["close_peers", "eof_with_data"])
@pytest.mark.parametrize("mode", ["gpu", "gpu_batch", "gpu_batch_chunk1", "gpu_batch_flush"])
def test_dropin_same_step_reads_match_reference(cuda, scenario, mode, monkeypatch):
    """Two reads in one FLoop step (tests/dropin_steps.py): (close_peers) A's
    on_read closes connection B while B's read of the same step is still to be
    handled -- the batched hook hands it to the reference's closing-state
    callback as the per-read path does, so B's TCP socket is closed at once;
    (eof_with_data) B's last data and its EOF arrive in one event -- the batched
    hook decodes B's pending read before on_close (floop.h:715-730), so the
    message is counted as in the reference. Everything both clients receive and
    the server's message count and close log equal the reference server's."""
    import dropin_steps
    ref = dropin_steps.run_scenario(DROPIN, "reference", scenario)
    if mode == "gpu_batch_chunk1":  # every read submitted as it arrives, dispatched at the next one
        monkeypatch.setenv("FWS_HOOK_CHUNK", "1")
        mode = "gpu_batch"
    elif mode == "gpu_batch_flush":  # every step flushed at its end (SetDeferLastChunk(false))
        monkeypatch.setenv("FWS_HOOK_DEFER", "0")
        mode = "gpu_batch"
    got = dropin_steps.run_scenario(DROPIN, mode, scenario)
    assert got["server"]["gpu_reads"] > 0
    if mode == "gpu_batch":
        assert got["server"]["gpu_batches"] > 0
    for k in ("msgs", "bytes", "close_log_hex"):
        assert got["server"][k] == ref["server"][k], (k, got["server"], ref["server"])
    assert got["a_frames"] == ref["a_frames"] and got["b_frames"] == ref["b_frames"], (got, ref)
    if scenario == "close_peers":
        assert ref["b_frames"] == [(1, 8, (1000).to_bytes(2, "big") + b"peer")]
    else:
        assert ref["server"]["msgs"] == 3          # sleep, shutwr and B's last data frame
