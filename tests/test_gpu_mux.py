"""GPU parity of fws_rx_mux: the reads of many connections decoded in one
round trip (FLoop::OneStep's shape, floop.h:661-703), each connection with its
own carried state (staged header bytes, unread payload, rotated key).

* every tests/golden/ KAT case is one connection of a single mux; round r
  feeds the r-th read of every case that has one, all in one call, and each
  read's return code, unmasked bytes, on_read / PONG / CLOSE events and
  carried state must equal what the compiled reference produced
  (w_socket.h:543-769) -- the same bar as test_gpu_session.py;
* both transfer modes: the batch copied to HBM and back, or (small batches)
  the kernel working on the pinned staging directly;
* 64 connections with random frame streams cut at random read sizes, some
  reads over the mux's segment limits (the per-connection session path):
  each connection's results equal a standalone fws_rx_session fed the same
  reads;
* fws_rx_mux_submit / _complete (the batched hook's pipeline): one batch at a
  time, and the result of a split call equals fws_rx_mux_feed.
"""
import gzip
import json
import os

import numpy as np
import pytest

import orc
from flashws_amd import gpu
from test_gpu_session import _out_matches, session_view
from wsframes import frame

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with gzip.open(os.path.join(GOLDEN, "kat_cases.json.gz"), "rt") as f:
    CASES = json.load(f)


@pytest.fixture(scope="module")
def mctx(cuda):
    c = gpu.Ctx(0, max_frames=1 << 16, max_stream_bytes=1 << 24)
    yield c
    c.close()


@pytest.fixture(params=["copy", "zero-copy"])
def zc_mode(request, monkeypatch):
    """the mux reads FWS_MUX_ZC_MAX at creation: 0 = every batch through the copy engines"""
    monkeypatch.setenv("FWS_MUX_ZC_MAX", "0" if request.param == "copy" else str(1 << 40))
    return request.param


def _state(st):
    return {k: int(getattr(st, k)) for k, _ in orc.RxStateHead._fields_}


def test_mux_all_kat_cases_at_once(mctx, zc_mode):
    names = sorted(CASES)
    mux = gpu.RxMux(mctx, len(names))
    closed = set()
    rounds = max(len(CASES[n]["reads"]) for n in names)
    for r in range(rounds):
        live = [ci for ci, n in enumerate(names) if r < len(CASES[n]["reads"])]
        got = mux.feed([(ci, bytes.fromhex(CASES[names[ci]]["reads"][r])) for ci in live])
        for ci, (ret, buf, ev, ctl) in zip(live, got):
            name, exp = names[ci], CASES[names[ci]]["expected"][r]
            assert ret == exp["ret"], (name, r)
            assert _out_matches(exp["out"], buf), (name, r)
            assert session_view(ev, ctl) == exp["events"], (name, r)
            if ret < 0:
                closed.add(ci)
            if ci not in closed:
                assert _state(mux.state(ci)) == exp["state"], (name, r)
    mux.close()


def _random_stream(rng, n_frames):
    out = []
    for i in range(n_frames):
        k = rng.random()
        if k < 0.15:                                   # a control frame
            out.append(frame(int(rng.choice([9, 10])), rng.integers(0, 256, int(rng.integers(0, 126)),
                                                                      dtype=np.uint8).tobytes(),
                             key=int(rng.integers(0, 2**32))))
            continue
        n = int(rng.choice([0, 5, 125, 126, 300, 4096, 65535, 65536, 70000, int(rng.integers(0, 9000))]))
        op = int(rng.choice([1, 2, 0]))
        out.append(frame(op, rng.integers(0, 256, n, dtype=np.uint8).tobytes(), fin=int(rng.random() < 0.6),
                         key=int(rng.integers(0, 2**32))))
    return b"".join(out)


@pytest.mark.parametrize("split", [False, True], ids=["feed", "submit_complete"])
@pytest.mark.parametrize("seed", range(2))
def test_mux_matches_per_connection_sessions(mctx, seed, zc_mode, split):
    rng = np.random.default_rng(900 + seed)
    n_conns = 64
    streams = [_random_stream(rng, int(rng.integers(5, 60))) for _ in range(n_conns)]
    cuts = []
    for s in streams:
        pos, c = 0, []
        while pos < len(s):
            step = int(rng.choice([1, 3, 7, 64, 1000, 4096, 20000, 300_000]))   # some over the segment limit
            c.append((pos, min(len(s), pos + step)))
            pos = c[-1][1]
        cuts.append(c)
    mux = gpu.RxMux(mctx, n_conns)
    ref = [gpu.RxSession(mctx) for _ in range(n_conns)]
    for r in range(max(len(c) for c in cuts)):
        live = [ci for ci in range(n_conns) if r < len(cuts[ci])]
        reads = [(ci, streams[ci][cuts[ci][r][0]:cuts[ci][r][1]]) for ci in live]
        got = mux.feed(reads, between=(lambda: None) if split else None)
        for (ci, data), (ret, buf, ev, ctl) in zip(reads, got):
            rret, rbuf, rev, rctl = ref[ci].feed(data)
            assert ret == rret, (ci, r)
            assert bytes(buf) == bytes(rbuf), (ci, r)
            assert session_view(ev, ctl) == session_view(rev, rctl), (ci, r)
            assert _state(mux.state(ci)) == _state(ref[ci].state()), (ci, r)
    for s in ref:
        s.close()
    mux.close()


def test_mux_reset_and_invalid_calls(mctx):
    mux = gpu.RxMux(mctx, 2)
    masked = frame(2, b"x" * 300, key=0x01020304)
    got = mux.feed([(0, masked[:100])])                # a frame in progress on slot 0
    assert got[0][0] == 0 and _state(mux.state(0))["recv_status"] == 1
    mux.reset(0)                                       # a new connection on the slot
    assert _state(mux.state(0))["recv_status"] == 0
    got = mux.feed([(0, masked), (1, masked)])
    assert [g[0] for g in got] == [0, 0] and bytes(got[0][1]) == bytes(got[1][1])
    with pytest.raises(Exception):
        mux.feed([(1, masked), (1, masked)])           # two reads of one connection in a call
    with pytest.raises(Exception):
        mux.feed([(2, masked)])                        # no such slot
    assert mux.feed([]) == []
    # submit / complete: one batch at a time, complete only after a submit
    from flashws_amd import _lib
    rr = np.zeros(1, dtype=_lib.RX_READ)
    buf = np.frombuffer(masked, dtype=np.uint8).copy()
    rr[0] = (1, 0, buf.ctypes.data, len(buf), len(buf))
    out = np.zeros(1, dtype=_lib.RX_READ_RESULT)
    assert mux.complete_raw(out) != 0                  # nothing submitted
    assert mux.submit_raw(rr, 1) == 0
    assert mux.submit_raw(rr, 1) != 0                  # a batch is in flight
    assert mux.complete_raw(out) == 0 and int(out[0]["ret"]) == 0
    assert bytes(buf[8:]) == b"x" * 300                # unmasked in place (8-B header: 16-bit length)
    assert mux.complete_raw(out) != 0
    assert mux.submit_raw(rr, 0) == 0 and mux.complete_raw(out[:0]) == 0   # an empty batch
    assert mux.submit_raw(rr, 1) == 0                  # left in flight: destroy waits for it
    mux.close()
