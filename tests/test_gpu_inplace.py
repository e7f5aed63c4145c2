"""GPU: reads in registered host memory decoded in place (the drop-in hook
registers the reference's MemPool read buffers, flash_alloc.h:44-73, with
fws_gpu_host_register; rx_session.cpp then skips the pinned staging copies).
The same bar as the staged paths: every tests/golden/ KAT case replayed read
by read against the compiled reference's results (w_socket.h:543-769), through
a session and all at once through a mux, with each read 16-B aligned (decoded
in place) or 5 bytes off (staged: the kernels' chunk grid needs 16-B aligned
parts), and random multi-connection traffic against standalone sessions."""
import gzip
import json
import os

import numpy as np
import pytest

import orc
from flashws_amd import gpu
from test_gpu_mux import _random_stream
from test_gpu_session import _out_matches, session_view
from wsframes import frame

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with gzip.open(os.path.join(GOLDEN, "kat_cases.json.gz"), "rt") as f:
    CASES = json.load(f)


@pytest.fixture(scope="module")
def ictx(cuda):
    c = gpu.Ctx(0, max_frames=1 << 16, max_stream_bytes=1 << 24)
    yield c
    c.close()


@pytest.fixture(scope="module")
def arena(cuda):
    a = gpu.HostArena(32 << 20)
    yield a
    a.close()


def _state(st):
    return {k: int(getattr(st, k)) for k, _ in orc.RxStateHead._fields_}


@pytest.mark.parametrize("align_off", [0, 5], ids=["aligned", "off5"])
def test_session_in_place_kat(ictx, arena, align_off):
    for name in sorted(CASES):
        case = CASES[name]
        s = gpu.RxSession(ictx)
        for i, (rd, exp) in enumerate(zip(case["reads"], case["expected"])):
            ret, buf, ev, ctl = s.feed(bytes.fromhex(rd), arena=arena, align_off=align_off)
            assert ret == exp["ret"], (name, i)
            assert _out_matches(exp["out"], buf), (name, i)
            assert session_view(ev, ctl) == exp["events"], (name, i)
            if ret < 0:
                break
            assert _state(s.state()) == exp["state"], (name, i)
        s.close()


@pytest.mark.parametrize("zc", ["copy", "zero-copy"])
def test_mux_in_place_kat(ictx, arena, zc, monkeypatch):
    monkeypatch.setenv("FWS_MUX_ZC_MAX", "0" if zc == "copy" else str(1 << 40))
    names = sorted(CASES)
    mux = gpu.RxMux(ictx, len(names))
    closed = set()
    rounds = max(len(CASES[n]["reads"]) for n in names)
    for r in range(rounds):
        live = [ci for ci, n in enumerate(names) if r < len(CASES[n]["reads"]) and ci not in closed]
        # every third read off the 16-B grid (staged), the rest in place
        got = mux.feed([(ci, bytes.fromhex(CASES[names[ci]]["reads"][r])) for ci in live], arena=arena,
                       align_off=lambda i: 7 if i % 3 == 2 else 0)
        for ci, (ret, buf, ev, ctl) in zip(live, got):
            name, exp = names[ci], CASES[names[ci]]["expected"][r]
            assert ret == exp["ret"], (name, r)
            assert _out_matches(exp["out"], buf), (name, r)
            assert session_view(ev, ctl) == exp["events"], (name, r)
            if ret < 0:
                closed.add(ci)
            else:
                assert _state(mux.state(ci)) == exp["state"], (name, r)
    mux.close()


def test_mux_in_place_random_vs_sessions(ictx, arena):
    """64 connections, random frame streams cut at random read sizes (some
    reads continuation-only, some with staged header bytes, some over the
    in-place limits), reads in registered memory: every connection's results
    equal a standalone unregistered session fed the same reads."""
    rng = np.random.default_rng(404)
    n = 64
    streams = [_random_stream(rng, int(rng.integers(5, 40))) for _ in range(n)]
    cuts = []
    for st in streams:
        pos, c = 0, []
        while pos < len(st):
            k = int(rng.choice([1, 7, 100, 4096, 5000, 70000, 300000]))
            c.append(st[pos:pos + k])
            pos += k
        cuts.append(c)
    mux = gpu.RxMux(ictx, n)
    ref = [gpu.RxSession(ictx) for _ in range(n)]
    dead = set()
    for r in range(max(len(c) for c in cuts)):
        live = [i for i in range(n) if r < len(cuts[i]) and i not in dead]
        got = mux.feed([(i, cuts[i][r]) for i in live], arena=arena)
        for i, (ret, buf, ev, ctl) in zip(live, got):
            eret, ebuf, eev, ectl = ref[i].feed(cuts[i][r])
            assert ret == eret, (i, r)
            assert bytes(buf) == bytes(ebuf), (i, r)
            assert session_view(ev, ctl) == session_view(eev, ectl), (i, r)
            if ret < 0:
                dead.add(i)
    mux.close()
    for s in ref:
        s.close()


def _declined_reads(rng, n_tiny):
    """A continuation of 48 B (a multiple of 16, so the header stream after it
    stays on the 16-B grid) followed by n_tiny frames of 0-6 B payload: more
    than kSmallFrames (256) headers, so the in-place one-launch decode declines
    and the parallel decode runs on the registered bytes (rx_session.cpp, the
    FWS_SMALL_DECLINED branch after k_decode_one)."""
    big = frame(2, rng.integers(0, 256, 1000, dtype=np.uint8).tobytes(), key=int(rng.integers(0, 2**32)))
    tiny = b"".join(frame(int(rng.choice([1, 2])), rng.integers(0x20, 0x7F, int(rng.integers(0, 7)),
                                                                 dtype=np.uint8).tobytes(),
                          key=int(rng.integers(0, 2**32))) for _ in range(n_tiny))
    return [big[:-48], big[-48:] + tiny]


@pytest.mark.parametrize("n_tiny", [300, 2000])
def test_session_in_place_declined_small_read(ictx, arena, n_tiny):
    """the declined in-place path (continuation unmasked in place by
    k_decode_one, then the parallel decode on the registered alias) against an
    unregistered session fed the same reads."""
    rng = np.random.default_rng(900 + n_tiny)
    reads = _declined_reads(rng, n_tiny)
    s, ref = gpu.RxSession(ictx), gpu.RxSession(ictx)
    for rd in reads:
        ret, buf, ev, ctl = s.feed(rd, arena=arena, align_off=0)
        eret, ebuf, eev, ectl = ref.feed(rd)
        assert ret == eret == 0
        assert bytes(buf) == bytes(ebuf)
        assert session_view(ev, ctl) == session_view(eev, ectl)
    assert len(ev) >= n_tiny                             # an event per tiny frame at least
    s.close()
    ref.close()


@pytest.mark.parametrize("zc", ["copy", "zero-copy"])
def test_mux_in_place_declined_small_read(ictx, arena, zc, monkeypatch):
    """The same reads on three connections of one mux (registered, in place),
    against unregistered standalone sessions."""
    monkeypatch.setenv("FWS_MUX_ZC_MAX", "0" if zc == "copy" else str(1 << 40))
    rng = np.random.default_rng(77)
    conns = [_declined_reads(rng, k) for k in (300, 40, 1200)]
    mux = gpu.RxMux(ictx, len(conns))
    ref = [gpu.RxSession(ictx) for _ in conns]
    for r in range(2):
        got = mux.feed([(i, conns[i][r]) for i in range(len(conns))], arena=arena)
        for i, (ret, buf, ev, ctl) in enumerate(got):
            eret, ebuf, eev, ectl = ref[i].feed(conns[i][r])
            assert ret == eret == 0, (i, r)
            assert bytes(buf) == bytes(ebuf), (i, r)
            assert session_view(ev, ctl) == session_view(eev, ectl), (i, r)
    mux.close()
    for x in ref:
        x.close()
