"""GPU: limits and hardening of the host-facing entry points, each against the
oracle (oracle/fws_oracle.c, pinned by tests/golden).

* RX session first reads around the pinned staging threshold (16 KiB): every
  size from 16 368 to 16 400 bytes as a fresh session's first read;
* control frames the reference would copy past its 125-byte buffer (a PING of
  1000 B split across reads, a 126-B PING, a 200-B CLOSE) are refused with
  FWS_ERR_CONTROL_FRAME (RFC 6455 §5.5; w_socket.h:654 only asserts); a small
  control frame with FIN = 0 is handled as the reference handles it (FIN is
  not checked, w_socket.h:659-711), compared with the oracle;
* descriptor batches larger than the context's reservation (unmask_batch in
  chunk space, gather) are still unmasked in full;
* fws_rx_pipe's frame-list copy-back (a guess from the previous batch, the
  remainder copied by the wait) under batches whose frame counts jump.
"""
import numpy as np
import pytest
import torch

import orc
from flashws_amd import gpu
from wsframes import frame

pytestmark = pytest.mark.gpu

FWS_ERR_CONTROL_FRAME = -10


def _norm_gpu(ev, ctl):
    out = []
    for e in ev:
        o, n = int(e["ctl_off"]), int(e["size"])
        rec = (int(e["kind"]), int(e["opcode"]), int(e["is_ctl"]), int(e["frame_end"]), int(e["msg_end"]), n)
        if int(e["kind"]) == 0 and not e["is_ctl"]:
            rec += (int(e["data_off"]), int(e["capacity"]))
        else:
            rec += (bytes(ctl[o:o + n]),)
        out.append(rec)
    return out


def _norm_orc(ev, ctl):
    out = []
    for e in ev:
        k = int(e["kind"])
        if k == 3:
            continue                                   # oracle-only header bookkeeping
        o, n = int(e["ctl_off"]), int(e["size"])
        rec = (k, int(e["opcode"]), int(e["is_ctl"]), int(e["frame_end"]), int(e["msg_end"]), n)
        if k == 0 and not e["is_ctl"]:
            rec += (int(e["data_off"]), int(e["capacity"]))
        else:
            rec += (bytes(ctl[o:o + n]),)
        out.append(rec)
    return out


def _stream_of(size, rng):
    """Client frames totalling exactly `size` bytes (the last one may be cut)."""
    out = b""
    while len(out) < size:
        n = int(rng.choice([0, 5, 125, 126, 700, 3000, 9000]))
        out += frame(int(rng.choice([1, 2])), rng.integers(0, 256, n, dtype=np.uint8).tobytes(),
                     key=int(rng.integers(0, 2**32)))
    return out[:size]


@pytest.fixture(scope="module")
def sctx(cuda):
    c = gpu.Ctx(0, max_frames=1 << 14, max_stream_bytes=1 << 22)
    yield c
    c.close()


@pytest.mark.parametrize("size", list(range(16368, 16401)))
def test_session_first_read_at_staging_threshold(sctx, size):
    rng = np.random.default_rng(size)
    full = _stream_of(size + 5000, rng)
    s, o = gpu.RxSession(sctx), orc.OrcSession()
    for rd in (full[:size], full[size:]):
        ret, buf, ev, ctl = s.feed(rd)
        eret, ebuf, eev, ectl = o.feed(rd)
        assert ret == eret == 0
        assert np.array_equal(buf, ebuf)
        assert _norm_gpu(ev, ctl) == _norm_orc(eev, ectl)
        st, est = s.state(), o.head()
        for k, _ in orc.RxStateHead._fields_:
            assert int(getattr(st, k)) == int(getattr(est, k)), k
    s.close()


@pytest.mark.parametrize("case", ["ping_1000_split", "ping_126", "close_200"])
def test_session_refuses_oversized_control_frames(sctx, case):
    lead = frame(2, b"before")
    if case == "ping_1000_split":
        bad = frame(9, bytes(range(256)) * 3 + bytes(232))
        reads = [lead + bad[:500], bad[500:] + frame(2, b"after")]
    elif case == "ping_126":
        reads = [lead + frame(9, b"p" * 126)]
    else:
        reads = [lead + frame(8, b"\x03\xe8" + b"r" * 198)]
    s = gpu.RxSession(sctx)
    ret, buf, ev, ctl = s.feed(reads[0])
    assert ret == FWS_ERR_CONTROL_FRAME, ret
    # the data frame before it was still delivered, unmasked, as the reference would
    ev = _norm_gpu(ev, ctl)
    assert ev[0][:6] == (0, 2, 0, 1, 1, 6)
    off = ev[0][6]
    assert bytes(buf[off:off + 6]) == b"before"
    s.close()


def test_session_control_frame_fin0_as_reference(sctx):
    """PING / PONG with FIN = 0 (<= 125 B), inside and between messages: the
    reference answers / delivers them at frame end without checking FIN; the
    session's events and PONG replies equal the oracle's."""
    data = (frame(2, b"before") + frame(9, b"abc", fin=0) + frame(1, b"He", fin=0) + frame(10, b"pong", fin=0)
            + frame(0, b"llo") + frame(9, b"def"))
    s, o = gpu.RxSession(sctx), orc.OrcSession()
    for rd in (data[:25], data[25:44], data[44:]):     # cuts inside data payloads
        ret, buf, ev, ctl = s.feed(rd)
        eret, ebuf, eev, ectl = o.feed(rd)
        assert ret == eret == 0
        assert np.array_equal(buf, ebuf)
        assert _norm_gpu(ev, ctl) == _norm_orc(eev, ectl)
    s.close()


def test_session_control_frame_125_ok(sctx):
    """The largest legal control payload still goes through (and matches the oracle)."""
    data = frame(2, b"x" * 10) + frame(9, bytes(range(125))) + frame(2, b"y")
    s, o = gpu.RxSession(sctx), orc.OrcSession()
    for rd in (data[:40], data[40:]):
        ret, buf, ev, ctl = s.feed(rd)
        eret, ebuf, eev, ectl = o.feed(rd)
        assert ret == eret == 0
        assert np.array_equal(buf, ebuf)
        assert _norm_gpu(ev, ctl) == _norm_orc(eev, ectl)
    s.close()


@pytest.mark.parametrize("order", ["sorted_sparse", "permuted"])
def test_unmask_batch_beyond_reservation(cuda, order):
    """A batch 64x larger than the context reserved: the plan's unit map ends
    at its capacity, the run finds the owners of later units by search."""
    rng = np.random.default_rng(31 if order == "permuted" else 32)
    n = 6000
    lens = rng.integers(1, 20000, n)
    gaps = rng.integers(0, 3000 if order == "sorted_sparse" else 40, n)
    offs = np.cumsum(np.concatenate([[7], (lens + gaps)[:-1]]))
    host = rng.integers(0, 256, int(offs[-1] + lens[-1] + 64), dtype=np.uint8)
    descs = np.zeros(n, dtype=gpu.FRAME_DESC)
    descs["payload_off"], descs["payload_len"] = offs, lens
    descs["key"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    descs["phase"] = rng.integers(0, 4, n)
    if order == "permuted":
        descs = descs[rng.permutation(n)]
    c = gpu.Ctx(0, max_frames=n, max_stream_bytes=1 << 20)      # ~60 MB batch, 1 MiB reserved
    dev = torch.from_numpy(host).to(cuda)
    gpu.unmask_batch(c, dev, gpu.descs_to_device(descs, cuda), n)
    exp = host.copy()
    for d in descs:
        o, ln = int(d["payload_off"]), int(d["payload_len"])
        orc.orc_mask("ws_mask_bytes", exp, orc.orc().orc_rotr32(int(d["key"]), 8 * int(d["phase"])), o, ln)
    assert np.array_equal(dev.cpu().numpy(), exp)
    c.close()


def test_gather_beyond_reservation(cuda):
    wire, descs, _ = gpu.config_c4(seed=5, target=48 << 20)
    c = gpu.Ctx(0, max_frames=len(descs), max_stream_bytes=1 << 20)
    src = torch.from_numpy(wire).to(cuda)
    total = int(descs["payload_len"].sum())
    dst = torch.zeros(total + 64, dtype=torch.uint8, device=cuda)
    gpu.unmask_gather(c, dst, src, gpu.descs_to_device(descs, cuda), len(descs))
    buf = wire.copy()
    ret, frames, _, _ = orc.orc_decode_stream(buf)
    assert ret == 0
    exp = np.zeros(total, dtype=np.uint8)
    assert orc.orc().orc_reassemble(buf.ctypes.data, frames.ctypes.data, len(frames), exp.ctypes.data) == total
    assert np.array_equal(dst[:total].cpu().numpy(), exp)
    assert int(dst[total:].sum()) == 0
    c.close()


def test_pipe_frame_copy_guess(cuda):
    """Frame counts jump between batches (few large frames, then many small
    ones): the records past the copied-back guess come from the wait."""
    specs = [("c2", 64), ("c3small", 0), ("c2", 8), ("c3small", 1), ("c3small", 2)]
    wires = []
    for i, (kind, k) in enumerate(specs):
        if kind == "c2":
            wires.append(gpu.config_c2(seed=400 + i, n_frames=k, payload=65536)[0])
        else:
            w, d, _ = gpu.gen_batch(gpu.GEN_MIXED, seed=410 + i, opcode=2, payload_min=1, payload_max=200,
                                    target_bytes=1 << 20)
            wires.append(w)
    pipe = gpu.RxPipe(0, max_batch_bytes=8 << 20, max_frames=1 << 16, depth=2)
    for w in wires:
        host = torch.from_numpy(w.copy()).pin_memory()
        frames, res, _ = pipe.wait(pipe.submit(host))
        buf = w.copy()
        ret, ef, _, _ = orc.orc_decode_stream(buf)
        assert int(res["status"]) == ret and int(res["n_frames"]) == len(ef)
        assert np.array_equal(host.numpy(), buf)
        for k in ("hdr_off", "payload_len", "key", "opcode", "fin", "hdr_len"):
            assert np.array_equal(frames[k], ef[k]), k
    pipe.close()
