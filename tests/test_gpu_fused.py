"""GPU parity of the one-pass decode (k_stream, stream_kernels.hip) on the
branches the shared decode tests (tests/test_gpu_decode.py, `fused` mode) do
not force: frames longer than the fast tables' key depth (4 super tiles of
32 KiB, so the look-back waits for the landing super tile's own inclusive
state), more frames than the frame list holds, an incomplete header that
starts one super tile before the last, a protocol error deep in a long stream
(the multi-launch fallback finishes it and skips the super tiles k_stream
unmasked), and repeated calls on one context (epoch-tagged words). Bit-exact
against the oracle (w_socket.h:435-769 restated) or against the multi-launch
path on the same input where the oracle has no counterpart (capacity).
"""
import numpy as np
import pytest
import torch

import orc
from flashws_amd import _lib, gpu

pytestmark = pytest.mark.gpu

ST = 32768                   # fws_internal.h kFusedStBytes
CNT_FMODE, CNT_FFAIL = 13, 14


@pytest.fixture(autouse=True)
def fused_forced():
    L = _lib.lib()
    old = L.fws_internal_set_fused(2)
    oldr = L.fws_internal_set_resolve_mode(0)
    yield
    L.fws_internal_set_fused(old)
    L.fws_internal_set_resolve_mode(oldr)


def np_frame(rng, opcode, n, fin=1):
    """A client frame (header, random key, payload masked) built with numpy."""
    key = int(rng.integers(0, 2**32))
    kb = np.frombuffer(key.to_bytes(4, "little"), dtype=np.uint8)
    if n < 126:
        hdr = [0x80 * fin | opcode, 0x80 | n]
    elif n < 65536:
        hdr = [0x80 * fin | opcode, 0x80 | 126] + list(n.to_bytes(2, "big"))
    else:
        hdr = [0x80 * fin | opcode, 0x80 | 127] + list(n.to_bytes(8, "big"))
    pay = rng.integers(0, 256, n, dtype=np.uint8)
    masked = pay ^ np.resize(kb, n)
    return np.concatenate([np.array(hdr, dtype=np.uint8), kb, masked])


def counters(ctx):
    import ctypes as C
    out = (C.c_uint32 * 32)()
    assert _lib.lib().fws_internal_decode_counters(ctx.h, out, 32) == 0
    return list(out)


def decode(ctx, wire, cuda, cap=None):
    dev = torch.from_numpy(np.array(wire, dtype=np.uint8, copy=True)).to(cuda)
    cap = cap if cap is not None else len(wire) // 6 + 16
    rc, fr, res, _ = gpu.decode_stream(ctx, dev, cap=cap)
    assert rc == 0, rc
    r = gpu.read_result(res)
    n = min(int(r["n_frames"]), cap)
    return dev.cpu().numpy(), gpu.read_frames(fr, n), r


def check(ctx, cuda, wire):
    got, gframes, r = decode(ctx, wire, cuda)
    buf = np.array(wire, dtype=np.uint8, copy=True)
    ret, frames, err_off, consumed = orc.orc_decode_stream(buf)
    assert int(r["status"]) == ret
    assert int(r["n_frames"]) == len(frames)
    for k in ("hdr_off", "payload_len", "key", "opcode", "fin", "hdr_len"):
        assert np.array_equal(gframes[k], frames[k]), k
    assert np.array_equal(got, buf)
    if ret < 0:
        assert int(r["err_off"]) == err_off
    else:
        assert int(r["consumed"]) == consumed
    return r


@pytest.mark.parametrize("seed", range(3))
def test_frames_longer_than_key_depth(ctx, cuda, seed):
    """Frames of 160 KiB .. 1.5 MiB (5 .. 48 super tiles) among small ones:
    the true chain lands beyond every fast-table key, and the look-back waits
    for that super tile's own resolution. k_stream must finish the stream."""
    rng = np.random.default_rng(100 + seed)
    parts = []
    for _ in range(12):
        parts.append(np_frame(rng, 2, int(rng.integers(5 * ST, 48 * ST))))
        for _ in range(int(rng.integers(0, 40))):
            parts.append(np_frame(rng, 2, int(rng.integers(0, 3000))))
    wire = np.concatenate(parts)
    check(ctx, cuda, wire)
    c = counters(ctx)
    assert c[CNT_FMODE] == 1 and c[CNT_FFAIL] == 0, "k_stream must decode this stream alone"


def test_repeated_calls_one_context(ctx, cuda):
    """Epoch-tagged granules: three calls on one context, each exact."""
    wire, descs, _ = gpu.config_c3(seed=5, target=24 << 20)
    for _ in range(3):
        r = check(ctx, cuda, wire)
        assert int(r["n_frames"]) == len(descs)
        c = counters(ctx)
        assert c[CNT_FMODE] == 1 and c[CNT_FFAIL] == 0


@pytest.mark.parametrize("where", [0.1, 0.5, 0.93])
def test_protocol_error_deep_in_stream(ctx, cuda, where):
    """An RSV-set header at 10 / 50 / 93 % of a 12 MiB stream: k_stream finishes
    the super tiles before it, the multi-launch path the rest (its unmask skips
    the finished ones), the result is OnRecvData's."""
    rng = np.random.default_rng(int(where * 100))
    parts, size = [], 0
    target = 12 << 20
    bad_at = int(where * target)
    placed = False
    while size < target:
        if not placed and size >= bad_at:
            parts.append(np.array([0xC2, 0x85, 1, 2, 3, 4, 9, 9, 9, 9, 9], dtype=np.uint8))
            placed = True
        f = np_frame(rng, 2, int(2 ** (6 + 10 * rng.random())))
        parts.append(f)
        size += len(f)
    wire = np.concatenate(parts)
    r = check(ctx, cuda, wire)
    assert int(r["status"]) == -1


@pytest.mark.parametrize("tail_len", [1, 5, 12])
def test_incomplete_header_before_last_super_tile(ctx, cuda, tail_len):
    """The stream ends tail_len (< 13) bytes into its last 32 KiB super tile, inside a
    14-byte header that starts one byte before that super tile."""
    rng = np.random.default_rng(tail_len)
    k = 40
    h = k * ST - 1                                      # the cut header starts in super tile k - 1
    parts, size = [], 0
    while h - size > 60000:
        f = np_frame(rng, 2, int(rng.integers(100, 9000)))
        parts.append(f)
        size += len(f)
    parts.append(np_frame(rng, 2, h - size - 8))        # 8-byte header: ends exactly at h
    body = np.concatenate(parts)
    assert len(body) == h
    wire = np.concatenate([body, np_frame(rng, 2, 70000)])[:k * ST + tail_len]
    r = check(ctx, cuda, wire)
    assert int(r["consumed"]) == h and int(r["carry_hdr_len"]) == tail_len + 1


def test_capacity_matches_multi_launch_path(ctx, cuda):
    """More frames than `cap`: k_stream declines (FAIL) and the multi-launch
    path produces the capacity result; bytes, frames and result must equal a
    run with k_stream off."""
    wire, descs, _ = gpu.config_c2(seed=3, n_frames=4000, payload=1000)
    cap = 2500
    got, gframes, r = decode(ctx, wire, cuda, cap=cap)
    L = _lib.lib()
    L.fws_internal_set_fused(0)
    try:
        got0, gframes0, r0 = decode(ctx, wire, cuda, cap=cap)
    finally:
        L.fws_internal_set_fused(2)
    assert int(r["status"]) == int(r0["status"]) == -20
    assert int(r["n_frames"]) == int(r0["n_frames"])
    assert np.array_equal(gframes, gframes0)
    assert np.array_equal(got, got0)
