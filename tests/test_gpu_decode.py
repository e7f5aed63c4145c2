"""GPU parity of the fused header parse + unmask (fws_gpu_decode_stream) against
the oracle's restatement of OnRecvData / ParseFrameHdr (net/w_socket.h:435-769),
bit-exact: unmasked bytes, frame list (offset, length, key, opcode, FIN,
header length), status / error offset / carry-out.

Sizes the oracle finishes in seconds are compared byte-for-byte; full
BASELINE sizes additionally through size-independent properties.
"""
import numpy as np
import pytest
import torch

import orc
from flashws_amd import gpu
from wsframes import frame

pytestmark = pytest.mark.gpu

# mode -> (fws_internal_set_resolve_mode, fws_internal_set_st_target)
RESOLVE_MODES = {"super_tile": (0, 512), "big_st": (1, 512), "small_read": (2, 512), "st_1mib": (0, 1)}
CNT_FAILED = 9              # decode_common.h Counter::kCntFallback (the resolve failed)
CNT_BIG = 12                # decode_common.h Counter::kCntBig (super tiles on the big-ST path)


@pytest.fixture(params=list(RESOLVE_MODES), autouse=True)
def resolve_mode(request):
    """Every decode test runs on every decode path: the multi-launch path with
    the super-tile resolve in LDS (merge_kernels.hip) and with the big-ST path
    forced for every super tile; and the RX session's one-launch small-read
    kernel (small_kernels.hip; streams <= 128 KiB with <= 256 headers, the rest
    fall back to the super-tile path as the session does); and the super-tile
    path with the largest super tiles (1 MiB, r05: streams of 512 MiB and up get
    them) on every stream (st_1mib)."""
    from flashws_amd import _lib
    L = _lib.lib()
    mode, target = RESOLVE_MODES[request.param]
    old = L.fws_internal_set_resolve_mode(mode)
    old_t = L.fws_internal_set_st_target(target)
    yield request.param
    L.fws_internal_set_resolve_mode(old)
    L.fws_internal_set_st_target(old_t)


def counters(ctx):
    import ctypes as C
    from flashws_amd import _lib
    out = (C.c_uint32 * 32)()
    assert _lib.lib().fws_internal_decode_counters(ctx.h, out, 32) == 0
    return list(out)


def fell_back(ctx):
    """True if the last decode failed in the resolve or took the big-ST path."""
    c = counters(ctx)
    return c[CNT_FAILED] != 0 or c[CNT_BIG] != 0


def decode(ctx, wire, cuda, cap=None):
    dev = torch.from_numpy(np.ascontiguousarray(wire)).to(cuda)
    cap = cap if cap is not None else len(wire) // 6 + 16
    rc, fr, res, _ = gpu.decode_stream(ctx, dev, cap=cap)
    assert rc == 0, rc
    r = gpu.read_result(res)
    n = min(int(r["n_frames"]), cap)
    return dev.cpu().numpy(), gpu.read_frames(fr, n), r


def expect(wire):
    buf = np.array(wire, dtype=np.uint8, copy=True)
    ret, frames, err_off, consumed = orc.orc_decode_stream(buf)
    return buf, frames, ret, err_off, consumed


def check(ctx, cuda, wire):
    wire = np.frombuffer(bytes(wire), dtype=np.uint8) if not isinstance(wire, np.ndarray) else wire
    got, gframes, r = decode(ctx, wire, cuda)
    buf, frames, ret, err_off, consumed = expect(wire)
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


def test_rfc_hello(ctx, cuda):
    r = check(ctx, cuda, bytes.fromhex("818537fa213d7f9f4d5158"))
    assert int(r["n_frames"]) == 1 and int(r["consumed"]) == 11


def test_empty_stream(ctx, cuda):
    dev = torch.zeros(16, dtype=torch.uint8, device=cuda)
    rc, fr, res, _ = gpu.decode_stream(ctx, dev, cap=4, n=0)
    assert rc == 0
    r = gpu.read_result(res)
    assert int(r["status"]) == 0 and int(r["n_frames"]) == 0


@pytest.mark.parametrize("tail", [b"", b"\x82", b"\x82\xfe\x01", bytes([0x82, 0xFF]) + b"\0" * 5])
def test_incomplete_trailing_header(ctx, cuda, tail):
    wire = frame(2, b"abc" * 100) + frame(1, b"x") + tail
    r = check(ctx, cuda, wire)
    assert int(r["carry_hdr_len"]) == len(tail)


def test_truncated_payload(ctx, cuda):
    wire = frame(2, b"p" * 5000) + frame(2, bytes(range(256)) * 100)
    wire = wire[:-777]
    r = check(ctx, cuda, wire)
    assert int(r["carry_unread"]) == 777


@pytest.mark.parametrize("plen", [0, 1, 3, 4, 5, 15, 16, 17, 125, 126, 127, 4095, 4096, 65535, 65536, 70001])
def test_one_frame_streams(ctx, cuda, plen):
    """Streams that are one frame (the small-read decode's one-frame path,
    small_kernels.hip decode_one_frame, r05: the header parsed per wave from one
    broadcast load, chunks unmasked straight from memory): every length form at
    its boundaries, whole and cut -- inside the header (the general path: an
    incomplete header), right after it, one byte into the payload, one byte
    short of the end -- with keys whose bytes have the top bit set (a
    sign-extension bug in the header bytes' widening showed only with those),
    forced 16- and 64-bit length forms too, TEXT and BIN; bit-exact with the
    oracle in every resolve mode."""
    rng = np.random.default_rng(plen + 11)
    payload = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
    for key in (0x3D21FA37, 0xF1E2D3C4, 0x80808080):
        forms = [None] + ([126] if plen <= 65535 else []) + [127]
        for form in forms:
            for opcode in (1, 2):
                w = frame(opcode, payload, key=key, len_form=form)
                hdr = len(w) - plen
                for cut in sorted({len(w), len(w) - 1, hdr, hdr + 1, hdr - 1, 2}):
                    if 0 < cut <= len(w):
                        check(ctx, cuda, w[:cut])


@pytest.mark.parametrize("cut", [1, 3, 7, 40, 97, 3001])
def test_dense_units_cut_anywhere(ctx, cuda, cut):
    """Units that meet 3-64 frames (k_unmask_stream's register-held frames,
    unit-relative offsets clamped to the unit) with the stream ending inside a
    payload, inside a header, or on a unit edge: frames of 0-180 B with random
    keys, bit-exact with the oracle including the carry-out."""
    rng = np.random.default_rng(5000 + cut)
    parts, total = [], 0
    while total < 3 * 4096 + cut + 500:
        n = int(rng.integers(0, 180))
        parts.append(frame(int(rng.choice([1, 2, 0])), rng.integers(0, 256, n, dtype=np.uint8).tobytes(),
                           fin=int(rng.random() < 0.8), key=int(rng.integers(0, 2**32))))
        total += len(parts[-1])
    wire = b"".join(parts)
    check(ctx, cuda, wire[:3 * 4096 + cut])
    check(ctx, cuda, wire[:len(wire) - cut])


@pytest.mark.parametrize("bad,code", [(bytes([0xC2, 0x80]), -1), (bytes([0x83, 0x80]), -9),
                                      (bytes([0x82, 0x05]), -3),
                                      (bytes([0x82, 0xFF]) + (2**32 + 1).to_bytes(8, "big"), -2)])
@pytest.mark.parametrize("lead", [0, 1, 40, 20000, 40000])
def test_protocol_errors(ctx, cuda, bad, code, lead):
    rng = np.random.default_rng(lead)
    pre = b"".join(frame(2, rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes())
                   for _ in range(lead // 1000 + (1 if lead else 0)))
    wire = pre + bad + b"\0" * 64 + frame(2, b"never")
    r = check(ctx, cuda, wire)
    assert int(r["status"]) == code and int(r["err_off"]) == len(pre)


def test_first_header_invalid(ctx, cuda):
    r = check(ctx, cuda, bytes([0x80 | 3, 0x80]) + b"\0" * 100)
    assert int(r["status"]) == -9 and int(r["n_frames"]) == 0


def test_zero_length_and_control_frames(ctx, cuda):
    parts = [frame(2, b""), frame(9, b"ping"), frame(1, b"t", fin=0), frame(10, b"pong"),
             frame(0, b"", fin=0), frame(0, b"end"), frame(8, b"\x03\xe8")]
    check(ctx, cuda, b"".join(parts) * 50)


def test_length_forms(ctx, cuda):
    parts = [frame(2, b"hello", len_form=126), frame(2, b"hello", len_form=127),
             frame(2, b"q" * 65535), frame(2, b"r" * 65536), frame(2, b"s" * 125), frame(2, b"t" * 126)]
    check(ctx, cuda, b"".join(parts))


def test_len_2p32_header_only(ctx, cuda):
    wire = bytes([0x82, 0xFF]) + (1 << 32).to_bytes(8, "big") + b"\1\2\3\4" + b"\x55" * 300
    r = check(ctx, cuda, wire)
    assert int(r["carry_unread"]) == (1 << 32) - 300


@pytest.mark.parametrize("seed", range(8))
def test_random_small_frames(ctx, cuda, seed):
    """Dense frames (0..300 B) so every scan tile holds many true headers."""
    rng = np.random.default_rng(100 + seed)
    out = []
    total = 0
    while total < 200_000:
        n = int(rng.integers(0, 300))
        op = int(rng.choice([1, 2, 0, 9, 10])) if n <= 125 else int(rng.choice([1, 2, 0]))
        out.append(frame(op, rng.integers(0, 256, n, dtype=np.uint8).tobytes(),
                         fin=int(rng.random() < 0.7), key=int(rng.integers(0, 2**32))))
        total += len(out[-1])
    check(ctx, cuda, b"".join(out))


@pytest.mark.parametrize("seed", range(2))
def test_false_chains_join_the_path(ctx, cuda, seed):
    """Planted headers inside payloads whose exits land exactly on the next
    true header: false chains that merge into the true one inside a super tile
    (k_emit's tail-equality marking must see the extra survivors and fall back
    to pointer doubling). Bit-exact with the oracle."""
    rng = np.random.default_rng(700 + seed)
    frames = []
    for i in range(4000):
        n = int(rng.integers(60, 2000))
        frames.append(bytearray(frame(2, rng.integers(0, 256, n, dtype=np.uint8).tobytes(),
                                      key=int(rng.integers(0, 2**32)))))
    for i in range(0, len(frames) - 1, 3):
        f = frames[i]
        hl = 8 if len(f) - 8 >= 126 else 6               # this frame's header length
        pl = len(f) - hl
        # a fake 6-byte header at payload offset q whose next header is frames[i + 1]
        if pl < 6:
            continue
        flen = int(rng.integers(0, min(126, pl - 5)))      # its payload ends at frames[i + 1]
        q = pl - 6 - flen
        pos = hl + q
        f[pos:pos + 6] = bytes([0x82, 0x80 | flen]) + int(rng.integers(0, 2**32)).to_bytes(4, "little")
    check(ctx, cuda, b"".join(bytes(f) for f in frames))


@pytest.mark.parametrize("stride", [256, 1000, 2900, 4500])
def test_many_exit_tails_per_super_tile(ctx, cuda, stride, resolve_mode):
    """Planted 126-form headers of 65,000 B inside long payloads, one every
    `stride` bytes: each survives its tile and leaves its super tile, so every
    64 KiB super tile of this 2.4 MB stream has ~250, ~65, ~22 or ~14 EXIT
    tails -- past, past and just past k_merge's per-super-tile run of 16 (the
    overflow area, taken with an atomic, and k_link's loop over it), and
    within it. Bit-exact with the oracle; at ~250 per super tile the tail list
    of a workspace sized for this stream (64 per super tile + 4096) is full and
    the decode ends with FWS_ERR_CAPACITY, nothing listed or unmasked. With
    1 MiB super tiles (st_1mib) a planted header's exit lands in its own super
    tile: few EXIT tails, and the decode is checked bit-exact instead."""
    rng = np.random.default_rng(stride)
    frames = []
    for i in range(40):
        f = bytearray(frame(2, rng.integers(0, 256, 60000, dtype=np.uint8).tobytes(),
                            key=int(rng.integers(0, 2**32))))
        for q in range(8 + 64, len(f) - 16, stride):
            f[q:q + 8] = bytes([0x82, 0xFE]) + (65000).to_bytes(2, "big") + int(rng.integers(0, 2**32)).to_bytes(4, "little")
        frames.append(bytes(f))
    wire = np.frombuffer(b"".join(frames), dtype=np.uint8)
    # a fresh context: its decode workspace (tail list included) is sized by this
    # stream, not by the larger streams earlier tests decoded
    small = gpu.Ctx(0, max_frames=len(wire) // 6 + 16, max_stream_bytes=len(wire))
    try:
        if stride > 256 or resolve_mode == "st_1mib":
            check(small, cuda, wire)
            return
        got, _, r = decode(small, wire, cuda)
        from flashws_amd import _lib
        assert int(r["status"]) == _lib.FWS_ERR_CAPACITY and int(r["n_frames"]) == 0
        assert np.array_equal(got, wire)
    finally:
        small.close()


@pytest.mark.parametrize("seed", range(3))
def test_tiny_frames_dense_tiles(ctx, cuda, seed):
    """Frames of 0..24 B payload (~100 headers per 2 KiB tile): k_scan leaves
    every such tile to dense_tile() in k_merge (more live nodes than lanes);
    mixed with 4 KiB frames so sparse and dense tiles alternate."""
    rng = np.random.default_rng(500 + seed)
    out, total = [], 0
    while total < 600_000:
        if rng.random() < 0.02:
            n = 4096
        else:
            n = int(rng.integers(0, 25))
        op = int(rng.choice([1, 2, 0, 9, 10]))
        out.append(frame(op, rng.integers(0, 256, n, dtype=np.uint8).tobytes(),
                         fin=int(rng.random() < 0.7), key=int(rng.integers(0, 2**32))))
        total += len(out[-1])
    check(ctx, cuda, b"".join(out))
    c = counters(ctx)
    assert c[CNT_FAILED] == 0


@pytest.mark.parametrize("size", [1, 15, 16, 2030, 2047, 2048, 2049, 4103, 16383, 16384, 16385, 16390, 32768 + 7])
def test_single_frame_tile_boundaries(ctx, cuda, size):
    for lead in (0, 1, 7, 2030, 2041, 16370):
        wire = frame(2, b"a" * lead) + frame(1, bytes(range(256)) * (size // 256) + b"z" * (size % 256))
        check(ctx, cuda, wire)


def test_c3_mixed_parity(ctx, cuda, resolve_mode):
    """BASELINE config 3 shape (log-uniform 64 B..64 KiB) at 64 MiB, bit-exact."""
    wire, descs, _ = gpu.config_c3(seed=9, target=64 << 20)
    r = check(ctx, cuda, wire)
    assert int(r["n_frames"]) == len(descs)
    if resolve_mode == "super_tile":
        assert not fell_back(ctx), "C3 must resolve on the super-tile path with LDS tables"


def test_c2_full_parity(ctx, cuda, resolve_mode):
    wire, descs, _ = gpu.config_c2()
    r = check(ctx, cuda, wire)
    assert int(r["n_frames"]) == 65536
    if resolve_mode == "super_tile":
        assert not fell_back(ctx), "C2 must resolve on the super-tile path with LDS tables"


@pytest.mark.parametrize("n_frames,payload", [(200_000, 64), (200_000, 120), (1_600_000, 16)])
def test_dense_64b_frames(ctx, cuda, resolve_mode, n_frames, payload):
    """200 000 x 64 B frames, 120 B, and 1 600 000 x 16 B. These
    streams (14-35 MiB) are short, so the resolve uses 32 or 64 KiB super
    tiles (st_tiles_for, merge_kernels.hip): 64 B and 120 B frames then fit
    the LDS tables; 16 B frames in the 35 MiB stream (~3 000 per 64 KiB super
    tile) take the big-ST path, merged and emitted in LDS (merge_mid /
    emit_mid), or over global scratch when forced -- bit-exact either way."""
    wire, descs, _ = gpu.config_c2(seed=65, n_frames=n_frames, payload=payload)
    r = check(ctx, cuda, wire)
    assert int(r["n_frames"]) == n_frames
    c = counters(ctx)
    assert c[CNT_FAILED] == 0
    if resolve_mode != "small_read" and payload == 16:
        assert c[CNT_BIG] > 0


def test_c3_full_roundtrip(ctx, cuda):
    """Full C3 (256 MiB): frames equal the generator's, payload regions equal
    the descriptor-mode unmask of the same input (size-independent check)."""
    wire, descs, _ = gpu.config_c3()
    got, gframes, r = decode(ctx, wire, cuda, cap=len(descs) + 16)
    assert int(r["status"]) == 0 and int(r["n_frames"]) == len(descs)
    assert np.array_equal(gframes["hdr_off"] + gframes["hdr_len"], descs["payload_off"])
    assert np.array_equal(gframes["key"], descs["key"])
    dev = torch.from_numpy(wire).to(cuda)
    gpu.unmask_batch(ctx, dev, gpu.descs_to_device(descs, cuda), len(descs))
    assert np.array_equal(dev.cpu().numpy(), got)


def test_adversarial_all_valid_positions(ctx, cuda):
    """Every offset parses as a valid empty frame (0x80 0x80 ...): 6-byte frames."""
    wire = (bytes([0x80, 0x80]) + b"\x80" * 4) * 10000
    check(ctx, cuda, wire)


@pytest.mark.parametrize("pattern", [b"\x82\x82\x70\x70", b"\x82\x82\x70\x70\x70", b"\x82", b"\x89\x80",
                                     b"\x82\x82\x82\x82\x70", b"\x82\x82\x00",
                                     b"\x81\xfe\x00"])
def test_candidate_density(ctx, cuda, pattern):
    """Key-0 payloads whose wire bytes make many offsets pass the two-byte test:
    tiles with more candidate offsets than the sparse node list holds (every
    4th / every byte) next to sparse ones, all in one stream."""
    rng = np.random.default_rng(len(pattern))
    parts = []
    for i in range(12):
        n = int(rng.integers(1000, 40000))
        parts.append(frame(2, (pattern * (n // len(pattern) + 1))[:n], key=0))
        parts.append(frame(2, rng.integers(0, 256, int(rng.integers(0, 5000)), dtype=np.uint8).tobytes()))
    check(ctx, cuda, b"".join(parts))


@pytest.mark.parametrize("seed", range(2))
def test_candidate_counts_at_node_limits(ctx, cuda, seed):
    """2 KiB regions with 56-72, 120-136 and 248-264 two-byte candidates
    (0x81 0x80: an empty masked TEXT header) on filler that never passes the
    test: tiles on both sides of k_scan's direct-node limit (64 candidates,
    every candidate a node), of the live-node limit and of the dense-tile
    limit (256). Candidates 6 bytes apart chain into runs of false headers."""
    rng = np.random.default_rng(500 + seed)
    parts = []
    for lo in (56, 120, 248):
        pay = bytearray(b"\x10" * (2048 * 17))
        for r in range(17):
            k = lo + r
            for sl in rng.choice(682, size=k, replace=False):
                q = 2048 * r + 3 * int(sl)
                pay[q:q + 2] = b"\x81\x80"
        parts.append(frame(2, bytes(pay), key=0))
        parts.append(frame(2, rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()))
    check(ctx, cuda, b"".join(parts))


@pytest.fixture(params=[1, 0], ids=["pf", "no_pf"])
def stream_utf8_pf(request):
    """k_unmask_stream<utf8> with (default) and without the cross-unit prefetch"""
    from flashws_amd._lib import lib
    old = lib().fws_internal_set_stream_utf8_pf(request.param)
    yield request.param
    lib().fws_internal_set_stream_utf8_pf(old)


def test_utf8_flags_c5_shape(ctx, cuda, stream_utf8_pf):
    wire, descs, ok = gpu.config_c5(seed=5, n_frames=512, payload=16384, invalid_permille=100)
    dev = torch.from_numpy(wire).to(cuda)
    flags = torch.zeros(len(descs), dtype=torch.uint8, device=cuda)
    rc, fr, res, _ = gpu.decode_stream(ctx, dev, cap=len(descs) + 4, utf8_ok=flags)
    assert rc == 0
    got = flags.cpu().numpy()
    assert np.array_equal(got, ok), (got.sum(), ok.sum())
    unm = dev.cpu().numpy()
    exp = [orc.orc_utf8_valid(unm[o:o + n]) for o, n in zip(descs["payload_off"], descs["payload_len"])]
    assert np.array_equal(got.astype(bool), np.array(exp))


def _utf8_payload(rng, n_chars, corrupt):
    s = "".join(chr(int(c)) for c in rng.integers(0x20, 0x10FFFF, n_chars) if not 0xD800 <= int(c) <= 0xDFFF)
    b = bytearray(s.encode())
    if corrupt == 1 and len(b):
        b[int(rng.integers(0, len(b)))] = int(rng.integers(0x80, 0x100))
    elif corrupt == 2 and len(b):
        b = b[:-1]                                   # a sequence cut at the frame end (or not)
    return bytes(b)


@pytest.mark.parametrize("seed", range(4))
def test_utf8_flags_mixed_stream(ctx, cuda, seed, stream_utf8_pf):
    """Fused decode + UTF-8 flags on TEXT frames of every size (tiny frames take
    the per-chunk unmask path, big ones the uniform path), misaligned against
    the 4 KiB stream units and 16-B chunks, next to BIN / non-FIN / control
    frames; flags must equal Python's strict decoder on eligible frames."""
    rng = np.random.default_rng(40 + seed)
    parts, kinds = [], []
    total = 0
    while total < 600_000:
        r = rng.random()
        if r < 0.08:
            op, fin, body = 2, 1, _utf8_payload(rng, int(rng.integers(0, 2000)), 0)
        elif r < 0.12:
            op, fin, body = 1, 0, _utf8_payload(rng, int(rng.integers(0, 500)), 0)
        elif r < 0.15:
            op, fin, body = 9, 1, _utf8_payload(rng, int(rng.integers(0, 30)), 0)
        else:
            size = int(rng.choice([rng.integers(0, 40), rng.integers(40, 2000), rng.integers(2000, 9000)]))
            op, fin, body = 1, 1, _utf8_payload(rng, size, int(rng.integers(0, 3)))
        parts.append(frame(op, body, fin=fin, key=int(rng.integers(0, 2**32))))
        kinds.append((op, fin, body))
        total += len(parts[-1])
    wire = np.frombuffer(b"".join(parts), dtype=np.uint8)
    dev = torch.from_numpy(wire.copy()).to(cuda)
    flags = torch.full((len(parts) + 4,), 7, dtype=torch.uint8, device=cuda)
    rc, fr, res, _ = gpu.decode_stream(ctx, dev, cap=len(parts) + 4, utf8_ok=flags)
    assert rc == 0
    r = gpu.read_result(res)
    assert int(r["status"]) == 0 and int(r["n_frames"]) == len(parts)
    got = flags.cpu().numpy()[:len(parts)]
    for i, (op, fin, body) in enumerate(kinds):
        exp = False
        if op == 1 and fin:
            try:
                body.decode("utf-8")
                exp = True
            except UnicodeDecodeError:
                pass
        assert bool(got[i]) == exp, (i, op, fin, body[-8:])


def test_utf8_flags_unit_seams(ctx, cuda, stream_utf8_pf):
    """TEXT frames placed so that multi-byte sequences, cut sequences, invalid
    bytes and frame ends straddle 4 KiB stream-unit boundaries (the seam
    kernel's bytes)."""
    rng = np.random.default_rng(77)
    parts, bodies = [], []
    pos = 0
    for k in range(150):
        # the payload end lands at unit boundary + d, d in -3..3
        d = int(rng.integers(-3, 4))
        target = (pos // 4096 + 2) * 4096 + d
        seq = rng.choice([b"\xe2\x82\xac", b"\xf0\x9d\x84\x9e", b"\xc3\xa9", b"a"])
        n = target - pos - 8
        body = bytearray((seq * (n // len(seq) + 2))[:n])
        if k % 5 == 1:
            body[-1] = 0xE2                              # cut at the end
        elif k % 5 == 2:
            body[-int(rng.integers(1, 4))] = 0x80        # stray continuation near the end
        elif k % 5 == 3:
            # an invalid byte at or near the end: the table check flags it at the byte after
            # it, which may be the next unit's first bytes or the zero bytes past the payload
            body[-int(rng.integers(1, 5))] = int(rng.choice([0xC0, 0xC1, 0xF5, 0xF8, 0xFF]))
        elif k % 5 == 4:
            # ... or at a unit seam inside the payload
            at = ((pos + 8) // 4096 + 1) * 4096 + int(rng.integers(-4, 4)) - pos - 8
            if 0 <= at < len(body):
                body[at] = int(rng.choice([0xC0, 0xC1, 0xF5, 0xF8, 0xFF]))
        parts.append(frame(1, bytes(body), key=int(rng.integers(0, 2**32)), len_form=126))
        bodies.append(bytes(body))
        pos += len(parts[-1])
    wire = np.frombuffer(b"".join(parts), dtype=np.uint8)
    dev = torch.from_numpy(wire.copy()).to(cuda)
    flags = torch.zeros(len(parts), dtype=torch.uint8, device=cuda)
    rc, _, res, _ = gpu.decode_stream(ctx, dev, cap=len(parts), utf8_ok=flags)
    assert rc == 0 and int(gpu.read_result(res)["n_frames"]) == len(parts)
    got = flags.cpu().numpy()
    for i, b in enumerate(bodies):
        try:
            b.decode("utf-8")
            exp = True
        except UnicodeDecodeError:
            exp = False
        assert bool(got[i]) == exp, (i, b[-6:])


def test_validate_utf8_edge_cases(ctx, cuda):
    cases = [b"", b"a", b"\xc2\x80", b"\xc2", b"\xe0\xa0\x80", b"\xe0\x9f\x80", b"\xed\x9f\xbf", b"\xed\xa0\x80",
             b"\xf0\x90\x80\x80", b"\xf0\x8f\xbf\xbf", b"\xf4\x8f\xbf\xbf", b"\xf4\x90\x80\x80", b"\xf5\x80\x80\x80",
             b"\xc0\x80", b"\xc1\xbf", b"\x80", b"a\xe2\x82", "héllo wörld €𝄞".encode(), b"\xff", b"ab\xe2\x82\xacd"]
    rng = np.random.default_rng(3)
    for _ in range(300):
        cases.append(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes())
        s = "".join(chr(int(c)) for c in rng.integers(0x20, 0x2FFF, 20) if not 0xD800 <= int(c) <= 0xDFFF)
        b = bytearray(s.encode())
        if len(b) and rng.random() < 0.5:
            b[int(rng.integers(0, len(b)))] = int(rng.integers(0x80, 0x100))
        cases.append(bytes(b))
    # long strings: sequences across lanes and 1 KiB wave steps, errors anywhere
    for _ in range(60):
        s = "".join(chr(int(c)) for c in rng.integers(0x20, 0x10FFFF, int(rng.integers(100, 1500)))
                    if not 0xD800 <= int(c) <= 0xDFFF)
        b = bytearray(s.encode())
        k = int(rng.integers(0, 4))
        if k == 1:
            b[int(rng.integers(0, len(b)))] = int(rng.integers(0x80, 0x100))
        elif k == 2:
            b = b[:-1]                                  # maybe cut a sequence at the end
        cases.append(bytes(b))
    blob, regions, pos = bytearray(), [], 0
    for c in cases:
        pad = int(rng.integers(0, 20))
        # bytes around a region are arbitrary (leads, continuations): outside bytes never count
        blob += rng.integers(0x80, 0x100, pad, dtype=np.uint8).tobytes()
        pos += pad
        regions.append((pos, len(c), 0, 0))
        blob += c
        pos += len(c)
    dev = torch.frombuffer(bytearray(blob) + b"\xf0" * 32, dtype=torch.uint8).to(cuda)
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    ok = torch.zeros(len(descs), dtype=torch.uint8, device=cuda)
    gpu.validate_utf8(ctx, dev, gpu.descs_to_device(descs, cuda), len(descs), ok)
    got = ok.cpu().numpy().astype(bool)
    for c, g in zip(cases, got):
        try:
            c.decode("utf-8")
            exp = True
        except UnicodeDecodeError:
            exp = False
        assert g == exp, c
        assert orc.orc_utf8_valid(c) == exp, c


def test_gather_reassembly_c4_shape(ctx, cuda):
    wire, descs, _ = gpu.config_c4(seed=3, target=32 << 20)
    src = torch.from_numpy(wire).to(cuda)
    total = int(descs["payload_len"].sum())
    dst = torch.zeros(total + 64, dtype=torch.uint8, device=cuda)
    gpu.unmask_gather(ctx, dst, src, gpu.descs_to_device(descs, cuda), len(descs))
    buf = wire.copy()
    ret, frames, _, _ = orc.orc_decode_stream(buf)
    assert ret == 0
    exp = np.zeros(total, dtype=np.uint8)
    w = orc.orc().orc_reassemble(buf.ctypes.data, frames.ctypes.data, len(frames), exp.ctypes.data)
    assert w == total
    assert np.array_equal(dst[:total].cpu().numpy(), exp)
    assert int(dst[total:].sum()) == 0
    assert torch.equal(src.cpu(), torch.from_numpy(wire))          # source untouched


def test_gather_small_regions(ctx, cuda):
    rng = np.random.default_rng(8)
    regions, pos = [], 5
    for _ in range(3000):
        n = int(rng.integers(0, 40))
        regions.append((pos, n, int(rng.integers(0, 2**32)), int(rng.integers(0, 4))))
        pos += n + int(rng.integers(0, 5))
    host = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    total = int(descs["payload_len"].sum())
    dst = torch.zeros(total + 16, dtype=torch.uint8, device=cuda)
    gpu.unmask_gather(ctx, dst, torch.from_numpy(host).to(cuda), gpu.descs_to_device(descs, cuda), len(descs))
    exp, w = np.zeros(total, dtype=np.uint8), 0
    for o, n, k, ph in regions:
        seg = host[o:o + n].copy()
        orc.orc_mask("mask1", seg, orc.orc().orc_rotr32(k, 8 * ph))
        exp[w:w + n] = seg
        w += n
    assert np.array_equal(dst[:total].cpu().numpy(), exp)


@pytest.mark.parametrize("shape", ["many_mixed", "one_huge_among_small", "permuted_sources"])
def test_gather_plan_shapes(ctx, cuda, shape):
    """k_out_plan layouts: > 16 384 regions (256 per workgroup), a long run of
    unit-map entries among short ones (64 per workgroup), sources in any order."""
    rng = np.random.default_rng({"many_mixed": 21, "one_huge_among_small": 22, "permuted_sources": 23}[shape])
    if shape == "many_mixed":
        lens = [int(x) for x in rng.choice([0, 7, 100, 4096, 9000, 70000], 20000)]
    elif shape == "one_huge_among_small":
        lens = [int(x) for x in rng.integers(0, 3000, 500)]
        lens[217] = 8 << 20
    else:
        lens = [int(x) for x in rng.integers(1, 20000, 3000)]
    offs, pos = [], 3
    for n in lens:
        offs.append(pos)
        pos += n + int(rng.integers(0, 9))
    host = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    regions = [(o, n, int(rng.integers(0, 2**32)), int(rng.integers(0, 4))) for o, n in zip(offs, lens)]
    if shape == "permuted_sources":
        regions = [regions[i] for i in rng.permutation(len(regions))]
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    total = int(descs["payload_len"].sum())
    dst = torch.zeros(total + 16, dtype=torch.uint8, device=cuda)
    gpu.unmask_gather(ctx, dst, torch.from_numpy(host).to(cuda), gpu.descs_to_device(descs, cuda), len(descs))
    exp, w = np.zeros(total, dtype=np.uint8), 0
    for o, n, k, ph in regions:
        seg = host[o:o + n].copy()
        orc.orc_mask("ws_mask_fast", seg, orc.orc().orc_rotr32(k, 8 * ph))
        exp[w:w + n] = seg
        w += n
    got = dst[:total].cpu().numpy()
    assert np.array_equal(got, exp), int(np.flatnonzero(got != exp)[0])
    assert int(dst[total:].sum()) == 0


@pytest.mark.parametrize("nfr", [1, 2, 255, 256, 257, 400])
@pytest.mark.parametrize("tail", ["none", "truncated", "partial_header"])
def test_small_read_frame_counts(ctx, cuda, nfr, tail):
    """Header counts around the small-read kernel's walk limit (256: more are
    declined and decoded by the parallel path), with the read ending at a
    frame end, inside a payload or inside a header."""
    rng = np.random.default_rng(nfr * 7 + len(tail))
    parts = [frame(int(rng.choice([1, 2, 0])), rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes(),
                   fin=int(rng.random() < 0.8), key=int(rng.integers(0, 2**32))) for _ in range(nfr)]
    wire = b"".join(parts)
    if tail == "truncated":
        wire += frame(2, b"z" * 3000)[:-1234]
    elif tail == "partial_header":
        wire += frame(2, b"z" * 300)[:5]
    check(ctx, cuda, wire)


@pytest.mark.parametrize("size", [65537, 131072 - 7, 131072, 131073, 140000])
def test_small_read_size_limit(ctx, cuda, size):
    """Streams either side of the small-read kernel's 128 KiB limit."""
    rng = np.random.default_rng(size)
    parts, n = [], 0
    while n < size:
        p = int(min(rng.integers(100, 9000), max(size - n - 8, 0)))
        f = frame(2, rng.integers(0, 256, p, dtype=np.uint8).tobytes(), key=int(rng.integers(0, 2**32)))
        parts.append(f)
        n += len(f)
    wire = b"".join(parts)[:size]
    check(ctx, cuda, wire)


def test_small_read_capacity(ctx, cuda, resolve_mode):
    """cap below the header count: the first cap frames listed and unmasked,
    FWS_ERR_CAPACITY, n_frames = all headers; identical on every path (each
    mode is compared with the default super-tile path)."""
    rng = np.random.default_rng(5)
    wire = np.frombuffer(b"".join(frame(2, rng.integers(0, 256, int(rng.integers(0, 400)), dtype=np.uint8).tobytes(),
                                       key=int(rng.integers(0, 2**32))) for _ in range(60)), dtype=np.uint8)
    got, gframes, r = decode(ctx, wire, cuda, cap=23)
    from flashws_amd import _lib
    L = _lib.lib()
    old = L.fws_internal_set_resolve_mode(0)
    try:
        ref, rframes, rr = decode(ctx, wire, cuda, cap=23)
    finally:
        L.fws_internal_set_resolve_mode(old)
    assert int(r["status"]) == int(rr["status"]) == -20
    assert int(r["n_frames"]) == int(rr["n_frames"]) == 60
    for k in ("hdr_off", "payload_len", "key", "opcode", "fin", "hdr_len"):
        assert np.array_equal(gframes[k], rframes[k]), k
    assert np.array_equal(got, ref)
