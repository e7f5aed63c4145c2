"""GPU parity: fws_gpu_unmask_sorted_utf8 (one-pass unmask + per-region UTF-8
flags, BASELINE config 5 in descriptor mode). Bytes vs the oracle's
WSMaskBytesFast restatement (crypto/ws_mask.h:175-197); flags vs Python's
strict UTF-8 decoder (the reference does not validate UTF-8: parity unpinned
against it, pinned to Unicode Table 3-7 / RFC 3629) and vs the
two-pass fws_gpu_unmask_sorted + fws_gpu_validate_utf8."""
import numpy as np
import pytest
import torch

from flashws_amd import gpu
from test_gpu_unmask import aligned_host, oracle_unmask_regions

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=[0, 1, 2], ids=["plain", "pipe", "early"])
def utf8_pipe(request):
    """every test runs on every form of k_unmask_sorted_utf8 (plain, software-pipelined,
    loads before the owner lookup)"""
    from flashws_amd import lib
    old = lib().fws_internal_set_sorted_utf8_pipe(request.param)
    yield request.param
    lib().fws_internal_set_sorted_utf8_pipe(old)


def _valid(b):
    try:
        b.decode("utf-8")
        return True
    except UnicodeDecodeError:
        return False


def _cases(rng, n_short, n_long, long_chars):
    cases = [b"", b"a", b"\xc2\x80", b"\xc2", b"\xe0\xa0\x80", b"\xe0\x9f\x80", b"\xed\x9f\xbf", b"\xed\xa0\x80",
             b"\xf0\x90\x80\x80", b"\xf0\x8f\xbf\xbf", b"\xf4\x8f\xbf\xbf", b"\xf4\x90\x80\x80", b"\xf5\x80\x80\x80",
             b"\xc0\x80", b"\xc1\xbf", b"\x80", b"a\xe2\x82", "héllo wörld €𝄞".encode(), b"\xff", b"ab\xe2\x82\xacd"]
    for _ in range(n_short):
        cases.append(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes())
        s = "".join(chr(int(c)) for c in rng.integers(0x20, 0x2FFF, 20) if not 0xD800 <= int(c) <= 0xDFFF)
        b = bytearray(s.encode())
        if len(b) and rng.random() < 0.5:
            b[int(rng.integers(0, len(b)))] = int(rng.integers(0x80, 0x100))
        cases.append(bytes(b))
    for _ in range(n_long):      # sequences across lanes, chunks, 4 KiB units (seams), errors anywhere
        s = "".join(chr(int(c)) for c in rng.integers(0x20, 0x10FFFF, int(rng.integers(*long_chars)))
                    if not 0xD800 <= int(c) <= 0xDFFF)
        b = bytearray(s.encode())
        k = int(rng.integers(0, 4))
        if k == 1:
            b[int(rng.integers(0, len(b)))] = int(rng.integers(0x80, 0x100))
        elif k == 2:
            b = b[:-1]
        cases.append(bytes(b))
    return cases


def _layout(rng, cases, max_pad):
    """Plain text regions separated by 0..max_pad arbitrary non-ASCII bytes, masked with
    random keys and phases (the XOR is an involution: masking = the oracle unmask)."""
    regions, pos, parts = [], int(rng.integers(0, 16)), []
    parts.append(rng.integers(0x80, 0x100, pos, dtype=np.uint8).tobytes())
    for c in cases:
        regions.append((pos, len(c), int(rng.integers(0, 2**32)), int(rng.integers(0, 4))))
        parts.append(c)
        pos += len(c)
        pad = int(rng.integers(0, max_pad + 1))
        parts.append(rng.integers(0x80, 0x100, pad, dtype=np.uint8).tobytes())
        pos += pad
    plain = aligned_host(pos + 32)
    plain[:] = np.frombuffer(b"".join(parts) + b"\xf0" * 32, dtype=np.uint8)[:len(plain)]
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    return plain, oracle_unmask_regions(plain, descs), descs


def _run(ctx, cuda, masked, descs, shift=0):
    dev = torch.from_numpy(np.concatenate([np.zeros(shift, np.uint8), masked])).to(cuda)
    dd = gpu.descs_to_device(descs, cuda)
    ok = torch.full((len(descs),), 7, dtype=torch.uint8, device=cuda)
    gpu.unmask_sorted_utf8(ctx, dev[shift:], dd, len(descs), ok)
    torch.cuda.synchronize()
    return dev[shift:].cpu().numpy(), ok.cpu().numpy()


@pytest.mark.parametrize("max_pad,shift", [(0, 0), (3, 0), (20, 5), (600, 11)])
def test_sorted_utf8_edge_cases(ctx, cuda, max_pad, shift):
    rng = np.random.default_rng(100 + max_pad)
    cases = _cases(rng, 300, 60, (100, 1500))
    plain, masked, descs = _layout(rng, cases, max_pad)
    got, ok = _run(ctx, cuda, masked, descs, shift)
    assert np.array_equal(got, plain)
    exp = np.array([_valid(c) for c in cases])
    assert np.array_equal(ok.astype(bool), exp), np.nonzero(ok.astype(bool) != exp)[0][:10]


@pytest.mark.parametrize("max_pad", [14, 0, 2, 3, 6])
def test_sorted_utf8_long_frames(ctx, cuda, max_pad):
    """Frames of 4-40 KiB (fast-kind units, every unit seam inside a frame),
    0-14 bytes apart, a third of them ending in a truncated sequence (its error
    falls on the bytes after the frame: the frame's own, not the next's)."""
    rng = np.random.default_rng(7 + max_pad)
    cases = _cases(rng, 0, 40, (1000, 12000))
    for i in range(0, len(cases), 3):                    # truncated sequences right at a frame end
        cases[i] = cases[i] + [b"\xc3", b"\xe2\x82", b"\xf0\x9f\x98"][i % 3]
    plain, masked, descs = _layout(rng, cases, max_pad)
    got, ok = _run(ctx, cuda, masked, descs)
    assert np.array_equal(got, plain)
    assert np.array_equal(ok.astype(bool), np.array([_valid(c) for c in cases]))


def test_sorted_utf8_c5_shape(ctx, cuda):
    """BASELINE C5 layout (16 KiB TEXT frames, 8-B headers, ~1 % invalid), 4096 frames:
    flags vs the generator's, bytes and flags vs the two-pass path."""
    wire, descs, ok_exp = gpu.config_c5(seed=5, n_frames=4096)
    got, ok = _run(ctx, cuda, wire, descs)
    assert np.array_equal(ok, np.asarray(ok_exp, dtype=np.uint8)[:len(descs)])
    assert (ok == 0).sum() > 0
    dev = torch.from_numpy(wire).to(cuda)
    dd = gpu.descs_to_device(descs, cuda)
    ok2 = torch.zeros(len(descs), dtype=torch.uint8, device=cuda)
    gpu.unmask_sorted(ctx, dev, dd, len(descs))
    gpu.validate_utf8(ctx, dev, dd, len(descs), ok2)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), got)
    assert np.array_equal(ok2.cpu().numpy(), ok)


@pytest.mark.parametrize("pipe", [0, 1, 2])
def test_sorted_utf8_both_variants(ctx, cuda, pipe):
    """The plain, software-pipelined and early-load fused kernels give the same bytes and flags."""
    from flashws_amd import lib
    old = lib().fws_internal_set_sorted_utf8_pipe(pipe)
    try:
        rng = np.random.default_rng(300 + pipe)
        cases = _cases(rng, 200, 40, (100, 9000))
        plain, masked, descs = _layout(rng, cases, 30)
        got, ok = _run(ctx, cuda, masked, descs, 3)
        assert np.array_equal(got, plain)
        assert np.array_equal(ok.astype(bool), np.array([_valid(c) for c in cases]))
    finally:
        lib().fws_internal_set_sorted_utf8_pipe(old)


def test_sorted_utf8_unreserved_ctx_wide_frames(cuda):
    """A context without a stream reservation sizes its seam words from 4 KiB per
    frame; TEXT frames of 64 KiB-1 MiB span far more units than that, so most
    units have no seam words: the kernels must stay inside the buffer (units
    past it leave their seam bytes to the stream reads of the seam check) and the
    flags must still be exact at every unit seam."""
    rng = np.random.default_rng(11)
    cases = []
    for n in (70000, 1 << 20, 200000, 65536):
        s = "".join(chr(int(c)) for c in rng.integers(0x20, 0x10FFFF, n // 3) if not 0xD800 <= int(c) <= 0xDFFF)
        b = bytearray(s.encode())[:n]
        while b and (b[-1] & 0xC0) == 0x80:     # cut back to a whole character
            b = b[:-1]
        if b and b[-1] >= 0xC0:
            b = b[:-1]
        cases.append(bytes(b))
    # one invalid byte placed right at a 4 KiB unit seam of the second frame
    bad = bytearray(cases[1])
    bad[4096 * 9 + 1] = 0xFF
    cases.append(bytes(bad))
    plain, masked, descs = _layout(rng, cases, 7)
    c = gpu.Ctx(0)                                        # no reservation
    try:
        got, ok = _run(c, cuda, masked, descs)
    finally:
        c.close()
    assert np.array_equal(got, plain)
    assert np.array_equal(ok.astype(bool), np.array([_valid(x) for x in cases]))


def test_sorted_utf8_invalid_bytes_at_seams(ctx, cuda):
    """An invalid byte (C0, C1, F5, F8, FF) or a lead whose sequence is cut, at
    every offset -4..+4 around a 4 KiB unit seam and as a frame's last byte: the
    table form flags an invalid byte at the byte after it, which may be the next
    unit's first bytes (k_utf8_seam_sorted's) or the 3 zero bytes past the frame."""
    rng = np.random.default_rng(41)
    base = "".join(chr(int(c)) for c in rng.integers(0x20, 0x7F, 30000)).encode()   # ASCII: byte = char
    cases = []
    for bad in (b"\xc0", b"\xc1", b"\xf5", b"\xf8", b"\xff", b"\xe2\x82", b"\xc3"):
        for seam in (4096, 8192, 12288):
            for d in range(-4, 5):
                b = bytearray(base[:20000])
                # the frame starts 16-B aligned plus the layout's offset; seams are relative to
                # the batch origin, so cover them by position within the frame as well
                at = seam + d
                b[at:at + len(bad)] = bad
                cases.append(bytes(b))
        cases.append(bytes(base[:9000]) + bad)                        # the frame's last byte(s)
        cases.append(bytes(base[:4096 - len(bad)]) + bad)            # ends right before a seam
        cases.append(b"\xe2\x82\xac" * 1365 + bad)                    # ends at 4095 + len(bad)
    plain, masked, descs = _layout(rng, cases, 0)
    got, ok = _run(ctx, cuda, masked, descs)
    assert np.array_equal(got, plain)
    exp = np.array([_valid(c) for c in cases])
    assert not exp.any()
    assert np.array_equal(ok.astype(bool), exp), np.nonzero(ok.astype(bool) != exp)[0][:10]


@pytest.mark.parametrize("lead", [0, 1, 2, 3, 17])
@pytest.mark.parametrize("first", [b"\x80abc", b"\xc0\x80", b"\xbf" * 5, b"ok\xff"])
def test_sorted_utf8_first_bytes_of_batch(ctx, cuda, lead, first):
    """The batch's first region starting 0-2 bytes past a 16-B boundary: its
    first bytes are unit 0's bytes 0..2, whose error flags the unmask kernel
    leaves to the seam pass (they have no left context in the unit). An
    invalid byte there must still clear the region's flag."""
    rng = np.random.default_rng(lead * 7 + len(first))
    cases = [first, "héllo".encode(), b"\x80", b"fine"]
    regions, pos, parts = [], lead, [bytes(lead)]
    for c in cases:
        regions.append((pos, len(c), int(rng.integers(0, 2**32)), int(rng.integers(0, 4))))
        parts.append(c)
        pos += len(c) + 3
        parts.append(b"\x00\x00\x00")
    plain = aligned_host(pos + 32)
    plain[:] = np.frombuffer(b"".join(parts) + bytes(32), dtype=np.uint8)[:len(plain)]
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    masked = oracle_unmask_regions(plain, descs)
    got, ok = _run(ctx, cuda, masked, descs)
    assert np.array_equal(got, plain)
    exp = np.array([_valid(c) for c in cases])
    assert np.array_equal(ok.astype(bool), exp), (ok, exp)
