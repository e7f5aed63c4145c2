"""GPU parity: device XOR unmask (fws_gpu_mask / fws_gpu_unmask_batch) vs the
oracle's restatement of WSMaskBytesFast (crypto/ws_mask.h:175-197), bit-exact.
Sweeps the alignment/length/phase space the reference's own test_mask.cpp
(tests/test-utils/test_mask.cpp:148-177) only samples at offset 1."""
import numpy as np
import pytest
import torch

import orc
from flashws_amd import _lib, gpu

pytestmark = pytest.mark.gpu

ALIGN = 256


def aligned_host(n):
    raw = np.zeros(n + ALIGN, dtype=np.uint8)
    off = (-raw.ctypes.data) % ALIGN
    return raw[off:off + n]


def oracle_unmask_regions(buf, descs):
    out = buf.copy()
    for d in descs:
        o, n, k, ph = int(d["payload_off"]), int(d["payload_len"]), int(d["key"]), int(d["phase"])
        key = orc.orc().orc_rotr32(k, 8 * ph)   # phase == RotateR(key, 8*phase) (w_socket.h:758)
        orc.orc_mask("ws_mask_fast", out, key, o, n)
    return out


@pytest.fixture(params=["any", "plan"])
def batch_path(request):
    """fws_gpu_unmask_batch's two forms: k_plan + k_unmask_desc (the default)
    and one launch, descriptor-major (k_unmask_any + queued pieces; opt-in
    through fws_internal_set_unmask_any(1))."""
    L = _lib.lib()
    old = L.fws_internal_set_unmask_any(1 if request.param == "any" else 0)
    yield request.param
    L.fws_internal_set_unmask_any(old)


@pytest.fixture(params=[0, 3], ids=["lookup_first", "xcd_runs"])
def sorted_kernel(request):
    """fws_gpu_unmask_sorted's one-launch forms: k_unmask_sorted (owner
    lookup, then the unit's loads) and the same kernel with the XCD-run
    workgroup order (a bijection on any grid: the C2 shape covers full groups
    of 64 workgroups and a partial last one)."""
    L = _lib.lib()
    old = L.fws_internal_set_sorted_early(request.param)
    yield request.param
    L.fws_internal_set_sorted_early(old)


@pytest.fixture
def planned():
    """The planned form only (the tests that read the plan's mode)."""
    L = _lib.lib()
    old = L.fws_internal_set_unmask_any(0)
    yield
    L.fws_internal_set_unmask_any(old)


def run_batch(ctx, host, descs, cuda):
    dev = torch.from_numpy(host.copy()).to(cuda)
    dd = gpu.descs_to_device(descs, cuda)
    gpu.unmask_batch(ctx, dev, dd, len(descs))
    torch.cuda.synchronize()
    return dev.cpu().numpy()


def test_mask_single_sweep(cuda):
    """fws_gpu_mask over offsets 0..63 x lens 0..300 (+ big) x 2 keys."""
    rng = np.random.default_rng(1)
    base = rng.integers(0, 256, 70000, dtype=np.uint8)
    dev = torch.from_numpy(base).to(cuda)
    ptr_mod = dev.data_ptr() % 256
    assert ptr_mod == 0
    lens = list(range(0, 301, 7)) + [511, 512, 513, 2047, 2048, 2049, 4093, 4096, 16384, 65535]
    for key in (0xA1B2C3D4, 0x00000001):
        for off in range(0, 64, 3):
            for n in lens:
                d = dev.clone()
                gpu.ws_mask_bytes_fast(d, key, off, n)
                got = d.cpu().numpy()
                exp = base.copy()
                orc.orc_mask("ws_mask_fast", exp, key, off, n)
                assert np.array_equal(got, exp), (hex(key), off, n)


def test_unmask_batch_alignment_sweep(ctx, cuda, batch_path):
    """One batch: every (offset mod 64, len 0..600, phase) region, packed with gaps."""
    rng = np.random.default_rng(2)
    regions = []
    pos = 0
    for ln in range(0, 601):
        for sh in (0, 1, 5, 13, 31, 47, 63):
            pos = (pos + 63) // 64 * 64 + sh
            regions.append((pos, ln, int(rng.integers(0, 2**32)), int(rng.integers(0, 4))))
            pos += ln + int(rng.integers(0, 9))
    host = aligned_host(pos + 64)
    host[:] = rng.integers(0, 256, len(host), dtype=np.uint8)
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    order = rng.permutation(len(descs))          # any order is allowed
    descs = descs[order]
    got = run_batch(ctx, host, descs, cuda)
    exp = oracle_unmask_regions(host, descs)
    assert np.array_equal(got, exp)


def test_unmask_batch_adjacent_regions(ctx, cuda, batch_path):
    """Regions sharing 16-B chunks (1..15-byte gaps and zero gaps)."""
    rng = np.random.default_rng(3)
    regions, pos = [], 3
    for i in range(5000):
        ln = int(rng.integers(0, 40))
        regions.append((pos, ln, int(rng.integers(0, 2**32)), int(rng.integers(0, 4))))
        pos += ln + int(rng.integers(0, 3))
    host = aligned_host(pos + 32)
    host[:] = rng.integers(0, 256, len(host), dtype=np.uint8)
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    got = run_batch(ctx, host, descs, cuda)
    assert np.array_equal(got, oracle_unmask_regions(host, descs))


@pytest.mark.parametrize("n_frames", [1, 7, 4096])
def test_unmask_batch_c2_shape(ctx, cuda, batch_path, n_frames):
    wire, descs, _ = gpu.config_c2(seed=7, n_frames=n_frames)
    got = run_batch(ctx, wire, descs, cuda)
    exp = wire.copy()
    ret, frames, _, consumed = orc.orc_decode_stream(exp)
    assert ret == 0 and consumed == len(wire) and len(frames) == n_frames
    assert np.array_equal(got, exp)


def test_unmask_batch_c2_full(ctx, cuda, batch_path):
    """BASELINE config 2 at full size: 65 536 x 4 KiB, seed 42, bit-exact."""
    wire, descs, _ = gpu.config_c2()
    got = run_batch(ctx, wire, descs, cuda)
    exp = wire.copy()
    ret, frames, _, consumed = orc.orc_decode_stream(exp)
    assert ret == 0 and len(frames) == 65536
    assert np.array_equal(got, exp)


def test_unmask_batch_mixed(ctx, cuda, batch_path):
    wire, descs, _ = gpu.config_c3(seed=5, target=16 << 20)
    got = run_batch(ctx, wire, descs, cuda)
    exp = wire.copy()
    ret, frames, _, _ = orc.orc_decode_stream(exp)
    assert ret == 0 and len(frames) == len(descs)
    assert np.array_equal(got, exp)


def test_unmask_batch_involution(ctx, cuda, batch_path):
    """Size-independent property at full C2 size: two passes restore the input."""
    wire, descs, _ = gpu.config_c2(seed=11)
    dev = torch.from_numpy(wire).to(cuda)
    dd = gpu.descs_to_device(descs, cuda)
    gpu.unmask_batch(ctx, dev, dd, len(descs))
    gpu.unmask_batch(ctx, dev, dd, len(descs))
    torch.cuda.synchronize()
    assert torch.equal(dev.cpu(), torch.from_numpy(wire))


# ---- k_plan modes: byte space (sorted, disjoint payloads) vs chunk space ----

def _rand_regions(rng, n, max_len, max_gap, start=5):
    regions, pos = [], start
    for _ in range(n):
        ln = int(rng.integers(0, max_len + 1))
        regions.append((pos, ln, int(rng.integers(0, 2**32)), int(rng.integers(0, 4))))
        pos += ln + int(rng.integers(0, max_gap + 1))
    return regions, pos


@pytest.mark.parametrize("permute", [False, True])
def test_plan_mode_sorted_vs_permuted(ctx, cuda, planned, permute):
    """The same regions sorted take the byte-space run, permuted the chunk-space
    run; both bit-exact (alignment sweep layout, gaps up to 70 B)."""
    rng = np.random.default_rng(21)
    regions, pos = [], 0
    for ln in range(0, 400):
        for sh in (0, 3, 9, 15, 40):
            pos = (pos + 63) // 64 * 64 + sh
            regions.append((pos, ln, int(rng.integers(0, 2**32)), int(rng.integers(0, 4))))
            pos += ln + int(rng.integers(0, 9))
    host = aligned_host(pos + 64)
    host[:] = rng.integers(0, 256, len(host), dtype=np.uint8)
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    if permute:
        descs = descs[rng.permutation(len(descs))]
    got = run_batch(ctx, host, descs, cuda)
    assert gpu.plan_mode(ctx)["byte_space"] == (0 if permute else 1)
    assert np.array_equal(got, oracle_unmask_regions(host, descs))


@pytest.mark.parametrize("where", [10, 2500, 4990], ids=["first_block", "middle", "last_block"])
def test_plan_partly_sorted(ctx, cuda, planned, where):
    """Sorted except for one swapped pair in one 1024-frame plan block: the
    batch is planned in chunk space (k_plan writes byte-space records only while
    the blocks up to its own are sorted, so some were written before the
    unsorted block and are never read) and the result is bit-exact."""
    rng = np.random.default_rng(33 + where)
    regions, pos = _rand_regions(rng, 5000, 600, 20)
    regions[where], regions[where + 1] = regions[where + 1], regions[where]
    host = aligned_host(pos + 64)
    host[:] = rng.integers(0, 256, len(host), dtype=np.uint8)
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    got = run_batch(ctx, host, descs, cuda)
    assert gpu.plan_mode(ctx)["byte_space"] == 0
    assert np.array_equal(got, oracle_unmask_regions(host, descs))


@pytest.mark.parametrize("n,max_len,max_gap", [(1, 5, 0), (3, 20, 3), (1023, 64, 2), (1024, 64, 2),
                                                (1025, 64, 2), (70000, 30, 3), (300000, 12, 1)])
def test_plan_lookback_many_blocks(ctx, cuda, planned, n, max_len, max_gap):
    """Frame counts around the 1024-frame plan block and far past it (the
    look-back runs over up to 293 blocks), tiny frames with 0-3-byte gaps."""
    rng = np.random.default_rng(n)
    regions, pos = _rand_regions(rng, n, max_len, max_gap)
    host = aligned_host(pos + 32)
    host[:] = rng.integers(0, 256, len(host), dtype=np.uint8)
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    got = run_batch(ctx, host, descs, cuda)
    assert gpu.plan_mode(ctx)["byte_space"] == 1
    assert np.array_equal(got, oracle_unmask_regions(host, descs))


def test_plan_large_frames_block_fill(ctx, cuda, planned):
    """Frames spanning many 4 KiB units (unit maps filled by the whole block):
    16 MiB + 1 MiB + odd sizes, sorted then permuted."""
    rng = np.random.default_rng(31)
    lens = [16 << 20, 3, 1 << 20, 4097, 12345, 0, 65536 * 3 + 7, 9]
    regions, pos = [], 7
    for ln in lens:
        regions.append((pos, ln, int(rng.integers(0, 2**32)), int(rng.integers(0, 4))))
        pos += ln + 14
    host = aligned_host(pos + 32)
    host[:] = rng.integers(0, 256, len(host), dtype=np.uint8)
    for perm in (False, True):
        descs = np.array(regions, dtype=gpu.FRAME_DESC)
        if perm:
            descs = descs[rng.permutation(len(descs))]
        got = run_batch(ctx, host, descs, cuda)
        assert gpu.plan_mode(ctx)["byte_space"] == (0 if perm else 1)
        assert np.array_equal(got, oracle_unmask_regions(host, descs)), perm


def test_plan_sparse_batch_takes_chunk_space(ctx, cuda, planned):
    """Sorted but sparse payloads (64 B every 1 MiB) stay in chunk space."""
    rng = np.random.default_rng(41)
    regions = [(i * (1 << 20) + 3, 64, int(rng.integers(0, 2**32)), 0) for i in range(64)]
    host = aligned_host(64 << 20)
    host[:] = rng.integers(0, 256, len(host), dtype=np.uint8)
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    got = run_batch(ctx, host, descs, cuda)
    assert gpu.plan_mode(ctx)["byte_space"] == 0
    assert np.array_equal(got, oracle_unmask_regions(host, descs))


def test_plan_reused_across_buffers(ctx, cuda):
    """unmask_plan on one buffer, unmask_run on another of the same alignment
    (the plan is base-relative), C3-shaped mixed frames."""
    wire, descs, _ = gpu.config_c3(seed=9, target=8 << 20)
    a = torch.from_numpy(wire).to(cuda)
    b = torch.from_numpy(wire).to(cuda)
    dd = gpu.descs_to_device(descs, cuda)
    gpu.unmask_plan(ctx, a, dd, len(descs))
    gpu.unmask_run(ctx, b, dd, len(descs))
    torch.cuda.synchronize()
    assert gpu.plan_mode(ctx)["byte_space"] == 1
    exp = wire.copy()
    orc.orc_decode_stream(exp)
    assert np.array_equal(b.cpu().numpy(), exp)
    assert torch.equal(a.cpu(), torch.from_numpy(wire))


# ---- fws_gpu_unmask_sorted: one launch, no plan (sorted, disjoint regions) ----

def run_sorted(ctx, host, descs, cuda, base_shift=0):
    """Unmask through fws_gpu_unmask_sorted; base_shift moves dev_base off the
    allocation's alignment (descriptor offsets are base-relative)."""
    dev = torch.from_numpy(np.concatenate([np.zeros(base_shift, np.uint8), host])).to(cuda)
    dd = gpu.descs_to_device(descs, cuda)
    gpu.unmask_sorted(ctx, dev[base_shift:], dd, len(descs))
    torch.cuda.synchronize()
    return dev[base_shift:].cpu().numpy()


@pytest.mark.parametrize("n_frames", [1, 2, 7, 4096, 65536])
def test_sorted_c2_shape(ctx, cuda, sorted_kernel, n_frames):
    """BASELINE C2 layout (65 536 at full size): interpolation guesses hit."""
    wire, descs, _ = gpu.config_c2(seed=17, n_frames=n_frames)
    got = run_sorted(ctx, wire, descs, cuda)
    exp = wire.copy()
    ret, frames, _, _ = orc.orc_decode_stream(exp)
    assert ret == 0 and len(frames) == n_frames
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("shift", [1, 3, 8, 15])
def test_sorted_unaligned_base(ctx, cuda, sorted_kernel, shift):
    wire, descs, _ = gpu.config_c2(seed=19, n_frames=300)
    got = run_sorted(ctx, wire, descs, cuda, base_shift=shift)
    exp = wire.copy()
    orc.orc_decode_stream(exp)
    assert np.array_equal(got, exp)


def test_sorted_mixed_c3(ctx, cuda, sorted_kernel):
    """C3-shaped 64 B-64 KiB frames: guesses miss, binary search finds owners."""
    wire, descs, _ = gpu.config_c3(seed=23, target=16 << 20)
    got = run_sorted(ctx, wire, descs, cuda)
    exp = wire.copy()
    ret, frames, _, _ = orc.orc_decode_stream(exp)
    assert ret == 0 and len(frames) == len(descs)
    assert np.array_equal(got, exp)


def test_sorted_alignment_sweep(ctx, cuda, sorted_kernel):
    rng = np.random.default_rng(29)
    regions, pos = [], 0
    for ln in range(0, 601):
        for sh in (0, 1, 5, 13, 31, 47, 63):
            pos = (pos + 63) // 64 * 64 + sh
            regions.append((pos, ln, int(rng.integers(0, 2**32)), int(rng.integers(0, 4))))
            pos += ln + int(rng.integers(0, 9))
    host = aligned_host(pos + 64)
    host[:] = rng.integers(0, 256, len(host), dtype=np.uint8)
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    assert np.array_equal(run_sorted(ctx, host, descs, cuda), oracle_unmask_regions(host, descs))


@pytest.mark.parametrize("n,max_len,max_gap", [(1, 5, 0), (3, 20, 3), (1025, 64, 2), (70000, 30, 3),
                                                (300000, 12, 1), (5000, 0, 2)])
def test_sorted_tiny_frames(ctx, cuda, sorted_kernel, n, max_len, max_gap):
    """Many frames per 4 KiB unit (slow-kind units), zero-length frames."""
    rng = np.random.default_rng(n + 7)
    regions, pos = _rand_regions(rng, n, max_len, max_gap)
    host = aligned_host(pos + 32)
    host[:] = rng.integers(0, 256, len(host), dtype=np.uint8)
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    assert np.array_equal(run_sorted(ctx, host, descs, cuda), oracle_unmask_regions(host, descs))


def test_sorted_large_and_sparse(ctx, cuda, sorted_kernel):
    """A 16 MiB frame among tiny ones (guesses miss), then a sparse batch
    (64 B every 1 MiB: gap units skipped)."""
    rng = np.random.default_rng(37)
    lens = [16 << 20, 3, 1 << 20, 4097, 12345, 0, 65536 * 3 + 7, 9]
    regions, pos = [], 7
    for ln in lens:
        regions.append((pos, ln, int(rng.integers(0, 2**32)), int(rng.integers(0, 4))))
        pos += ln + 14
    host = aligned_host(pos + 32)
    host[:] = rng.integers(0, 256, len(host), dtype=np.uint8)
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    assert np.array_equal(run_sorted(ctx, host, descs, cuda), oracle_unmask_regions(host, descs))
    regions = [(i * (1 << 20) + 3, 64, int(rng.integers(0, 2**32)), 0) for i in range(64)]
    host = aligned_host(64 << 20)
    host[:] = rng.integers(0, 256, len(host), dtype=np.uint8)
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    assert np.array_equal(run_sorted(ctx, host, descs, cuda), oracle_unmask_regions(host, descs))


def test_sorted_matches_batch_and_involution(ctx, cuda, sorted_kernel, batch_path):
    """Full C2 size: _sorted and _batch agree, and two _sorted passes restore the input."""
    wire, descs, _ = gpu.config_c2(seed=43)
    dev = torch.from_numpy(wire).to(cuda)
    ref = torch.from_numpy(wire).to(cuda)
    dd = gpu.descs_to_device(descs, cuda)
    gpu.unmask_sorted(ctx, dev, dd, len(descs))
    gpu.unmask_batch(ctx, ref, dd, len(descs))
    torch.cuda.synchronize()
    assert torch.equal(dev, ref)
    gpu.unmask_sorted(ctx, dev, dd, len(descs))
    torch.cuda.synchronize()
    assert torch.equal(dev.cpu(), torch.from_numpy(wire))


@pytest.mark.parametrize("shift", [1, 7, 15])
def test_batch_unaligned_base(ctx, cuda, batch_path, shift):
    """fws_gpu_unmask_batch with dev_base off 16-B alignment and the first
    payload within 15 B of it (the byte-space unit origin lies below the base)."""
    wire, descs, _ = gpu.config_c2(seed=47, n_frames=300)
    dev = torch.from_numpy(np.concatenate([np.zeros(shift, np.uint8), wire])).to(cuda)
    dd = gpu.descs_to_device(descs, cuda)
    gpu.unmask_batch(ctx, dev[shift:], dd, len(descs))
    torch.cuda.synchronize()
    assert gpu.plan_mode(ctx)["byte_space"] == 1
    exp = wire.copy()
    orc.orc_decode_stream(exp)
    assert np.array_equal(dev[shift:].cpu().numpy(), exp)
    assert not dev[:shift].cpu().numpy().any()


def test_sorted_early_variant(ctx, cuda):
    """The tuning variant k_unmask_sorted_early (data loads before the lookup)
    on C2, mixed and tiny-frame batches, bit-exact like the default."""
    from flashws_amd import lib
    old = lib().fws_internal_set_sorted_early(1)
    try:
        for wire, descs, _ in (gpu.config_c2(seed=53, n_frames=5000), gpu.config_c3(seed=59, target=4 << 20)):
            exp = wire.copy()
            orc.orc_decode_stream(exp)
            assert np.array_equal(run_sorted(ctx, wire, descs, cuda), exp)
        rng = np.random.default_rng(61)
        regions, pos = _rand_regions(rng, 20000, 30, 3)
        host = aligned_host(pos + 32)
        host[:] = rng.integers(0, 256, len(host), dtype=np.uint8)
        descs = np.array(regions, dtype=gpu.FRAME_DESC)
        assert np.array_equal(run_sorted(ctx, host, descs, cuda), oracle_unmask_regions(host, descs))
    finally:
        lib().fws_internal_set_sorted_early(old)


def test_check_sorted_contract(ctx, cuda):
    """fws_gpu_check_sorted finds the first descriptor that breaks the
    sorted / disjoint contract of fws_gpu_unmask_sorted."""
    wire, descs, _ = gpu.config_c2(n_frames=5000, payload=1000)
    dd = gpu.descs_to_device(descs, cuda)
    assert gpu.check_sorted(ctx, dd, len(descs)) is None
    sw = descs.copy()
    sw[[1234, 1235]] = sw[[1235, 1234]]                # two frames out of order
    assert gpu.check_sorted(ctx, gpu.descs_to_device(sw, cuda), len(sw)) == 1234
    ov = descs.copy()
    ov["payload_len"][3000] += 20                      # overlaps the next region
    assert gpu.check_sorted(ctx, gpu.descs_to_device(ov, cuda), len(ov)) == 3000
    assert gpu.check_sorted(ctx, dd, 0) is None


def test_check_sorted_debug_mode_refuses(cuda, tmp_path):
    """FWS_CHECK_SORTED=1: fws_gpu_unmask_sorted refuses an unsorted batch
    with FWS_ERR_INVALID and writes nothing (a child process: the mode is read
    once per process)."""
    import subprocess
    import sys
    script = tmp_path / "chk.py"
    script.write_text(
        "import sys, numpy as np, torch\n"
        f"sys.path.insert(0, {repr(str(__import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__)))))})\n"
        "from flashws_amd import gpu, _lib\n"
        "wire, d, _ = gpu.config_c2(n_frames=3000, payload=700)\n"
        "dev = torch.device('cuda:0')\n"
        "ctx = gpu.Ctx(0, max_frames=4000, max_stream_bytes=len(wire))\n"
        "w = torch.from_numpy(wire).to(dev)\n"
        "bad = d.copy(); bad[[10, 11]] = bad[[11, 10]]\n"
        "rc = _lib.lib().fws_gpu_unmask_sorted(ctx.h, w.data_ptr(), gpu.descs_to_device(bad, dev).data_ptr(), len(bad),"
        " torch.cuda.current_stream().cuda_stream)\n"
        "torch.cuda.synchronize()\n"
        "same = bool(np.array_equal(w.cpu().numpy(), wire))\n"
        "rc2 = _lib.lib().fws_gpu_unmask_sorted(ctx.h, w.data_ptr(), gpu.descs_to_device(d, dev).data_ptr(), len(d),"
        " torch.cuda.current_stream().cuda_stream)\n"
        "torch.cuda.synchronize()\n"
        "print(rc, same, rc2)\n")
    env = dict(__import__("os").environ, FWS_CHECK_SORTED="1")
    out = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    rc, same, rc2 = out.stdout.split()[-3:]
    assert int(rc) == _lib_invalid() and same == "True" and int(rc2) == 0


def _lib_invalid():
    from flashws_amd import _lib
    return _lib.FWS_ERR_INVALID


# ---- fws_gpu_unmask_batch in one launch: long regions cut into queued pieces ----

@pytest.mark.parametrize("permute", [False, True])
def test_any_long_regions_pieces(ctx, cuda, permute):
    """Regions of 64 KiB +- 1 (the piece size), 1 MiB + odd, 16 MiB, mixed with
    small ones, at odd offsets, sorted and permuted: the first piece by the
    region's wave, the rest from the queue (k_unmask_pieces)."""
    L = _lib.lib()
    old = L.fws_internal_set_unmask_any(1)
    try:
        rng = np.random.default_rng(77 + permute)
        lens = [65535, 65536, 65537, 3, (1 << 20) + 13, 0, 16 << 20, 131072 * 3 + 5, 17, 4096]
        regions, pos = [], 5
        for ln in lens:
            regions.append((pos, ln, int(rng.integers(0, 2**32)), int(rng.integers(0, 4))))
            pos += ln + int(rng.integers(0, 20))
        host = aligned_host(pos + 64)
        host[:] = rng.integers(0, 256, len(host), dtype=np.uint8)
        descs = np.array(regions, dtype=gpu.FRAME_DESC)
        if permute:
            descs = descs[rng.permutation(len(descs))]
        got = run_batch(ctx, host, descs, cuda)
        assert np.array_equal(got, oracle_unmask_regions(host, descs))
    finally:
        L.fws_internal_set_unmask_any(old)


def test_any_queue_overflow(cuda):
    """A context reserved for 1 MiB (a 80-entry piece queue) unmasking 40 regions
    of 1-3 MiB (~1,100 pieces): the queue fills and the waves whose pieces do
    not fit do them themselves. Twice, so the next call's count starts at zero."""
    L = _lib.lib()
    old = L.fws_internal_set_unmask_any(1)
    c = gpu.Ctx(0, max_frames=64, max_stream_bytes=1 << 20)
    try:
        rng = np.random.default_rng(91)
        regions, pos = [], 3
        for _ in range(40):
            ln = int(rng.integers(1 << 20, 3 << 20))
            regions.append((pos, ln, int(rng.integers(0, 2**32)), int(rng.integers(0, 4))))
            pos += ln + int(rng.integers(0, 9))
        host = aligned_host(pos + 64)
        host[:] = rng.integers(0, 256, len(host), dtype=np.uint8)
        descs = np.array(regions, dtype=gpu.FRAME_DESC)
        descs = descs[rng.permutation(len(descs))]
        exp = oracle_unmask_regions(host, descs)
        for _ in range(2):
            assert np.array_equal(run_batch(c, host, descs, cuda), exp)
    finally:
        c.close()
        L.fws_internal_set_unmask_any(old)
