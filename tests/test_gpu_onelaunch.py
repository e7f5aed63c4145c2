"""GPU: the one-launch forms of the output-space batches (no plan launch):
k_gather_one (fws_gpu_unmask_gather for <= 2048 regions: every workgroup keeps
the whole dst prefix in LDS) against the plan + k_gather_fast path and the
oracle (reassembly is pinned to the concatenation of the on_read
parts, tests/new-ws-echo/test_ws_server.cpp:205-206; the key at each region's
phase is RotateR(key, 8 * phase), w_socket.h:758)."""
import numpy as np
import pytest
import torch

import orc
from flashws_amd import _lib, gpu

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["one", "plan", "plan_r05", "one_dpp", "one_w8", "one_w8_dpp"])
def gather_mode(request):
    """k_gather_one, plan + k_gather_fast (r06 kFlat: one load per chunk and
    the neighbour lane's block by DPP; plan_r05: two loads per chunk),
    k_gather_one with one load per chunk + DPP, and k_gather_one_w8 (8 waves
    per SIMD, seam chunks after the full ones) (fws_internal_set_gather_dpp)."""
    L = _lib.lib()
    old = L.fws_internal_set_gather_one(0 if request.param.startswith("plan") else 1)
    old_flat = L.fws_internal_set_gather_flat(0 if request.param == "plan_r05" else 1)
    old_dpp = L.fws_internal_set_gather_dpp({"one_dpp": 1, "one_w8": 2, "one_w8_dpp": 3}.get(request.param, 0))
    yield request.param
    L.fws_internal_set_gather_one(old)
    L.fws_internal_set_gather_flat(old_flat)
    L.fws_internal_set_gather_dpp(old_dpp)


def _regions(shape, rng):
    if shape == "single":
        lens = [123457]
    elif shape == "two":
        lens = [4095, 70001]
    elif shape == "small_2000":
        lens = [int(x) for x in rng.integers(0, 40, 2000)]
    elif shape == "exactly_2048":
        lens = [int(x) for x in rng.choice([0, 1, 15, 16, 17, 4095, 4096, 4097, 9000], 2048)]
    elif shape == "over_2048":
        lens = [int(x) for x in rng.choice([0, 3, 700, 5000], 2049)]
    elif shape == "zeros_at_ends":
        lens = [0, 0, 0] + [int(x) for x in rng.integers(1, 30000, 300)] + [0, 0]
    elif shape == "c4_like":
        lens = [int(2 ** (12 + 8 * rng.random())) for _ in range(600)]
    else:
        raise ValueError(shape)
    offs, pos = [], 5
    for n in lens:
        offs.append(pos)
        pos += n + int(rng.integers(0, 15))
    host = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    regions = [(o, n, int(rng.integers(0, 2**32)), int(rng.integers(0, 4))) for o, n in zip(offs, lens)]
    if shape == "c4_like":
        regions = [regions[i] for i in rng.permutation(len(regions))]     # sources in any order
    return host, regions


@pytest.mark.parametrize("shape", ["single", "two", "small_2000", "exactly_2048", "over_2048", "zeros_at_ends",
                                   "c4_like"])
def test_gather_one_launch(ctx, cuda, gather_mode, shape):
    rng = np.random.default_rng(hash(shape) & 0xFFFF)
    host, regions = _regions(shape, rng)
    descs = np.array(regions, dtype=gpu.FRAME_DESC)
    total = int(descs["payload_len"].sum())
    dst = torch.zeros(total + 48, dtype=torch.uint8, device=cuda)
    src = torch.from_numpy(host).to(cuda)
    gpu.unmask_gather(ctx, dst, src, gpu.descs_to_device(descs, cuda), len(descs))
    exp, w = np.zeros(total, dtype=np.uint8), 0
    for o, n, k, ph in regions:
        seg = host[o:o + n].copy()
        orc.orc_mask("ws_mask_fast", seg, orc.orc().orc_rotr32(k, 8 * ph))
        exp[w:w + n] = seg
        w += n
    got = dst[:total].cpu().numpy()
    assert np.array_equal(got, exp), int(np.flatnonzero(got != exp)[0])
    assert int(dst[total:].sum()) == 0
    assert torch.equal(src.cpu(), torch.from_numpy(host))          # source untouched


def test_gather_one_small_context(cuda, gather_mode):
    """A context reserved for 1 MiB gathering a 40 MiB message: the
    grid is sized from the reservation, its grid-stride loop still covers every
    unit."""
    wire, descs, _ = gpu.config_c4(seed=9, target=40 << 20)
    assert len(descs) <= 2048
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


@pytest.mark.parametrize("threads", [256, 512])
@pytest.mark.parametrize("blocks", [1, 3, 0])
@pytest.mark.parametrize("shape", ["c4_like", "small_2000", "exactly_2048"])
def test_gather_one_grid_sizes(ctx, cuda, shape, blocks, threads):
    """The one-launch gather at a forced grid (fws_internal_set_gather_blocks)
    and workgroup size (fws_internal_set_gather_shape): 1 and 3 workgroups
    leave hundreds of units per wave (past the 64 found up front, one per
    lane: the per-unit probe path), 0 the default 4 x resident."""
    L = _lib.lib()
    old_one, old_blocks = L.fws_internal_set_gather_one(1), L.fws_internal_set_gather_blocks(blocks)
    assert L.fws_internal_set_gather_shape(threads, 0) == 0
    try:
        rng = np.random.default_rng(7 + blocks)
        host, regions = _regions(shape, rng)
        descs = np.array(regions, dtype=gpu.FRAME_DESC)
        total = int(descs["payload_len"].sum())
        dst = torch.zeros(total + 48, dtype=torch.uint8, device=cuda)
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
    finally:
        L.fws_internal_set_gather_one(old_one)
        L.fws_internal_set_gather_blocks(old_blocks)
        L.fws_internal_set_gather_shape(0, 0)
