"""GPU: fws_decode_engine (batched stream decode, include/fws_gpu.h). Every
job's unmasked bytes, frame list, result and UTF-8 flags must equal
fws_gpu_decode_stream on that job alone -- the engine only reorders launches
over its workspaces and two streams, in each schedule: whole decodes
alternating over the streams (the default) and the split-phase schedule (scans
on one stream, resolve + unmask on the other), with or without a CU partition. The single-stream decode is itself pinned to the
oracle and the reference's vectors (test_gpu_decode.py, test_gpu_configs.py);
here the jobs mix random frame streams, protocol errors, incomplete tails,
streams shorter than one tile, empty streams and generator batches, in runs
longer than the three workspaces so every slot is reused."""
import numpy as np
import pytest
import torch

from flashws_amd import _lib, gpu
from test_gpu_mux import _random_stream

pytestmark = pytest.mark.gpu


def _streams(rng, n):
    out = []
    for i in range(n):
        kind = i % 6
        if kind == 0:
            s = _random_stream(rng, int(rng.integers(20, 200)))
        elif kind == 1:                                  # a protocol error part-way
            s = bytearray(_random_stream(rng, int(rng.integers(20, 120))))
            s += bytes([0xF2, 0x85]) + bytes(rng.integers(0, 256, 9, dtype=np.uint8))   # RSV set
            s += _random_stream(rng, 5)
            s = bytes(s)
        elif kind == 2:                                  # an incomplete trailing header
            s = _random_stream(rng, int(rng.integers(5, 50))) + bytes([0x82, 0xFE, 0x10])
        elif kind == 3:                                  # shorter than a tile + halo
            s = _random_stream(rng, 3)[:int(rng.integers(1, 2000))]
        elif kind == 4:
            s = b""
        else:                                            # a generator batch (mixed sizes)
            w, _, _ = gpu.gen_batch(gpu.GEN_MIXED, seed=int(rng.integers(0, 1 << 30)), opcode=2,
                                    payload_min=1, payload_max=70000, target_bytes=int(rng.integers(1, 6)) << 20)
            s = w.tobytes()
        out.append(s)
    return out


def _dev(data, cuda):
    t = torch.zeros(max(len(data), 1) + 64, dtype=torch.uint8, device=cuda)
    if data:
        t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(cuda)
    return t


def _run_reference(ctx, streams, cap, cuda, utf8):
    outs = []
    for s in streams:
        w = _dev(s, cuda)
        fr = torch.zeros(cap * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=cuda)
        rs = torch.zeros(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=cuda)
        ok = torch.zeros(cap, dtype=torch.uint8, device=cuda) if utf8 else None
        rc, _, _, _ = gpu.decode_stream(ctx, w, cap, frames=fr, result=rs, utf8_ok=ok, n=len(s))
        assert rc == 0
        outs.append((w, fr, rs, ok))
    torch.cuda.synchronize()
    return outs


def _compare(got, exp, n_bytes):
    (gw, gf, gr, go), (ew, ef, er, eo) = got, exp
    assert torch.equal(gw[:n_bytes], ew[:n_bytes])
    assert torch.equal(gr, er)
    nf = int(gpu.read_result(er)["n_frames"])
    k = min(nf, gf.numel() // gpu.FRAME_INFO.itemsize) * gpu.FRAME_INFO.itemsize
    assert torch.equal(gf[:k], ef[:k])
    if go is not None:
        m = min(nf, go.numel())
        assert torch.equal(go[:m], eo[:m])


SCHEDULES = [(0, 0), (1, 0), (1, 96)]               # (mode, scan_cus): default, split phases, + CU partition


@pytest.mark.parametrize("sched", SCHEDULES, ids=["alternate", "split", "split_cu96"])
@pytest.mark.parametrize("utf8", [False, True], ids=["plain", "utf8"])
def test_engine_matches_single_decodes(ctx, cuda, sched, utf8):
    mode, scan_cus = sched
    rng = np.random.default_rng(4040 + 7 * mode + scan_cus + utf8)
    streams = _streams(rng, 14)
    cap = 1 << 16
    exp = _run_reference(ctx, streams, cap, cuda, utf8)
    eng = gpu.DecodeEngine(0, max_frames=cap, max_stream_bytes=8 << 20, mode=mode, scan_cus=scan_cus)
    got, jobs = [], []
    for s in streams:
        w = _dev(s, cuda)
        fr = torch.zeros(cap * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=cuda)
        rs = torch.zeros(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=cuda)
        ok = torch.zeros(cap, dtype=torch.uint8, device=cuda) if utf8 else None
        got.append((w, fr, rs, ok))
        jobs.append((w[:max(len(s), 0)] if len(s) else w[:0], cap, fr, rs) + ((ok,) if utf8 else ()))
    assert eng.run(jobs) == 0
    torch.cuda.synchronize()
    for g, e, s in zip(got, exp, streams):
        _compare(g, e, len(s))
    eng.close()


@pytest.mark.parametrize("sched", SCHEDULES, ids=["alternate", "split", "split_cu96"])
def test_engine_repeated_runs_and_growth(ctx, cuda, sched):
    """Several runs on one engine (workspaces reused across runs), the second
    with jobs larger than the reservation (the engine drains and grows)."""
    rng = np.random.default_rng(77)
    cap = 1 << 15
    eng = gpu.DecodeEngine(0, max_frames=1024, max_stream_bytes=1 << 20, mode=sched[0], scan_cus=sched[1])
    for run in range(3):
        streams = _streams(rng, 7 + run)
        if run == 1:
            w, _, _ = gpu.config_c3(seed=5, target=24 << 20)
            streams.append(w.tobytes())
        exp = _run_reference(ctx, streams, cap, cuda, False)
        got = [(_dev(s, cuda), torch.zeros(cap * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=cuda),
                torch.zeros(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=cuda), None) for s in streams]
        jobs = [(g[0][:len(s)], cap, g[1], g[2]) for g, s in zip(got, streams)]
        assert eng.run(jobs) == 0
        torch.cuda.synchronize()
        for g, e, s in zip(got, exp, streams):
            _compare(g, e, len(s))
    eng.close()


def test_engine_c3_batches(ctx, cuda):
    """Eight C3 batches (256 MiB each would not fit the test budget: 32 MiB
    slices of the C3 generator) through the default engine."""
    cap = 1 << 16
    streams = [gpu.config_c3(seed=60 + i, target=32 << 20)[0].tobytes() for i in range(8)]
    exp = _run_reference(ctx, streams, cap, cuda, False)
    eng = gpu.DecodeEngine(0, max_frames=cap, max_stream_bytes=32 << 20)
    got = [(_dev(s, cuda), torch.zeros(cap * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=cuda),
            torch.zeros(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=cuda), None) for s in streams]
    assert eng.run([(g[0][:len(s)], cap, g[1], g[2]) for g, s in zip(got, streams)]) == 0
    torch.cuda.synchronize()
    for g, e, s in zip(got, exp, streams):
        _compare(g, e, len(s))
        assert int(gpu.read_result(e[2])["status"]) == 0
    eng.close()


def test_engine_rejects_bad_jobs_before_queueing(cuda):
    eng = gpu.DecodeEngine(0)
    w = torch.zeros(4096 + 64, dtype=torch.uint8, device=cuda)
    fr = torch.zeros(64 * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=cuda)
    rs = torch.zeros(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=cuda)
    good = (w[:4096], 64, fr, rs)
    bad = (w[1:4097], 64, fr, rs)                        # not 16-B aligned
    assert eng.run([good, bad]) == _lib.FWS_ERR_INVALID
    torch.cuda.synchronize()
    assert int(rs.sum()) == 0                            # nothing ran, not even the good job
    with pytest.raises(_lib.FwsError):
        gpu.DecodeEngine(0, mode=1, scan_cus=100000)      # more CUs than the device has
    eng.close()
