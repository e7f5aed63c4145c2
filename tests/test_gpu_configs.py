"""GPU parity on the BASELINE configs at full size, against digests the REAL
reference produced (tests/golden/configs.json, tests/golden/make_golden.py:
the compiled flashws OnRecvData over 2 MiB reads of the same wire bytes).

For each config the generator's wire bytes are pinned by their SHA-256, the
device path unmasks them, and the unmasked stream's SHA-256 must equal the
reference's. Frame lists are checked against the generator's descriptors;
UTF-8 flags (C5) against Python's strict decoder (digest in the fixture, the
reference has no UTF-8 validation). Reassembly (C4) is pinned to the
concatenation of the reference-unmasked payloads.

* C2: 65 536 x 4 KiB        fws_gpu_decode_stream, fws_gpu_unmask_sorted
* C3: mixed 64 B..64 KiB    fws_gpu_decode_stream, fws_gpu_unmask_sorted, fws_gpu_unmask_batch
* C4: 256 MiB fragmented    fws_gpu_decode_stream, fws_gpu_unmask_gather
* C5: 16 384 and 262 144 (4 GiB, one GPU's share) x 16 KiB TEXT:
                            fws_gpu_decode_stream(utf8), fws_gpu_unmask_sorted_utf8
"""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from flashws_amd import _lib, gpu

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "configs.json")))

GEN = {
    "C2": lambda: gpu.config_c2(),
    "C3": lambda: gpu.config_c3(),
    "C4": lambda: gpu.config_c4(),
    "C5_16k_frames": lambda: gpu.config_c5(n_frames=16384),
    "C5_full_per_gpu": lambda: gpu.config_c5(),
}


def sha(t):
    h = hashlib.sha256()
    a = t.cpu().numpy() if isinstance(t, torch.Tensor) else t
    step = 1 << 28
    for o in range(0, len(a), step):
        h.update(memoryview(a[o:o + step]))
    return h.hexdigest()


def _gen(name):
    assert name in GOLDEN, f"no golden digest for {name} in tests/golden/configs.json"
    g = GOLDEN[name]
    wire, descs, ok = GEN[name]()
    assert len(wire) == g["wire_bytes"] and len(descs) == g["frames"]
    assert int(descs["payload_len"].sum()) == g["payload_bytes"]
    assert sha(wire) == g["wire_sha256"], "generator drifted from the golden wire bytes"
    return g, wire, descs, ok


def _check_frames(ctx, fr, res, descs):
    r = gpu.read_result(res)
    assert int(r["status"]) == 0 and int(r["n_frames"]) == len(descs)
    assert int(r["consumed"]) == int(descs["payload_off"][-1] + descs["payload_len"][-1])
    f = gpu.read_frames(fr, len(descs))
    assert np.array_equal(f["hdr_off"] + f["hdr_len"], descs["payload_off"])
    assert np.array_equal(f["payload_len"], descs["payload_len"])
    assert np.array_equal(f["key"], descs["key"])


@pytest.mark.parametrize("name", ["C2", "C3", "C4", "C5_16k_frames"])
def test_decode_stream_full_config(ctx, cuda, name):
    g, wire, descs, ok = _gen(name)
    dev = torch.from_numpy(wire).to(cuda)
    utf8 = name.startswith("C5")
    okd = torch.zeros(len(descs) + 16, dtype=torch.uint8, device=cuda) if utf8 else None
    rc, fr, res, _ = gpu.decode_stream(ctx, dev, len(descs) + 16, utf8_ok=okd)
    assert rc == 0
    torch.cuda.synchronize()
    _check_frames(ctx, fr, res, descs)
    assert sha(dev) == g["unmasked_sha256"]
    if utf8:
        flags = okd[:len(descs)].cpu().numpy()
        assert hashlib.sha256(flags.tobytes()).hexdigest() == g["utf8_ok_sha256_python_strict"]
        assert int(len(flags) - flags.sum()) == g["utf8_invalid_frames"]


@pytest.mark.parametrize("name", ["C2", "C3", "C5_16k_frames"])
@pytest.mark.parametrize("path", ["sorted", "batch", "batch_permuted", "any_permuted"])
def test_descriptor_unmask_full_config(ctx, cuda, name, path):
    """Every descriptor-mode entry point on the full config against the golden
    digest of the reference-unmasked bytes; `*_permuted`: the descriptor array
    shuffled (any order is allowed), planned (chunk space) or by the opt-in
    one-launch form (fws_internal_set_unmask_any)."""
    g, wire, descs, ok = _gen(name)
    dev = torch.from_numpy(wire).to(cuda)
    if path.endswith("permuted"):
        descs = descs[np.random.default_rng(9).permutation(len(descs))]
    dd = gpu.descs_to_device(descs, cuda)
    if path == "sorted":
        gpu.unmask_sorted(ctx, dev, dd, len(descs))
    else:
        L = _lib.lib()
        old = L.fws_internal_set_unmask_any(1 if path == "any_permuted" else 0)
        try:
            gpu.unmask_batch(ctx, dev, dd, len(descs))
            torch.cuda.synchronize()
        finally:
            L.fws_internal_set_unmask_any(old)
    assert sha(dev) == g["unmasked_sha256"]


def test_gather_full_c4(ctx, cuda):
    """Reassembly of the 256 MiB fragmented message: the concatenation of the
    reference-unmasked payloads."""
    g, wire, descs, ok = _gen("C4")
    src = torch.from_numpy(wire).to(cuda)
    total = int(descs["payload_len"].sum())
    dst = torch.zeros(total + 64, dtype=torch.uint8, device=cuda)
    gpu.unmask_gather(ctx, dst, src, gpu.descs_to_device(descs, cuda), len(descs))
    rc, fr, res, _ = gpu.decode_stream(ctx, src, len(descs) + 16)       # in place: the reference's bytes
    assert rc == 0
    torch.cuda.synchronize()
    assert sha(src) == g["unmasked_sha256"]
    idx = torch.cat([torch.arange(int(o), int(o) + int(n), device=cuda, dtype=torch.int64)
                     for o, n in zip(descs["payload_off"], descs["payload_len"])])
    assert torch.equal(dst[:total], src[idx])
    assert int(dst[total:].sum()) == 0


def test_c5_full_per_gpu_share(ctx, cuda):
    """One GPU's share of the 8-GPU config: 262 144 x 16 KiB TEXT frames (4 GiB).
    Unmasked bytes vs the reference's OnRecvData digest, flags vs Python's
    strict decoder, through both the stream decode and the descriptor path."""
    g, wire, descs, ok = _gen("C5_full_per_gpu")
    n = len(descs)
    dev = torch.from_numpy(wire).to(cuda)
    del wire
    c = gpu.Ctx(0, max_frames=n + 64, max_stream_bytes=dev.numel())
    okd = torch.zeros(n + 64, dtype=torch.uint8, device=cuda)
    rc, fr, res, _ = gpu.decode_stream(c, dev, n + 64, utf8_ok=okd)
    assert rc == 0
    torch.cuda.synchronize()
    _check_frames(c, fr, res, descs)
    assert sha(dev) == g["unmasked_sha256"]
    flags = okd[:n].cpu().numpy()
    assert hashlib.sha256(flags.tobytes()).hexdigest() == g["utf8_ok_sha256_python_strict"]
    assert np.array_equal(flags, ok)
    # re-mask (XOR involution), then the descriptor path
    dd = gpu.descs_to_device(descs, cuda)
    gpu.unmask_sorted(c, dev, dd, n)
    ok2 = torch.zeros(n, dtype=torch.uint8, device=cuda)
    gpu.unmask_sorted_utf8(c, dev, dd, n, ok2)
    torch.cuda.synchronize()
    assert sha(dev) == g["unmasked_sha256"]
    assert hashlib.sha256(ok2.cpu().numpy().tobytes()).hexdigest() == g["utf8_ok_sha256_python_strict"]
    c.close()
