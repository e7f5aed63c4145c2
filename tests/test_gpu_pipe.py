"""GPU: fws_rx_pipe (batched, pipelined receive over host memory, SURVEY §8f
rank 1) against the oracle's restatement of OnRecvData: every batch's
unmasked bytes, frame list and result bit-exact, with more batches in flight
than slots (back-pressure) and the optional per-frame UTF-8 flags."""
import numpy as np
import pytest
import torch

import orc
from flashws_amd import gpu

pytestmark = pytest.mark.gpu


def _expect(wire):
    buf = np.array(wire, dtype=np.uint8, copy=True)
    ret, frames, err_off, consumed = orc.orc_decode_stream(buf)
    return buf, frames, ret


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_pipe_batches_bit_exact(cuda, depth):
    batches = []
    for i in range(7):
        wire, descs, _ = gpu.config_c3(seed=200 + i, target=(2 + i) << 20)
        if i == 3:                                     # a batch that ends in a cut header + a truncated payload
            wire = np.concatenate([wire, np.frombuffer(bytes([0x82, 0xFE, 0x10]), dtype=np.uint8)])
        batches.append(wire)
    pipe = gpu.RxPipe(0, max_batch_bytes=16 << 20, max_frames=1 << 14, depth=depth)
    hosts = [torch.from_numpy(w.copy()).pin_memory() for w in batches]
    tickets = [pipe.submit(h) for h in hosts[:depth]]
    done = 0
    for i in range(len(hosts)):
        frames, res, _ = pipe.wait(tickets[i])
        exp_buf, exp_frames, ret = _expect(batches[i])
        assert int(res["status"]) == ret and int(res["n_frames"]) == len(exp_frames)
        assert np.array_equal(hosts[i].numpy(), exp_buf), i
        for k in ("hdr_off", "payload_len", "key", "opcode", "fin", "hdr_len"):
            assert np.array_equal(frames[k], exp_frames[k]), (i, k)
        done += 1
        if i + depth < len(hosts):
            tickets.append(pipe.submit(hosts[i + depth]))
    assert done == len(batches)
    pipe.close()


def test_pipe_submit_beyond_depth_waits(cuda):
    """Submitting more batches than slots before any wait blocks on the oldest
    slot instead of overwriting it; the last `depth` batches stay readable."""
    pipe = gpu.RxPipe(0, max_batch_bytes=4 << 20, max_frames=4096, depth=2)
    wires = [gpu.config_c2(seed=300 + i, n_frames=256, payload=4096)[0] for i in range(5)]
    hosts = [torch.from_numpy(w.copy()).pin_memory() for w in wires]
    tickets = [pipe.submit(h) for h in hosts]
    for i in (3, 4):
        frames, res, _ = pipe.wait(tickets[i])
        exp_buf, exp_frames, ret = _expect(wires[i])
        assert ret == 0 and int(res["n_frames"]) == 256
        assert np.array_equal(hosts[i].numpy(), exp_buf)
    for i in range(3):                                  # these were all processed too
        exp_buf, _, _ = _expect(wires[i])
        assert np.array_equal(hosts[i].numpy(), exp_buf)
    pipe.close()


def test_pipe_utf8_flags(cuda):
    wire, descs, ok = gpu.config_c5(seed=9, n_frames=400, payload=16384, invalid_permille=50)
    pipe = gpu.RxPipe(0, max_batch_bytes=len(wire) + 64, max_frames=512, depth=2, utf8=True)
    host = torch.from_numpy(wire.copy()).pin_memory()
    frames, res, flags = pipe.wait(pipe.submit(host))
    assert int(res["status"]) == 0 and int(res["n_frames"]) == 400
    assert np.array_equal(flags, ok)
    pipe.close()


def test_pipe_dense_64b_frames(cuda):
    """SURVEY §6's dense workload: 200 000 x 64 B masked frames (~3 700
    headers per 256 KiB super tile, over the LDS tables: the big-ST path),
    through the pipe with 3 batches in flight; every batch bit-exact against
    the oracle."""
    wire, descs, _ = gpu.config_c2(seed=64, n_frames=200_000, payload=64)
    exp_buf, exp_frames, ret = _expect(wire)
    assert ret == 0 and len(exp_frames) == 200_000
    pipe = gpu.RxPipe(0, max_batch_bytes=len(wire) + 64, max_frames=200_064, depth=3)
    hosts = [torch.from_numpy(wire.copy()).pin_memory() for _ in range(3)]
    tickets = [pipe.submit(h) for h in hosts]
    for i, t in enumerate(tickets):
        frames, res, _ = pipe.wait(t)
        assert int(res["status"]) == 0 and int(res["n_frames"]) == 200_000, i
        assert np.array_equal(hosts[i].numpy(), exp_buf), i
        for k in ("hdr_off", "payload_len", "key", "opcode", "fin", "hdr_len"):
            assert np.array_equal(frames[k], exp_frames[k]), (i, k)
    pipe.close()
