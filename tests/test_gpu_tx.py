"""GPU parity: the batch frame builder fws_gpu_encode_frames vs the reference's
SendFrame bytes (net/w_socket.h:832-944), bit-exact.

* the reference's own frames (tests/golden/tx_cases.json.gz, client and server
  sessions) rebuilt in one device batch, sequenced by fws_tx_next;
* random batches vs the oracle's orc_tx_frame: every length form, masked and
  unmasked frames mixed, payloads at arbitrary source offsets, batches of tiny
  frames (the bytewise path) and large ones (the shifted 16-B path);
* capacity overflow (~0, nothing written), the empty batch;
* round trip: client frames encoded here, decoded by fws_gpu_decode_stream.
"""
import numpy as np
import pytest
import torch

import orc
from flashws_amd import gpu
from flashws_amd._lib import TX_DESC
from test_tx_cpu import SESSIONS, frame_matches, tx_payload

pytestmark = pytest.mark.gpu


def build_batch(payloads, metas, rng, gap_max=40):
    """src bytes holding each payload at a random offset; TX_DESC records."""
    offs, pos = [], int(rng.integers(0, 16))
    for p in payloads:
        offs.append(pos)
        pos += len(p) + int(rng.integers(0, gap_max))
    src = rng.integers(0, 256, pos + 16, dtype=np.uint8)
    d = np.zeros(len(payloads), dtype=TX_DESC)
    for i, (p, (op, fin, key, masked)) in enumerate(zip(payloads, metas)):
        src[offs[i]:offs[i] + len(p)] = np.frombuffer(p, dtype=np.uint8)
        d[i] = (offs[i], len(p), key, op, fin, masked, 0)
    return src, d


def encode(ctx, cuda, src, d, out_cap=None, fill=0xEE):
    total = sum(int(x["len"]) + 2 + 4 * int(x["masked"]) + (0 if x["len"] < 126 else 2 if x["len"] < 65536 else 8)
                for x in d)
    cap = total if out_cap is None else out_cap
    out = torch.full((max(cap, 1),), fill, dtype=torch.uint8, device=cuda)
    dsrc = torch.from_numpy(src).to(cuda)
    dd = torch.from_numpy(d.view(np.uint8).copy()).to(cuda)
    ol = gpu.encode_frames(ctx, out[:cap] if cap else out[:0], dsrc, dd, len(d))
    torch.cuda.synchronize()
    return out.cpu().numpy().tobytes(), int(ol.cpu().item()), total


def oracle_frames(payloads, metas):
    res = []
    for p, (op, fin, key, masked) in zip(payloads, metas):
        st = orc.OrcTx(not masked)
        # orc_tx_frame sequences from its state; a fresh state emits frame_type
        # as the opcode, so pass the wire opcode (0 -> continuation via state)
        if op == 0:
            st.frame(b"", 2, 0, 0)                  # open a message so the next data frame continues it
            res.append(st.frame(p, 2, fin, key))
        else:
            res.append(st.frame(p, op, fin, key))
    return res


@pytest.mark.parametrize("sess", SESSIONS, ids=lambda s: "server" if s["server"] else "client")
def test_encode_reference_session(ctx, cuda, sess):
    rng = np.random.default_rng(5 + sess["server"])
    st = gpu.TxState()
    payloads, metas = [], []
    for r in sess["frames"]:
        op, fin = st.next(r["frame_type"], r["last"])
        payloads.append(tx_payload(r["seed"], r["len"]))
        metas.append((op, fin, r["key"], 0 if sess["server"] else 1))
    src, d = build_batch(payloads, metas, rng)
    out, n, total = encode(ctx, cuda, src, d)
    assert n == total
    pos = 0
    for i, r in enumerate(sess["frames"]):
        assert frame_matches(r, out[pos:pos + r["size"]]), (i, r["len"], r["frame_type"])
        pos += r["size"]
    assert pos == total


LEN_CHOICES = [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 64, 124, 125, 126, 127, 200, 1000, 4095, 4096, 4097, 8191,
               65535, 65536, 65537, 100003]


@pytest.mark.parametrize("mode", ["tiny", "mixed", "large"])
def test_encode_random_vs_oracle(ctx, cuda, mode):
    rng = np.random.default_rng({"tiny": 1, "mixed": 2, "large": 3}[mode])
    n = {"tiny": 20000, "mixed": 3000, "large": 300}[mode]
    payloads, metas = [], []
    for i in range(n):
        if mode == "tiny":
            ln = int(rng.integers(0, 40))
        elif mode == "large":
            ln = int(rng.integers(4000, 300000))
        else:
            ln = int(rng.choice(LEN_CHOICES))
        payloads.append(rng.integers(0, 256, ln, dtype=np.uint8).tobytes())
        masked = int(rng.random() < 0.7)
        op = int(rng.choice([1, 2, 0])) if ln > 125 else int(rng.choice([0, 1, 2, 8, 9, 10]))
        metas.append((op, int(rng.random() < 0.5), int(rng.integers(0, 1 << 32)), masked))
    src, d = build_batch(payloads, metas, rng, gap_max=64 if mode != "tiny" else 5)
    out, got, total = encode(ctx, cuda, src, d)
    assert got == total
    exp = b"".join(oracle_frames(payloads, metas))
    assert len(exp) == total
    if out != exp:
        diff = np.flatnonzero(np.frombuffer(out, np.uint8) != np.frombuffer(exp, np.uint8))
        pytest.fail(f"{len(diff)} bytes differ, first at {diff[0]}")


def test_encode_overflow_and_empty(ctx, cuda):
    rng = np.random.default_rng(9)
    payloads = [rng.integers(0, 256, 5000, dtype=np.uint8).tobytes() for _ in range(4)]
    metas = [(2, 1, 0x01020304, 1)] * 4
    src, d = build_batch(payloads, metas, rng)
    out, got, total = encode(ctx, cuda, src, d, out_cap=4 * 5000)            # 32 bytes short
    assert got == -1                                                           # ~0 as int64
    assert out == b"\xEE" * len(out)                                           # nothing written
    out, got, total = encode(ctx, cuda, src, d, out_cap=total)
    assert got == total
    # the empty batch: length 0
    out_len = torch.full((1,), 7, dtype=torch.int64, device=cuda)
    e = torch.empty(16, dtype=torch.uint8, device=cuda)
    gpu.encode_frames(ctx, e, e, e, 0, out_len=out_len)
    assert int(out_len.cpu().item()) == 0


def test_encode_then_decode_round_trip(ctx, cuda):
    """Client frames from the builder, decoded by the server-side decode."""
    rng = np.random.default_rng(11)
    payloads, metas = [], []
    st = gpu.TxState()
    for i in range(5000):
        ln = int(rng.choice([0, 3, 125, 126, 1400, 4096, 65535, 65536, 70001]))
        ft = int(rng.choice([1, 2])) if ln > 125 else int(rng.choice([2, 9, 10]))
        op, fin = st.next(ft, int(rng.random() < 0.7))
        payloads.append(rng.integers(0, 256, ln, dtype=np.uint8).tobytes())
        metas.append((op, fin, int(rng.integers(1, 1 << 32)), 1))
    src, d = build_batch(payloads, metas, rng)
    out, got, total = encode(ctx, cuda, src, d)
    assert got == total
    wire = torch.frombuffer(bytearray(out[:total]), dtype=torch.uint8).to(cuda)
    rc, frames, result, _ = gpu.decode_stream(ctx, wire, len(d) + 16)
    torch.cuda.synchronize()
    assert rc == 0
    res = gpu.read_result(result)
    assert res["status"] == 0 and res["n_frames"] == len(d) and res["consumed"] == total
    fi = gpu.read_frames(frames, len(d))
    host = wire.cpu().numpy()
    for i in range(len(d)):
        assert fi[i]["opcode"] == metas[i][0] and fi[i]["fin"] == metas[i][1] and fi[i]["key"] == metas[i][2]
        o = int(fi[i]["hdr_off"]) + int(fi[i]["hdr_len"])
        assert host[o:o + len(payloads[i])].tobytes() == payloads[i], i
