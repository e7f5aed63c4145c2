"""GPU parity: the batch frame builder fws_gpu_encode_frames vs the reference's
SendFrame bytes (net/w_socket.h:832-944), bit-exact.

* the reference's own frames (tests/golden/tx_cases.json.gz, client and server
  sessions) rebuilt in one device batch, sequenced by fws_tx_next;
* random batches vs the oracle's orc_tx_frame: every length form, masked and
  unmasked frames mixed, payloads at arbitrary source offsets, batches of tiny
  frames (the bytewise path) and large ones (the shifted 16-B path);
* capacity overflow (~0; nothing at or past out_cap, and with the plan form
  nothing at all), the empty batch; both forms (one launch, plan + encode);
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


TX_FORMS = {"one": 1, "plan": 1, "plan_dpp": 2, "plan_so": 3, "plan_sod": 4, "plan_sr": 5}


@pytest.fixture(autouse=True, params=list(TX_FORMS))
def tx_form(request):
    """every test runs on each form of fws_gpu_encode_frames: one launch
    (k_tx_one, forced for every batch), k_out_plan + k_tx_encode_w5 (two
    aligned loads per chunk), k_out_plan + k_tx_encode_dpp (one nontemporal
    load per chunk, the second block from the next lane), and k_out_plan +
    k_tx_encode_so (full chunks only, two loads / DPP) + k_tx_seams (the seam
    chunks, one thread per frame), and k_tx_plan_seams (the plan building the
    seam chunks into records) + k_tx_encode_sr"""
    from flashws_amd._lib import lib
    old = lib().fws_internal_set_tx_one(2 if request.param == "one" else 0, 0)
    old_w = lib().fws_internal_set_tx_w5(TX_FORMS[request.param])
    yield request.param
    lib().fws_internal_set_tx_one(old, 0)
    lib().fws_internal_set_tx_w5(old_w)


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
    out = torch.full((max(cap, 1) + 64,), fill, dtype=torch.uint8, device=cuda)   # + a guard band
    dsrc = torch.from_numpy(src).to(cuda)
    dd = torch.from_numpy(d.view(np.uint8).copy()).to(cuda)
    ol = gpu.encode_frames(ctx, out[:cap] if cap else out[:0], dsrc, dd, len(d))
    torch.cuda.synchronize()
    o = out.cpu().numpy().tobytes()
    assert o[max(cap, 1):] == bytes([fill]) * 64                               # nothing past out_cap
    return o[:max(cap, 1)], int(ol.cpu().item()), total


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


def test_encode_overflow_and_empty(ctx, cuda, tx_form):
    rng = np.random.default_rng(9)
    payloads = [rng.integers(0, 256, 5000, dtype=np.uint8).tobytes() for _ in range(4)]
    metas = [(2, 1, 0x01020304, 1)] * 4
    src, d = build_batch(payloads, metas, rng)
    for cap in (4 * 5000, 5007, 17):                                           # 32 bytes short .. one frame
        out, got, total = encode(ctx, cuda, src, d, out_cap=cap)
        assert got == -1                                                       # ~0 as int64
        if tx_form.startswith("plan"):                                         # plan + encode (any form)
            assert out == b"\xEE" * len(out)                                   # nothing written at all
        else:                                                                  # the frames that fit, exact
            exp = b"".join(oracle_frames(payloads, metas))
            k = max(j for j in range(5) if sum(5008 for _ in range(j)) <= cap)
            assert out[:5008 * k] == exp[:5008 * k]
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


# ---- fws_tx_session: SendFrame for host payloads of one connection ----------

@pytest.mark.parametrize("sess", SESSIONS, ids=lambda s: "server" if s["server"] else "client")
@pytest.mark.parametrize("batch", [1, 7, 1000])
def test_tx_session_reference(ctx, cuda, sess, batch):
    """The reference's own WriteFrame sequence (tests/golden/tx_cases.json.gz)
    sent through one session in calls of `batch` frames: every frame's bytes
    equal the reference's; sequencing carried across calls."""
    tx = gpu.TxSession(ctx, is_server=bool(sess["server"]))
    frames = [(tx_payload(r["seed"], r["len"]), r["frame_type"], r["last"], r["key"]) for r in sess["frames"]]
    recs = sess["frames"]
    for i0 in range(0, len(frames), batch):
        rc, out, n = tx.send(frames[i0:i0 + batch])
        assert rc == 0 and len(out) == n
        pos = 0
        for i in range(i0, min(i0 + batch, len(frames))):
            assert frame_matches(recs[i], out[pos:pos + recs[i]["size"]]), (i, recs[i]["len"])
            pos += recs[i]["size"]
        assert pos == len(out)
    tx.close()


def test_tx_session_capacity_keeps_state(ctx, cuda):
    """Too small an output: FWS_ERR_CAPACITY with the size needed, nothing sent,
    the open message stays open; the retry emits the same bytes."""
    tx = gpu.TxSession(ctx, is_server=False)
    rc, out, n = tx.send([(b"abc", 1, False, 0x11223344)])
    assert rc == 0 and out[0] == 0x01 and tx.last_msg_not_fin() == 1
    frames = [(b"x" * 200, 1, True, 0x01020304)]
    rc, _, need = tx.send(frames, out_cap=10)
    assert rc == -20 and need == 2 + 2 + 4 + 200 and tx.last_msg_not_fin() == 1
    rc, out, n = tx.send(frames)
    assert rc == 0 and n == need and out[0] == 0x80                 # FIN continuation of the open message
    exp = orc.OrcTx(False)
    exp.frame(b"abc", 1, 0, 0x11223344)
    assert out == exp.frame(b"x" * 200, 1, 1, 0x01020304)
    assert tx.last_msg_not_fin() == 0
    tx.close()


def test_tx_session_then_rx_session(ctx, cuda):
    """Client frames sent by fws_tx_session decode through the server-side
    fws_rx_session to the same payloads and message boundaries."""
    rng = np.random.default_rng(12)
    tx = gpu.TxSession(ctx, is_server=False)
    rx = gpu.RxSession(ctx, is_server=True)
    frames, wire = [], b""
    for i in range(300):
        ln = int(rng.choice([0, 5, 125, 126, 3000, 70000]))
        frames.append((rng.integers(0, 256, ln, dtype=np.uint8).tobytes(), int(rng.choice([1, 2])),
                       bool(rng.random() < 0.7), int(rng.integers(0, 1 << 32))))
    for i0 in range(0, 300, 64):
        rc, out, _ = tx.send(frames[i0:i0 + 64])
        assert rc == 0
        wire += out
    ret, buf, ev, ctl = rx.feed(wire)
    assert ret == 0
    got = b"".join(bytes(buf[int(e["data_off"]):int(e["data_off"]) + int(e["size"])]) for e in ev if e["kind"] == 0 and not e["is_ctl"])
    assert got == b"".join(f[0] for f in frames)
    assert sum(int(e["msg_end"]) for e in ev if e["kind"] == 0) == sum(1 for f in frames if f[2])
    tx.close()
    rx.close()
