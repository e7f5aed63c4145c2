"""CPU: the send path's byte builder and sequencing pinned to the REAL reference.

tests/golden/tx_cases.json.gz (make_golden.py tx_cases) holds WriteFrame calls
on a reference WSClientSocket<false> and WSServerSocket<false> and the bytes
SendFrame (net/w_socket.h:832-944) wrote for each. Replayed here through
  * the oracle's orc_tx_frame (oracle/fws_oracle.c), byte-for-byte, with the
    mask key the reference drew (SemiSecureRand32, w_socket.h:860) taken from
    the fixture, and
  * the product's host sequencing fws_tx_next (libfws_amd.so, host code only):
    its opcode / FIN must be the wire's b0.
"""
import ctypes as C
import gzip
import hashlib
import json
import os

import numpy as np
import pytest

import orc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_tx_golden():
    with gzip.open(os.path.join(GOLDEN, "tx_cases.json.gz"), "rt") as f:
        return json.load(f)


def tx_payload(seed, n):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def frame_matches(rec, b):
    if len(b) != rec["size"]:
        return False
    if "hex" in rec:
        return b.hex() == rec["hex"]
    return b[:64].hex() == rec["head_hex"] and hashlib.sha256(b).hexdigest() == rec["sha256"]


SESSIONS = load_tx_golden()


def test_tx_golden_shape():
    assert [s["server"] for s in SESSIONS] == [0, 1]
    for s in SESSIONS:
        lens = {r["len"] for r in s["frames"]}
        assert {0, 125, 126, 65535, 65536} <= lens          # every length form and its edges
        assert any(not r["last"] for r in s["frames"])       # fragmented messages
        assert s["frames"][-1]["frame_type"] == 8           # ends with CLOSE


@pytest.mark.parametrize("sess", SESSIONS, ids=lambda s: "server" if s["server"] else "client")
def test_oracle_tx_vs_reference(sess):
    tx = orc.OrcTx(sess["server"])
    for i, r in enumerate(sess["frames"]):
        b = tx.frame(tx_payload(r["seed"], r["len"]), r["frame_type"], r["last"], r["key"])
        assert frame_matches(r, b), (i, r["len"], r["frame_type"], r["last"])


@pytest.mark.parametrize("sess", SESSIONS, ids=lambda s: "server" if s["server"] else "client")
def test_tx_next_vs_reference(sess):
    from flashws_amd import gpu
    st = gpu.TxState()
    for i, r in enumerate(sess["frames"]):
        op, fin = st.next(r["frame_type"], r["last"])
        b0 = int((r.get("hex") or r["head_hex"])[:2], 16)
        assert (op, fin) == (b0 & 15, b0 >> 7), i
        b1 = int((r.get("hex") or r["head_hex"])[2:4], 16)
        assert (b1 >> 7) == (0 if sess["server"] else 1)


def test_tx_next_rules():
    """SendFrame's rule (w_socket.h:845-848, 903-913) on a hand-made sequence."""
    from flashws_amd import gpu
    st = gpu.TxState()
    seq = [(1, 0, (1, 0)), (2, 0, (0, 0)), (9, 1, (9, 1)), (1, 1, (0, 1)), (2, 1, (2, 1)),
           (10, 0, (10, 0)), (1, 0, (1, 0)), (8, 1, (8, 1)), (2, 1, (0, 1))]
    for ft, last, exp in seq:
        assert st.next(ft, last) == exp, (ft, last)
