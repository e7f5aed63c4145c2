"""CPU: pin the oracle (oracle/fws_oracle.c) to the REAL reference's outputs.

tests/golden/ was produced by tests/golden/make_golden.py, which drives the
compiled reference (WSServerSocket<false>::OnRecvData, net/w_socket.h:543-769;
WSMaskBytesFast and its variants, crypto/ws_mask.h:15-197). Every fixture is
replayed through the C restatement and must match byte-for-byte: return
codes, in-place unmasked bytes, the on_read()/PONG/CLOSE event sequence
(opcode, size, view offset and capacity, frame_end, msg_end, is_control),
and the carried RX state after each read.
"""
import gzip
import hashlib
import json
import os

import numpy as np
import pytest

import orc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load_cases():
    with gzip.open(os.path.join(GOLDEN, "kat_cases.json.gz"), "rt") as f:
        return json.load(f)


CASES = _load_cases()


def _out_matches(field, buf):
    b = bytes(buf)
    if isinstance(field, str):
        return b.hex() == field
    return len(b) == field["len"] and hashlib.sha256(b).hexdigest() == field["sha256"]


def _events_json(ev, ctl):
    res = []
    for e in orc.orc_to_reference_view(ev, ctl):
        e = dict(e)
        if "ctl" in e:
            e["ctl"] = e["ctl"].hex()
        res.append(e)
    return res


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_reference_kat(name):
    case = CASES[name]
    s = orc.OrcSession()
    for i, (rd, exp) in enumerate(zip(case["reads"], case["expected"])):
        ret, buf, ev, ctl = s.feed(bytes.fromhex(rd))
        assert ret == exp["ret"], (name, i)
        assert _out_matches(exp["out"], buf), (name, i)
        assert _events_json(ev, ctl) == exp["events"], (name, i)
        st = s.head()
        got_state = {k: int(getattr(st, k)) for k, _ in orc.RxStateHead._fields_}
        assert got_state == exp["state"], (name, i)


def test_rfc6455_known_answer_literal():
    """RFC 6455 §5.7: a single-frame masked text message containing "Hello"."""
    s = orc.OrcSession()
    ret, buf, ev, ctl = s.feed(bytes.fromhex("818537fa213d7f9f4d5158"))
    assert ret == 0 and bytes(buf[6:]) == b"Hello"
    vis = orc.user_visible(ev, ctl)
    assert vis == [{"kind": 0, "opcode": 1, "is_ctl": 0, "frame_end": 1, "msg_end": 1, "size": 5,
                    "data_off": 6, "capacity": 11}]


def _aligned(n):
    raw = np.zeros(n + 64, dtype=np.uint8)
    o = (-raw.ctypes.data) % 64
    return raw[o:o + n]


def test_oracle_mask_sweep_matches_reference():
    g = np.load(os.path.join(GOLDEN, "mask_sweep.npz"))
    base, keys, lens, dig = g["base"], g["keys"], g["lens"], g["digests"]
    work = _aligned(len(base))
    for ki, key in enumerate(keys):
        for off in range(64):
            for li, n in enumerate(lens):
                n = int(n)
                variants = orc.MASK_FUNCS if (off % 8 == 1 and li % 5 == 0) else ("ws_mask_fast",)
                for v in variants:
                    work[:] = base
                    orc.orc_mask(v, work, int(key), off, n)
                    d = np.frombuffer(hashlib.blake2b(work[off:off + n].tobytes(), digest_size=8).digest(), "<u8")[0]
                    assert d == dig[ki, off, li], (v, hex(int(key)), off, n)
                    assert np.array_equal(work[:off], base[:off])
                    assert np.array_equal(work[off + n:], base[off + n:])


def test_rotate_r():
    """base/constexpr_math.h:84-87 static_asserts."""
    r = orc.orc().orc_rotr32
    assert r(0xF0000000, 4) == 0x0F000000
    assert r(0xF0000000, 32) == 0xF0000000
    assert r(0xF0000000, 8) == 0x00F00000
    assert r(0xF0000000, 36) == 0x0F000000


def _event_digest(h, evs):
    for e in evs:
        e = dict(e)
        if "ctl" in e:
            e["ctl"] = e["ctl"].hex()
        h.update(json.dumps(e, sort_keys=True).encode())


CONFIGS = json.load(open(os.path.join(GOLDEN, "configs.json")))


# the 4 GiB per-GPU C5 digest is replayed on the GPU only (tests/test_gpu_configs.py)
@pytest.mark.parametrize("name", sorted(k for k in CONFIGS if k != "C5_full_per_gpu"))
def test_config_streams_match_reference(name):
    """Full-size BASELINE configs: generator bytes, unmasked output and the
    on_read event list (2 MiB reads) equal the reference's digests."""
    from flashws_amd import gpu
    exp = CONFIGS[name]
    fn = {"C2": gpu.config_c2, "C3": gpu.config_c3, "C4": gpu.config_c4,
          "C5_16k_frames": lambda: gpu.config_c5(n_frames=16384)}[name]
    wire, descs, ok = fn()
    assert len(wire) == exp["wire_bytes"] and len(descs) == exp["frames"]
    assert hashlib.sha256(wire.tobytes()).hexdigest() == exp["wire_sha256"]
    s = orc.OrcSession()
    h_out, h_ev = hashlib.sha256(), hashlib.sha256()
    read = 2 << 20
    for o in range(0, len(wire), read):
        ret, buf, ev, ctl = s.feed(wire[o:o + read].tobytes(), ev_cap=1 << 20)
        assert ret == 0
        h_out.update(buf.tobytes())
        _event_digest(h_ev, orc.orc_to_reference_view(ev, ctl))
    assert h_out.hexdigest() == exp["unmasked_sha256"]
    assert h_ev.hexdigest() == exp["events_sha256_2MiB_reads"]
    if "utf8_ok_sha256_python_strict" in exp:
        assert hashlib.sha256(ok.tobytes()).hexdigest() == exp["utf8_ok_sha256_python_strict"]
