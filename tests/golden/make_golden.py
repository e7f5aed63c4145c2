#!/usr/bin/env python3
"""Generate tests/golden/ fixtures from the REAL flashws reference.

Runs only in the build container, where /root/reference exists and
oracle/_ref/libfwsref.so (oracle/Makefile `ref`, compiled from the reference's
own headers by oracle/ref_driver.cpp) drives WSServerSocket<false>::OnRecvData
(net/w_socket.h:543-769) and fws::WSMaskBytesFast (crypto/ws_mask.h:175).
The fixtures are data only (inputs + the reference's outputs / digests).

    make -C oracle ref && python tests/golden/make_golden.py [tx | configs]

tx_cases.json.gz holds the send side: sequences of WriteFrame calls on a
WSClientSocket<false> / WSServerSocket<false> (-> SendFrame, w_socket.h:832-944)
with the frame bytes each call wrote (full hex for small frames, sha256 above).

Cases the reference cannot run (it dereferences a null control buffer: empty
PING/CLOSE, a control header that ends a read before its payload, a PONG whose
payload is split across reads; SURVEY §0 finding 3) are never generated.
"""
import gzip
import hashlib
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import orc  # noqa: E402
from wsframes import frame  # noqa: E402

MASK_LENS = list(range(0, 601)) + [1023, 1024, 1025, 2047, 2048, 2049, 4093, 4096, 16384, 65535, 65536]
MASK_KEYS = [0x3D21FA37, 0x00000001, 0xFFFFFFFF]
MASK_BASE_LEN = 65536 + 64 + 64


def raw_header(b0, b1, ext=b"", key=b"\x01\x02\x03\x04"):
    return bytes([b0, b1]) + ext + key


def run_ref(reads, extra_cap=0):
    s = orc.RefSession()
    out = []
    for r in reads:
        ret, buf, ev, ctl = s.feed(r, extra_cap=extra_cap)
        st = s.head()
        out.append({
            "ret": int(ret), "out": _out_field(bytes(buf)), "events": _json_events(orc.user_visible(ev, ctl)),
            "state": {k: int(getattr(st, k)) for k, _ in orc.RxStateHead._fields_}})
        if ret < 0:
            break
    return out


def _out_field(b):
    """Small outputs verbatim (hex), large ones as a SHA-256 digest."""
    return b.hex() if len(b) <= 512 else {"sha256": hashlib.sha256(b).hexdigest(), "len": len(b)}


def _json_events(evs):
    res = []
    for e in evs:
        e = dict(e)
        if "ctl" in e:
            e["ctl"] = e["ctl"].hex()
        res.append(e)
    return res


def splits(data, points):
    pts = [0] + sorted(points) + [len(data)]
    return [data[a:b] for a, b in zip(pts, pts[1:])]


def kat_cases():
    hello = bytes.fromhex("818537fa213d7f9f4d5158")          # RFC 6455 §5.7
    cases = [("rfc_hello", [hello]), ("rfc_hello_split_1_7", splits(hello, [1, 7]))]
    for p in range(1, len(hello)):
        cases.append((f"rfc_hello_split_{p}", splits(hello, [p])))
    frag = (frame(1, b"Hel", fin=0) + frame(9, b"x", key=0x01020304) + frame(0, b"l", fin=0, key=7)
            + frame(0, b"o", fin=1, key=0xA0B0C0D0))
    cases.append(("fragmented_with_ping", [frag]))
    ping_end = len(frame(1, b"Hel", fin=0)) + 6              # after the PING header
    for p in range(1, len(frag)):
        if p == ping_end:
            continue   # control header ending a read: the reference dereferences null (w_socket.h:652)
        cases.append((f"fragmented_split_{p}", splits(frag, [p])))
    good = frame(2, b"abcdef")
    cases += [
        ("err_rsv1", [good + bytes([0xC2, 0x80]) + b"\0" * 8]),
        ("err_rsv3", [good + bytes([0x92, 0x81]) + b"\0" * 8]),
        ("err_opcode3", [good + bytes([0x83, 0x80]) + b"\0" * 8]),
        ("err_opcode_b", [bytes([0x8B, 0x80]) + b"\0" * 8]),
        ("err_unmasked", [good + frame(2, b"zz", masked=False)]),
        ("err_len_2p32p1", [good + raw_header(0x82, 0xFF, struct.pack(">Q", (1 << 32) + 1))]),
        ("err_rsv_and_opcode", [bytes([0xF3, 0x80]) + b"\0" * 8]),
        ("len_2p32_header_only", [raw_header(0x82, 0xFF, struct.pack(">Q", 1 << 32))]),
        ("len_2p32_header_plus_bytes", [raw_header(0x82, 0xFF, struct.pack(">Q", 1 << 32)) + b"\x11" * 37]),
        ("zero_len_bin", [frame(2, b"")]),
        ("zero_len_text_then_data", [frame(1, b"") + frame(2, b"q")]),
        ("nonminimal_126_len5", [frame(2, b"hello", len_form=126)]),
        ("nonminimal_127_len5", [frame(2, b"hello", len_form=127)]),
        ("len_70000_127", [frame(2, bytes(range(256)) * 273 + b"x" * 112)]),
        ("pong_payload", [frame(10, b"pong!") + frame(2, b"after")]),
        ("ping_payload", [frame(9, b"are you there") + frame(1, b"yes")]),
        ("close_code_reason", [frame(2, b"last") + frame(8, b"\x03\xe8bye")]),
        ("close_code_only", [frame(8, b"\x03\xe9")]),
        ("ping_split_payload", splits(frame(9, b"abcdef") + frame(2, b"z"), [8])),
        ("close_split_payload", splits(frame(8, b"\x03\xe8reason"), [9, 11])),
        ("ping_125", [frame(9, bytes(range(125)))]),
        ("partial_header_1", [b"\x82"]),
        ("partial_header_8", splits(frame(2, b"y" * 300), [3]) + [b""]),
        ("empty_read", [b""]),
    ]
    big = frame(2, bytes(range(251)) * 262 + b"z" * 54)       # 65816 B: 14-B header
    for p in (1, 3, 9, 10, 13, 14, 15, 4097):
        cases.append((f"hdr14_split_{p}", splits(big, [p])))
    mid = frame(1, b"0123456789" * 30)                         # 300 B: 8-B header
    for p in range(1, 9):
        cases.append((f"hdr8_split_{p}", splits(mid + frame(2, b"tail"), [p])))
    # key rotation across many reads of odd sizes (w_socket.h:756-759)
    long = frame(2, bytes((i * 7 + 3) & 255 for i in range(5000)), key=0x89ABCDEF)
    for step in (3, 7, 13, 4093):
        cases.append((f"rotation_reads_of_{step}", [long[i:i + step] for i in range(0, len(long), step)]))
    cases.append(("rotation_reads_of_1", [long[i:i + 1] for i in range(0, 300)]))
    return cases


def random_stream_cases(n_cases=40):
    rng = np.random.default_rng(20251015)
    cases = []
    for c in range(n_cases):
        frames, in_msg = [], False
        for _ in range(int(rng.integers(1, 40))):
            kind = rng.random()
            key = int(rng.integers(0, 2**32))
            if kind < 0.12:
                op = int(rng.choice([9, 10]))
                pl = rng.integers(0, 256, int(rng.integers(1, 126)), dtype=np.uint8).tobytes()
                frames.append(("ctl", op, frame(op, pl, key=key)))
                continue
            n = int(rng.choice([rng.integers(0, 130), rng.integers(126, 3000), rng.integers(0, 20)]))
            pl = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            fin = int(rng.random() < 0.6)
            op = 0 if in_msg else int(rng.choice([1, 2]))
            form = None
            if rng.random() < 0.1:
                form = 127 if rng.random() < 0.5 else 126
            frames.append(("data", op, frame(op, pl, fin=fin, key=key, len_form=form)))
            in_msg = not fin
        data = b"".join(f[2] for f in frames)
        # forbidden split points: right after a control header, inside a PONG payload
        bad, pos = set(), 0
        for kind, op, fb in frames:
            if kind == "ctl":
                hl = 6
                bad.add(pos + hl)
                if op == 10:
                    bad.update(range(pos + hl, pos + len(fb)))
            pos += len(fb)
        max_read = int(rng.choice([7, 64, 500, 5000]))
        max_read = max(max_read, len(data) // 150)      # keep fixtures small: <= ~300 reads
        pts, p = [], 0
        while True:
            p += int(rng.integers(1, max_read + 1))
            if p >= len(data):
                break
            if p not in bad:
                pts.append(p)
        cases.append((f"random_{c}", splits(data, pts)))
    return cases


def mask_sweep():
    rng = np.random.default_rng(7)
    raw = np.zeros(MASK_BASE_LEN + 64, dtype=np.uint8)
    off0 = (-raw.ctypes.data) % 64
    base = raw[off0:off0 + MASK_BASE_LEN]
    base[:] = rng.integers(0, 256, MASK_BASE_LEN, dtype=np.uint8)
    dig = np.zeros((len(MASK_KEYS), 64, len(MASK_LENS)), dtype=np.uint64)
    for ki, key in enumerate(MASK_KEYS):
        for off in range(64):
            for li, n in enumerate(MASK_LENS):
                work = _aligned_copy(base)
                orc.ref_mask("ws_mask_fast", work, key, off, n)
                w = work[off:off + n].tobytes()
                for v in ("ws_mask_bytes", "mask_avx2", "mask_large_chunk_avx2", "mask1"):
                    other = _aligned_copy(base)
                    orc.ref_mask(v, other, key, off, n)
                    assert other[off:off + n].tobytes() == w, (v, key, off, n)
                dig[ki, off, li] = np.frombuffer(hashlib.blake2b(w, digest_size=8).digest(), "<u8")[0]
    np.savez_compressed(os.path.join(HERE, "mask_sweep.npz"), base=base, keys=np.array(MASK_KEYS, np.uint32),
                        lens=np.array(MASK_LENS, np.uint64), digests=dig)


def _aligned_copy(a):
    raw = np.zeros(len(a) + 64, dtype=np.uint8)
    o = (-raw.ctypes.data) % 64
    out = raw[o:o + len(a)]
    out[:] = a
    return out


def event_digest(h, evs):
    for e in evs:
        h.update(json.dumps(_json_events([e])[0], sort_keys=True).encode())


def config_digests():
    from flashws_amd import gpu
    out = {}
    specs = {
        "C2": lambda: gpu.config_c2(),
        "C3": lambda: gpu.config_c3(),
        "C4": lambda: gpu.config_c4(),
        "C5_16k_frames": lambda: gpu.config_c5(n_frames=16384),
        "C5_full_per_gpu": lambda: gpu.config_c5(),             # 262 144 x 16 KiB, seed 42 (rank 0's shard)
    }
    only = os.environ.get("GOLDEN_ONLY")
    if only:
        specs = {k: v for k, v in specs.items() if k in only.split(",")}
        with open(os.path.join(HERE, "configs.json")) as f:
            out = json.load(f)
    for name, fn in specs.items():
        wire, descs, ok = fn()
        rec = {"wire_bytes": int(len(wire)), "frames": int(len(descs)),
               "payload_bytes": int(descs["payload_len"].sum()),
               "wire_sha256": hashlib.sha256(wire.tobytes()).hexdigest()}
        s = orc.RefSession()
        h_out, h_ev = hashlib.sha256(), hashlib.sha256()
        read = 2 << 20
        ret_all = 0
        for o in range(0, len(wire), read):
            ret, buf, ev, ctl = s.feed(wire[o:o + read].tobytes(), ev_cap=1 << 20)
            ret_all = ret_all or ret
            h_out.update(buf.tobytes())
            event_digest(h_ev, orc.user_visible(ev, ctl))
        rec.update({"ret": int(ret_all), "unmasked_sha256": h_out.hexdigest(),
                    "events_sha256_2MiB_reads": h_ev.hexdigest()})
        if name.startswith("C5"):
            full = wire.copy()
            orc.orc_decode_stream(full)
            flags = []
            mv = memoryview(full)
            for d in descs:
                o, n = int(d["payload_off"]), int(d["payload_len"])
                try:
                    str(mv[o:o + n], "utf-8", "strict")
                    flags.append(1)
                except UnicodeDecodeError:
                    flags.append(0)
            flags = np.array(flags, np.uint8)
            assert np.array_equal(flags, ok), "generator's utf8_ok disagrees with Python's decoder"
            rec["utf8_ok_sha256_python_strict"] = hashlib.sha256(flags.tobytes()).hexdigest()
            rec["utf8_invalid_frames"] = int(len(flags) - flags.sum())
        out[name] = rec
        print(name, rec["frames"], rec["ret"], flush=True)
    with open(os.path.join(HERE, "configs.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def tx_payload(seed, n):
    """Payload of a TX golden record: PCG64(seed) bytes (stable across numpy)."""
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


TX_HEX_MAX = 512


def tx_sequence(rng):
    """(len, frame_type, last) calls: every length form edge, a fragmented
    message with a control frame inside it, then random calls, then CLOSE."""
    calls = [(n, 2, 1) for n in (0, 1, 2, 3, 4, 5, 7, 125, 126, 127, 128, 65535, 65536, 65537, (1 << 20) + 3)]
    calls += [(10, 1, 0), (300, 2, 0), (0, 9, 1), (70000, 1, 0), (5, 10, 1), (1, 2, 1), (0, 1, 1)]
    for _ in range(160):
        kind = rng.random()
        if kind < 0.25:
            calls.append((int(rng.integers(0, 126)), int(rng.choice([9, 10])), 1))
        else:
            n = int(rng.choice([rng.integers(0, 126), rng.integers(126, 65536), rng.integers(65536, 200000)],
                               p=[0.5, 0.4, 0.1]))
            calls.append((n, int(rng.choice([1, 2])), int(rng.random() < 0.6)))
    calls.append((2, 8, 1))
    return calls


def tx_cases():
    out = []
    for is_server in (0, 1):
        rng = np.random.default_rng(77 + is_server)
        h, write = orc.ref_tx_session(is_server)
        frames = []
        for i, (n, ft, last) in enumerate(tx_sequence(rng)):
            seed = 1000 * (1 + is_server) + i
            b = write(tx_payload(seed, n), ft, last)
            rec = {"seed": seed, "len": n, "frame_type": ft, "last": last, "size": len(b)}
            hl = len(b) - n
            rec["key"] = 0 if is_server else int.from_bytes(b[hl - 4:hl], "little")
            if len(b) <= TX_HEX_MAX:
                rec["hex"] = b.hex()
            else:
                rec["head_hex"] = b[:64].hex()
                rec["sha256"] = hashlib.sha256(b).hexdigest()
            frames.append(rec)
        orc.ref().ref_tx_free(h)
        out.append({"server": is_server, "frames": frames})
    with gzip.open(os.path.join(HERE, "tx_cases.json.gz"), "wt") as f:
        json.dump(out, f, sort_keys=True)
    print("tx sessions:", [len(x["frames"]) for x in out], flush=True)


def main():
    assert orc.ref_available(), "build oracle/_ref first: make -C oracle ref"
    if sys.argv[1:] == ["tx"]:
        tx_cases()
        return
    if sys.argv[1:] == ["configs"]:         # GOLDEN_ONLY=C5_full_per_gpu ... to regenerate one entry
        config_digests()
        return
    cases = {}
    for name, reads in kat_cases() + random_stream_cases():
        cases[name] = {"reads": [r.hex() for r in reads], "expected": run_ref(reads)}
    with gzip.open(os.path.join(HERE, "kat_cases.json.gz"), "wt") as f:
        json.dump(cases, f, sort_keys=True)
    print("kat cases:", len(cases), flush=True)
    mask_sweep()
    print("mask sweep done", flush=True)
    config_digests()
    tx_cases()


if __name__ == "__main__":
    main()
