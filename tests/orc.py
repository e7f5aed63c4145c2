"""ctypes bindings for the TEST-ONLY oracle (oracle/liborc.so) and, when it has
been built in this container, the compiled reference (oracle/_ref/libfwsref.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORC_SO = os.path.join(ORACLE_DIR, "liborc.so")
REF_SO = os.path.join(ORACLE_DIR, "_ref", "libfwsref.so")

EVENT_DTYPE = np.dtype([
    ("kind", "<u4"), ("opcode", "<u4"), ("is_ctl", "u1"), ("frame_end", "u1"),
    ("msg_end", "u1"), ("fin", "u1"), ("key", "<u4"), ("size", "<u8"),
    ("data_off", "<u8"), ("ctl_off", "<u8"), ("capacity", "<u8")])
assert EVENT_DTYPE.itemsize == 48

FRAME_DTYPE = np.dtype([("hdr_off", "<u8"), ("payload_len", "<u8"), ("key", "<u4"),
                        ("opcode", "u1"), ("fin", "u1"), ("hdr_len", "u1"), ("pad", "u1")])
assert FRAME_DTYPE.itemsize == 24

# orc_rx_state is 184 bytes; treat it as an opaque blob with the leading fields typed.
RX_STATE_SIZE = 4 + 4 + 8 + 4 + 4 + 14 + 128 + 4 + 4
RX_STATE_SIZE = (RX_STATE_SIZE + 7) // 8 * 8


class RxStateHead(C.Structure):
    _fields_ = [("recv_status", C.c_int32), ("last_rx_mask_key", C.c_uint32),
                ("unread_pl_len", C.c_uint64), ("last_rx_opcode", C.c_uint8),
                ("last_rx_control_opcode", C.c_uint8), ("last_rx_fin_flag", C.c_uint8),
                ("is_rx_control_frame", C.c_uint8), ("last_rx_hdr_part_len", C.c_uint32)]


_orc = None
_ref = None


def _u8p(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def orc():
    """Load (building if needed) the C restatement."""
    global _orc
    if _orc is None:
        if not os.path.exists(ORC_SO):
            subprocess.check_call(["make", "-s", "liborc.so"], cwd=ORACLE_DIR)
        lib = C.CDLL(ORC_SO)
        for n in ("orc_mask1", "orc_ws_mask_bytes", "orc_mask_avx2",
                  "orc_mask_large_chunk_avx2", "orc_ws_mask_fast"):
            getattr(lib, n).argtypes = [C.c_void_p, C.c_size_t, C.c_uint32]
            getattr(lib, n).restype = None
        lib.orc_rotr32.argtypes = [C.c_uint32, C.c_uint32]
        lib.orc_rotr32.restype = C.c_uint32
        lib.orc_rx_init.argtypes = [C.c_void_p, C.c_int]
        lib.orc_on_recv_data.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t,
                                         C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t),
                                         C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
        lib.orc_on_recv_data.restype = C.c_int
        lib.orc_decode_stream.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                          C.POINTER(C.c_size_t), C.POINTER(C.c_size_t),
                                          C.POINTER(C.c_size_t)]
        lib.orc_decode_stream.restype = C.c_int
        lib.orc_reassemble.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        lib.orc_reassemble.restype = C.c_size_t
        lib.orc_utf8_valid.argtypes = [C.c_void_p, C.c_size_t]
        lib.orc_tx_hdr_size.argtypes = [C.c_size_t, C.c_int]
        lib.orc_tx_hdr_size.restype = C.c_size_t
        lib.orc_tx_frame.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t, C.c_uint32, C.c_int,
                                     C.c_uint32, C.c_void_p]
        lib.orc_tx_frame.restype = C.c_size_t
        lib.orc_utf8_valid.restype = C.c_int
        _orc = lib
    return _orc


def ref_available():
    return os.path.exists(REF_SO)


def ref():
    """The compiled reference (container-built; travels to the GPU box as a .so)."""
    global _ref
    if _ref is None:
        lib = C.CDLL(REF_SO)
        for n in ("ref_ws_mask_fast", "ref_ws_mask_bytes", "ref_mask1", "ref_mask_avx2",
                  "ref_mask_large_chunk_avx2"):
            getattr(lib, n).argtypes = [C.c_void_p, C.c_size_t, C.c_uint32]
            getattr(lib, n).restype = None
        lib.ref_rotr32.argtypes = [C.c_uint32, C.c_uint32]
        lib.ref_rotr32.restype = C.c_uint32
        lib.ref_session_new.restype = C.c_void_p
        lib.ref_session_free.argtypes = [C.c_void_p]
        lib.ref_session_feed.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                         C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t),
                                         C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
        lib.ref_session_feed.restype = C.c_int
        lib.ref_session_state.argtypes = [C.c_void_p, C.c_void_p]
        lib.ref_time_onrecv.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_int,
                                        C.POINTER(C.c_uint64), C.POINTER(C.c_int)]
        lib.ref_time_onrecv.restype = C.c_double
        lib.ref_time_mask_parts.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.c_size_t, C.c_int]
        lib.ref_time_mask_parts.restype = C.c_double
        _ref = lib
    return _ref


# ---------------------------------------------------------------- mask helpers
MASK_FUNCS = ("mask1", "ws_mask_bytes", "mask_avx2", "mask_large_chunk_avx2", "ws_mask_fast")


def orc_mask(name, buf, key, off=0, n=None):
    """In-place mask of buf[off:off+n] (numpy uint8) with the oracle variant `name`."""
    n = len(buf) - off if n is None else n
    getattr(orc(), "orc_" + name)(buf.ctypes.data + off, n, key)


def ref_mask(name, buf, key, off=0, n=None):
    n = len(buf) - off if n is None else n
    getattr(ref(), "ref_" + name)(buf.ctypes.data + off, n, key)


# ---------------------------------------------------------------- RX sessions
class OrcSession:
    """Oracle WSocket RX state machine (server), fed one read at a time."""

    def __init__(self, is_server=True):
        self.state = C.create_string_buffer(512)
        orc().orc_rx_init(self.state, 1 if is_server else 0)

    def feed(self, data, extra_cap=0, ev_cap=1 << 16, ctl_cap=1 << 20):
        buf = np.frombuffer(bytes(data), dtype=np.uint8).copy()
        ev = np.zeros(ev_cap, dtype=EVENT_DTYPE)
        ctl = np.zeros(ctl_cap, dtype=np.uint8)
        n_ev, ctl_used = C.c_size_t(0), C.c_size_t(0)
        ret = orc().orc_on_recv_data(self.state, buf.ctypes.data if len(buf) else None, len(buf),
                                     len(buf) + extra_cap, ev.ctypes.data, ev_cap, C.byref(n_ev),
                                     ctl.ctypes.data, ctl_cap, C.byref(ctl_used))
        return ret, buf, ev[:n_ev.value].copy(), ctl[:ctl_used.value].copy()

    def head(self):
        return RxStateHead.from_buffer_copy(self.state.raw[:C.sizeof(RxStateHead)])


class RefSession:
    """The real reference's WSServerSocket<false>::OnRecvData (container only)."""

    def __init__(self):
        self.h = ref().ref_session_new()
        assert self.h

    def __del__(self):
        try:
            ref().ref_session_free(self.h)
        except Exception:
            pass

    def feed(self, data, extra_cap=0, ev_cap=1 << 16, ctl_cap=1 << 20):
        src = np.frombuffer(bytes(data), dtype=np.uint8).copy()
        out = np.zeros(len(src), dtype=np.uint8)
        ev = np.zeros(ev_cap, dtype=EVENT_DTYPE)
        ctl = np.zeros(ctl_cap, dtype=np.uint8)
        n_ev, ctl_used = C.c_size_t(0), C.c_size_t(0)
        ret = ref().ref_session_feed(self.h, src.ctypes.data if len(src) else None, len(src),
                                     out.ctypes.data if len(out) else None, extra_cap,
                                     ev.ctypes.data, ev_cap, C.byref(n_ev),
                                     ctl.ctypes.data, ctl_cap, C.byref(ctl_used))
        return ret, out, ev[:n_ev.value].copy(), ctl[:ctl_used.value].copy()

    def head(self):
        st = RxStateHead()
        ref().ref_session_state(self.h, C.byref(st))
        return st


def orc_decode_stream(buf, frames_cap=None):
    """In-place decode of a complete server stream (numpy uint8). Returns
    (ret, frames[FRAME_DTYPE], err_off, consumed)."""
    if frames_cap is None:
        frames_cap = max(16, len(buf) // 6 + 1)
    frames = np.zeros(frames_cap, dtype=FRAME_DTYPE)
    nf, eo, cons = C.c_size_t(0), C.c_size_t(0), C.c_size_t(0)
    ret = orc().orc_decode_stream(buf.ctypes.data, len(buf), frames.ctypes.data, frames_cap,
                                  C.byref(nf), C.byref(eo), C.byref(cons))
    return ret, frames[:min(nf.value, frames_cap)].copy(), eo.value, cons.value


def orc_utf8_valid(b):
    a = np.frombuffer(bytes(b), dtype=np.uint8)
    return bool(orc().orc_utf8_valid(a.ctypes.data if len(a) else None, len(a)))


# ---------------------------------------------------------------- comparisons
def user_visible(ev, ctl):
    """Events as the reference's user / peer sees them: on_read deliveries
    (kind 0), PONG replies (1), CLOSE (2: code + reason, 5: echoed payload).
    FRAME_HDR bookkeeping (kind 3) is oracle-only and dropped."""
    out = []
    for e in ev:
        k = int(e["kind"])
        if k == 3:
            continue
        rec = {"kind": k, "opcode": int(e["opcode"]), "is_ctl": int(e["is_ctl"]),
               "frame_end": int(e["frame_end"]), "msg_end": int(e["msg_end"]),
               "size": int(e["size"])}
        if k == 0 and not e["is_ctl"]:
            rec["data_off"] = int(e["data_off"])
            rec["capacity"] = int(e["capacity"])
        else:
            o = int(e["ctl_off"])
            rec["ctl"] = bytes(ctl[o:o + int(e["size"])])
        if k == 2:
            rec["code"] = int(e["key"])
        out.append(rec)
    return out


def orc_to_reference_view(ev, ctl):
    """Map oracle events onto what the reference driver records: a CLOSE frame
    produces the echoed frame (kind 5, full payload) followed by on_close
    (kind 2, reason only = payload[2:] when >= 2 bytes)."""
    out = []
    for rec in user_visible(ev, ctl):
        if rec["kind"] == 2:
            payload = rec["ctl"]
            echo = dict(kind=5, opcode=8, is_ctl=1, frame_end=1, msg_end=1,
                        size=len(payload), ctl=payload)
            out.append(echo)
            reason = payload[2:] if len(payload) >= 2 else b""
            out.append(dict(kind=2, opcode=8, is_ctl=1, frame_end=1, msg_end=1,
                            size=len(reason), ctl=reason, code=rec["code"]))
        else:
            out.append(rec)
    return out


class OrcTx:
    """The oracle's SendFrame byte builder for one connection (orc_tx_frame)."""

    def __init__(self, is_server=False):
        self.state = C.c_int(0)
        self.is_server = int(is_server)

    def frame(self, payload, frame_type, last, key):
        n = len(payload)
        out = (C.c_uint8 * (n + 14))()
        src = (C.c_uint8 * max(n, 1)).from_buffer_copy(bytes(payload) or b"\0")
        k = orc().orc_tx_frame(C.byref(self.state), self.is_server, src, n, frame_type, int(last), key & 0xFFFFFFFF,
                               out)
        return bytes(out[:k])


def ref_tx_session(is_server=False):
    """A real reference WSClientSocket (or WSServerSocket) over a socketpair
    (oracle/_ref); write(payload, frame_type, last) returns the frame bytes."""
    L = ref()
    if not getattr(L, "_tx_bound", False):
        L.ref_tx_new.restype = C.c_void_p
        L.ref_tx_new.argtypes = [C.c_int]
        L.ref_tx_free.argtypes = [C.c_void_p]
        L.ref_tx_write.restype = C.c_long
        L.ref_tx_write.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_int, C.c_void_p,
                                   C.c_size_t, C.POINTER(C.c_size_t)]
        L._tx_bound = True
    h = L.ref_tx_new(int(is_server))

    def write(payload, frame_type, last):
        n = len(payload)
        out = (C.c_uint8 * (n + 14))()
        src = (C.c_uint8 * max(n, 1)).from_buffer_copy(bytes(payload) or b"\0")
        got = C.c_size_t()
        r = L.ref_tx_write(h, src, n, frame_type, int(last), out, n + 14, C.byref(got))
        assert r == n, r
        return bytes(out[:got.value])

    return h, write
