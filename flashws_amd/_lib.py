"""ctypes binding of libfws_gpu.so (include/fws_gpu.h).

Loads the in-tree build (flashws_amd/lib/libfws_gpu.so) and fails loudly when
it is missing: there is no CPU fallback anywhere on the product path.

torch is imported first on purpose: it loads its bundled libamdhip64.so.7 and
libfws_gpu.so then binds to that same HIP runtime (same SONAME), so torch
tensors' device pointers and torch streams are valid handles for the ABI.
"""
import ctypes as C
import os

import numpy as np

try:  # noqa: SIM105 - see module docstring
    import torch  # noqa: F401
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# FWS_LIB_VARIANT=<tag> loads an in-tree A/B build, lib/libfws_gpu_<tag>.so (make exp), e.g. to run
# the parity tests on an experimental kernel; unset, the product library
_VARIANT = os.environ.get("FWS_LIB_VARIANT", "")
LIB_PATH = os.path.join(PKG_DIR, "lib", f"libfws_gpu_{_VARIANT}.so" if _VARIANT else "libfws_gpu.so")

FWS_OK = 0
FWS_ERR_RSV = -1
FWS_ERR_TOO_LARGE = -2
FWS_ERR_NOT_MASKED = -3
FWS_ERR_MASKED = -4
FWS_ERR_OPCODE = -9
FWS_ERR_CONTROL_FRAME = -10
FWS_ERR_CAPACITY = -20
FWS_ERR_INVALID = -21
FWS_ERR_NO_DEVICE = -22
FWS_ERR_INTERNAL = -23
FWS_ERR_HIP_BASE = -1000

# include/fws_gpu.h structs as numpy dtypes (device arrays are torch uint8 views)
FRAME_DESC = np.dtype([("payload_off", "<u8"), ("payload_len", "<u8"), ("key", "<u4"),
                       ("phase", "<u4")])
FRAME_INFO = np.dtype([("hdr_off", "<u8"), ("payload_len", "<u8"), ("key", "<u4"),
                       ("opcode", "u1"), ("fin", "u1"), ("hdr_len", "u1"), ("flags", "u1")])
DECODE_RESULT = np.dtype([("status", "<i4"), ("n_frames", "<u4"), ("consumed", "<u8"),
                          ("err_off", "<u8"), ("carry_unread", "<u8"), ("carry_hdr_len", "<u4"),
                          ("n_survivors", "<u4")])
RX_EVENT = np.dtype([("kind", "<u4"), ("opcode", "<u4"), ("is_ctl", "u1"), ("frame_end", "u1"),
                     ("msg_end", "u1"), ("fin", "u1"), ("code", "<u4"), ("size", "<u8"),
                     ("data_off", "<u8"), ("ctl_off", "<u8"), ("capacity", "<u8")])
TX_DESC = np.dtype([("src_off", "<u8"), ("len", "<u8"), ("key", "<u4"), ("opcode", "u1"), ("fin", "u1"),
                    ("masked", "u1"), ("pad", "u1")])
assert FRAME_DESC.itemsize == 24 and FRAME_INFO.itemsize == 24 and TX_DESC.itemsize == 24
assert DECODE_RESULT.itemsize == 40 and RX_EVENT.itemsize == 48
RX_READ = np.dtype([("conn", "<u4"), ("flags", "<u4"), ("buf", "<u8"), ("size", "<u8"), ("capacity", "<u8")])
RX_READ_RESULT = np.dtype([("ret", "<i4"), ("pad", "<u4"), ("events", "<u8"), ("n_events", "<u8"),
                           ("ctl", "<u8"), ("ctl_used", "<u8")])
assert RX_READ.itemsize == 32 and RX_READ_RESULT.itemsize == 40
DECODE_JOB = np.dtype([("wire", "<u8"), ("len", "<u8"), ("frames", "<u8"), ("cap", "<u4"), ("reserved", "<u4"),
                       ("result", "<u8"), ("utf8_ok", "<u8")])
assert DECODE_JOB.itemsize == 48


class RxState(C.Structure):
    """fws_rx_state (field names of the reference's members, w_socket.h:223-245)."""
    _fields_ = [("recv_status", C.c_int32), ("last_rx_mask_key", C.c_uint32),
                ("unread_pl_len", C.c_uint64), ("last_rx_opcode", C.c_uint8),
                ("last_rx_control_opcode", C.c_uint8), ("last_rx_fin_flag", C.c_uint8),
                ("is_rx_control_frame", C.c_uint8), ("last_rx_hdr_part_len", C.c_uint32)]


class GenParams(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("kind", C.c_uint32), ("opcode", C.c_uint32),
                ("n_frames", C.c_uint64), ("payload_min", C.c_uint64), ("payload_max", C.c_uint64),
                ("target_bytes", C.c_uint64), ("invalid_permille", C.c_uint32),
                ("pad_", C.c_uint32)]


# (name, restype, argtypes) for every symbol include/fws_gpu.h declares
_P, _U32, _U64, _I = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
_PU64 = C.POINTER(C.c_uint64)
SIGNATURES = [
    ("fws_gpu_abi_version", _I, []),
    ("fws_gpu_device_count", _I, [C.POINTER(C.c_int)]),
    ("fws_gpu_ctx_create", _I, [_I, C.POINTER(C.c_void_p)]),
    ("fws_gpu_ctx_destroy", None, [_P]),
    ("fws_gpu_ctx_reserve", _I, [_P, _U64, _U64]),
    ("fws_gpu_ctx_set_rx_persistent", _I, [_P, _U32]),
    ("fws_gpu_mask", _I, [_P, _U64, _U32, _P]),
    ("fws_gpu_unmask_batch", _I, [_P, _P, _P, _U32, _P]),
    ("fws_gpu_unmask_sorted", _I, [_P, _P, _P, _U32, _P]),
    ("fws_gpu_unmask_sorted_utf8", _I, [_P, _P, _P, _U32, _P, _P]),
    ("fws_gpu_unmask_plan", _I, [_P, _P, _P, _U32, _P]),
    ("fws_gpu_unmask_run", _I, [_P, _P, _P, _U32, _P]),
    ("fws_gpu_unmask_gather", _I, [_P, _P, _P, _P, _U32, _P]),
    ("fws_gpu_decode_stream", _I, [_P, _P, _U64, _P, _U32, _P, _P, _P]),
    ("fws_gpu_validate_utf8", _I, [_P, _P, _P, _U32, _P, _P]),
    ("fws_rx_session_create", _I, [_P, _I, C.POINTER(C.c_void_p)]),
    ("fws_rx_session_destroy", None, [_P]),
    ("fws_rx_session_feed", _I, [_P, _P, _U64, _U64, _P, _U64, _PU64, _P, _U64, _PU64]),
    ("fws_rx_session_state", _I, [_P, _P]),
    ("fws_rx_session_feed_view", _I, [_P, _P, _U64, _U64, C.POINTER(C.c_void_p), _PU64, C.POINTER(C.c_void_p),
                                      _PU64]),
    ("fws_rx_session_error", _I, [_P, C.POINTER(C.c_uint32)]),
    ("fws_gpu_check_sorted", _I, [_P, _P, _U32, _P, _P]),
    ("fws_rx_mux_create", _I, [_P, _U32, C.POINTER(C.c_void_p)]),
    ("fws_rx_mux_destroy", None, [_P]),
    ("fws_rx_mux_reset", _I, [_P, _U32]),
    ("fws_rx_mux_state", _I, [_P, _U32, _P]),
    ("fws_rx_mux_error", _I, [_P, _U32, C.POINTER(C.c_uint32)]),
    ("fws_rx_mux_feed", _I, [_P, _P, _U32, _P]),
    ("fws_rx_mux_submit", _I, [_P, _P, _U32]),
    ("fws_rx_mux_complete", _I, [_P, _P]),
    ("fws_rx_mux_ready", _I, [_P]),
    ("fws_gen_batch", _I, [C.POINTER(GenParams), _P, _U64, _PU64, _P, _U64, _PU64, _P]),
    ("fws_tx_next", None, [_U32, _I, C.POINTER(C.c_uint8), C.POINTER(C.c_uint8), C.POINTER(C.c_uint8)]),
    ("fws_gpu_encode_frames", _I, [_P, _P, _U64, _P, _P, _U32, _P, _P]),
    ("fws_tx_session_create", _I, [_P, _I, C.POINTER(C.c_void_p)]),
    ("fws_tx_session_destroy", None, [_P]),
    ("fws_tx_session_send", _I, [_P, _P, _P, _P, _P, _P, _U32, _P, _U64, _PU64]),
    ("fws_tx_session_state", _I, [_P, C.POINTER(C.c_uint8)]),
    ("fws_gpu_host_register", _I, [_P, _U64]),
    ("fws_gpu_host_unregister", _I, [_P]),
    ("fws_rx_pipe_create", _I, [_I, _U64, _U32, _U32, _I, C.POINTER(C.c_void_p)]),
    ("fws_rx_pipe_destroy", None, [_P]),
    ("fws_rx_pipe_submit", _I, [_P, _P, _U64, _PU64]),
    ("fws_rx_pipe_wait", _I, [_P, _U64, C.POINTER(C.c_void_p), _PU64, _P, C.POINTER(C.c_void_p)]),
    ("fws_decode_engine_create", _I, [_I, _U64, _U64, C.POINTER(C.c_void_p)]),
    ("fws_decode_engine_destroy", None, [_P]),
    ("fws_decode_engine_run", _I, [_P, _P, _U32, _P]),
]

_lib = None


class FwsError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__(f"{fn} failed with status {code}")
        self.code = code


def lib():
    """The loaded library. Raises if the in-tree build is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                f"g.build()'` (make -C flashws_amd/csrc). There is no CPU fallback.")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name, None)
            if fn is None:
                continue  # reported by exported_symbols(); callers fail on use
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def exported_symbols():
    """Names from SIGNATURES that the library actually exports."""
    L = lib()
    return [n for n, _, _ in SIGNATURES if hasattr(L, n)]


def check(fn, code):
    if code != 0:
        raise FwsError(fn, code)
    return code
