"""CPU: the C-ABI library loads and exports every function include/fws_gpu.h
declares; struct layouts agree between the header and the Python mirror; the
synthetic workload generator (host code) produces streams the oracle decodes
into exactly the frames it reports. No device calls."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import orc
from flashws_amd import _lib, gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fws_gpu.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fws_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_abi():
    names = declared_functions()
    assert "fws_gpu_decode_stream" in names and "fws_gpu_mask" in names
    assert len(names) >= 15


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing


def test_library_resolves_every_symbol_at_load():
    """dlopen with RTLD_NOW: an internal symbol left undefined (a stale object
    after a signature change) fails here, on the CPU, not on the GPU box."""
    C.CDLL(_lib.LIB_PATH, mode=os.RTLD_NOW | os.RTLD_LOCAL)


def test_python_signatures_cover_the_header():
    assert set(declared_functions()) == {n for n, _, _ in _lib.SIGNATURES}


def test_struct_sizes_match_header_comments():
    src = open(HEADER).read()
    sizes = dict(re.findall(r"\}\s*(fws_[a-z_]+);\s*/\*\s*(\d+) bytes", src))
    assert int(sizes["fws_frame_desc"]) == _lib.FRAME_DESC.itemsize
    assert int(sizes["fws_frame_info"]) == _lib.FRAME_INFO.itemsize
    assert int(sizes["fws_decode_result"]) == _lib.DECODE_RESULT.itemsize
    assert int(sizes["fws_rx_event"]) == _lib.RX_EVENT.itemsize
    assert int(sizes["fws_rx_state"]) == C.sizeof(_lib.RxState)


def test_abi_version_and_error_codes_are_reference_codes():
    assert _lib.lib().fws_gpu_abi_version() == 1
    # ParseFrameHdr's return values (w_socket.h:451-521) are the ABI's codes
    assert (_lib.FWS_ERR_RSV, _lib.FWS_ERR_TOO_LARGE, _lib.FWS_ERR_NOT_MASKED, _lib.FWS_ERR_MASKED,
            _lib.FWS_ERR_OPCODE) == (orc.orc() and -1, -2, -3, -4, -9)


def test_invalid_arguments_fail_without_a_device():
    L = _lib.lib()
    assert L.fws_gpu_ctx_create(0, None) == _lib.FWS_ERR_INVALID
    assert L.fws_gpu_unmask_batch(None, None, None, 1, None) == _lib.FWS_ERR_INVALID
    assert L.fws_gpu_unmask_sorted(None, None, None, 1, None) == _lib.FWS_ERR_INVALID
    assert L.fws_gpu_unmask_sorted_utf8(None, None, None, 1, None, None) == _lib.FWS_ERR_INVALID
    assert L.fws_gpu_decode_stream(None, None, 0, None, 0, None, None, None) == _lib.FWS_ERR_INVALID


@pytest.mark.parametrize("cfg", ["c2", "c3", "c4", "c5"])
def test_generator_streams_decode_to_their_descriptors(cfg):
    wire, descs, ok = {"c2": lambda: gpu.config_c2(n_frames=300),
                       "c3": lambda: gpu.config_c3(target=4 << 20),
                       "c4": lambda: gpu.config_c4(target=8 << 20),
                       "c5": lambda: gpu.config_c5(n_frames=300, payload=2000, invalid_permille=50)}[cfg]()
    buf = wire.copy()
    ret, frames, _, consumed = orc.orc_decode_stream(buf)
    assert ret == 0 and consumed == len(wire) and len(frames) == len(descs)
    assert np.array_equal(frames["hdr_off"] + frames["hdr_len"], descs["payload_off"])
    assert np.array_equal(frames["payload_len"], descs["payload_len"])
    assert np.array_equal(frames["key"], descs["key"])
    if cfg == "c4":
        assert frames["opcode"][0] == 2 and (frames["opcode"][1:] == 0).all()
        assert (frames["fin"][:-1] == 0).all() and frames["fin"][-1] == 1
        assert int(descs["payload_len"].sum()) == 8 << 20
    if cfg == "c5":
        for (o, n), good in zip(zip(descs["payload_off"], descs["payload_len"]), ok):
            try:
                buf[o:o + n].tobytes().decode("utf-8")
                v = 1
            except UnicodeDecodeError:
                v = 0
            assert v == good
        assert 0 < ok.sum() < len(ok)

