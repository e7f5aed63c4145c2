"""Python face of the MI355X decode path, mirroring the reference's interface
for this path (names and argument meaning of crypto/ws_mask.h and
net/w_socket.h, error codes of ParseFrameHdr). Device memory, streams and
events come from torch; all compute runs in libfws_gpu.so's HIP kernels.
"""
import ctypes as C

import numpy as np
import torch

from . import _lib
from ._lib import DECODE_JOB, FRAME_DESC, FRAME_INFO, DECODE_RESULT, RX_EVENT, TX_DESC, GenParams, check, lib


def _stream_handle(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def _ptr(t):
    return C.c_void_p(t.data_ptr())


_hip = None


def hip_stream():
    """A HIP stream created with hipStreamNonBlocking, as the library's own
    pipelines create theirs (rx_pipe.cpp, rx_session.cpp), wrapped for torch.
    Two of these overlap two decodes every time; two torch pool streams did so
    only in some runs (tools/stream_pair_probe.py: 165-171 vs 176-208 us per
    C3 batch)."""
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
    s = C.c_void_p()
    if _hip.hipStreamCreateWithFlags(C.byref(s), C.c_uint(1)) != 0:
        raise RuntimeError("hipStreamCreateWithFlags failed")
    return HipStream(s.value)


class HipStream(torch.cuda.ExternalStream):
    """A stream from hip_stream(); close() (or leaving a `with` block)
    synchronizes and destroys it, so probes that make fresh pairs do not leak
    streams and their queue bindings."""

    def close(self):
        h = self.cuda_stream
        if h and _hip is not None and not getattr(self, "_closed", False):
            self._closed = True
            _hip.hipStreamSynchronize(C.c_void_p(h))
            _hip.hipStreamDestroy(C.c_void_p(h))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def device_count():
    n = C.c_int(0)
    check("fws_gpu_device_count", lib().fws_gpu_device_count(C.byref(n)))
    return n.value


class Ctx:
    """fws_gpu_ctx: device workspace for one device / one host thread."""

    def __init__(self, device=0, max_frames=0, max_stream_bytes=0):
        self.device = device
        h = C.c_void_p()
        check("fws_gpu_ctx_create", lib().fws_gpu_ctx_create(device, C.byref(h)))
        self.h = h
        if max_frames or max_stream_bytes:
            self.reserve(max_frames, max_stream_bytes)

    def reserve(self, max_frames, max_stream_bytes):
        check("fws_gpu_ctx_reserve", lib().fws_gpu_ctx_reserve(self.h, max_frames, max_stream_bytes))

    def set_rx_persistent(self, workers):
        """fws_gpu_ctx_set_rx_persistent: the context's small reads decoded by a
        resident grid of `workers` workgroups (0 = a launch per read)."""
        check("fws_gpu_ctx_set_rx_persistent", lib().fws_gpu_ctx_set_rx_persistent(self.h, workers))

    def rx_service_stats(self):
        """(grid launches, requests) of the persistent receive decode"""
        out = (C.c_uint64 * 2)()
        check("fws_internal_rx_service_stats", lib().fws_internal_rx_service_stats(self.h, out))
        return int(out[0]), int(out[1])

    def rx_service_pushes(self):
        """reads the persistent decode took pushed into device memory (push mode)"""
        out = (C.c_uint64 * 1)()
        check("fws_internal_rx_service_pushes", lib().fws_internal_rx_service_pushes(self.h, out))
        return int(out[0])

    def close(self):
        if self.h:
            lib().fws_gpu_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def ws_mask_bytes_fast(buf, key, offset=0, n=None, stream=None):
    """Device twin of fws::WSMaskBytesFast(src, size, mask) (ws_mask.h:175):
    XOR buf[offset:offset+n] (a uint8 CUDA tensor) with the 4-byte key in place."""
    n = buf.numel() - offset if n is None else n
    check("fws_gpu_mask", lib().fws_gpu_mask(C.c_void_p(buf.data_ptr() + offset), n, key & 0xFFFFFFFF,
                                             _stream_handle(stream)))


def descs_to_device(descs, device="cuda"):
    """numpy FRAME_DESC array -> uint8 device tensor holding the structs."""
    a = np.ascontiguousarray(descs, dtype=FRAME_DESC)
    return torch.from_numpy(a.view(np.uint8)).to(device)


def unmask_batch(ctx, base, dev_descs, n, stream=None):
    """fws_gpu_unmask_batch: unmask every payload region in place."""
    check("fws_gpu_unmask_batch", lib().fws_gpu_unmask_batch(ctx.h, _ptr(base), _ptr(dev_descs), n,
                                                             _stream_handle(stream)))


def unmask_sorted(ctx, base, dev_descs, n, stream=None):
    """fws_gpu_unmask_sorted: one-launch unmask of a sorted, non-overlapping batch."""
    check("fws_gpu_unmask_sorted", lib().fws_gpu_unmask_sorted(ctx.h, _ptr(base), _ptr(dev_descs), n,
                                                               _stream_handle(stream)))


def unmask_sorted_utf8(ctx, base, dev_descs, n, ok, stream=None):
    """fws_gpu_unmask_sorted_utf8: one-pass unmask + per-region UTF-8 flags (ok: device uint8[n])."""
    check("fws_gpu_unmask_sorted_utf8", lib().fws_gpu_unmask_sorted_utf8(ctx.h, _ptr(base), _ptr(dev_descs), n,
                                                                         _ptr(ok), _stream_handle(stream)))


def unmask_plan(ctx, base, dev_descs, n, stream=None):
    check("fws_gpu_unmask_plan", lib().fws_gpu_unmask_plan(ctx.h, _ptr(base), _ptr(dev_descs), n,
                                                           _stream_handle(stream)))


def unmask_run(ctx, base, dev_descs, n, stream=None):
    check("fws_gpu_unmask_run", lib().fws_gpu_unmask_run(ctx.h, _ptr(base), _ptr(dev_descs), n,
                                                         _stream_handle(stream)))


def unmask_gather(ctx, dst, src, dev_descs, n, stream=None):
    check("fws_gpu_unmask_gather", lib().fws_gpu_unmask_gather(ctx.h, _ptr(dst), _ptr(src), _ptr(dev_descs),
                                                               n, _stream_handle(stream)))


def decode_stream(ctx, wire, cap, frames=None, result=None, utf8_ok=None, stream=None, n=None):
    """fws_gpu_decode_stream on a device uint8 tensor. Returns (status, frames
    tensor, result tensor, utf8 tensor) -- device tensors, nothing synchronised."""
    dev = wire.device
    if frames is None:
        frames = torch.empty(max(cap, 1) * FRAME_INFO.itemsize, dtype=torch.uint8, device=dev)
    if result is None:
        result = torch.empty(DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev)
    n = wire.numel() if n is None else n
    u = C.c_void_p(utf8_ok.data_ptr()) if utf8_ok is not None else None
    rc = lib().fws_gpu_decode_stream(ctx.h, _ptr(wire), n, _ptr(frames), cap, _ptr(result), u,
                                     _stream_handle(stream))
    return rc, frames, result, utf8_ok


class DecodeEngine:
    """fws_decode_engine: fws_gpu_decode_stream over many independent streams,
    decodes kept in flight on two HIP streams. mode / scan_cus select the
    schedule through the library's tuning hooks (0: whole decodes alternating
    over the two streams, the default; 1: scans on one stream, resolve + unmask
    on the other, CU-partitioned when scan_cus > 0) -- for A/B runs only."""

    def __init__(self, device=0, max_frames=0, max_stream_bytes=0, mode=None, scan_cus=0):
        L = lib()
        old = None
        if mode is not None:
            old = (L.fws_internal_set_engine_mode(mode), L.fws_internal_set_engine_scan_cus(scan_cus))
        try:
            h = C.c_void_p()
            check("fws_decode_engine_create", L.fws_decode_engine_create(device, max_frames, max_stream_bytes,
                                                                         C.byref(h)))
        finally:
            if old is not None:
                L.fws_internal_set_engine_mode(old[0])
                L.fws_internal_set_engine_scan_cus(old[1])
        self.h = h

    def run(self, jobs, stream=None):
        """jobs: (wire, cap, frames, result[, utf8_ok]) tuples of device tensors
        (len = wire.numel()). Returns the status; nothing synchronised."""
        a = np.zeros(len(jobs), dtype=DECODE_JOB)
        for i, j in enumerate(jobs):
            wire, cap, frames, result = j[:4]
            u = j[4] if len(j) > 4 else None
            a[i] = (wire.data_ptr(), wire.numel(), frames.data_ptr(), cap, 0, result.data_ptr(),
                    u.data_ptr() if u is not None else 0)
        self._jobs = a                                   # alive until the next run
        return lib().fws_decode_engine_run(self.h, C.c_void_p(a.ctypes.data), len(jobs), _stream_handle(stream))

    def close(self):
        if self.h:
            lib().fws_decode_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def read_result(result):
    return np.frombuffer(result.cpu().numpy().tobytes(), dtype=DECODE_RESULT)[0]


def read_frames(frames, count):
    raw = frames[:count * FRAME_INFO.itemsize].cpu().numpy()
    return np.frombuffer(raw.tobytes(), dtype=FRAME_INFO).copy()


def validate_utf8(ctx, base, dev_descs, n, ok, stream=None):
    check("fws_gpu_validate_utf8", lib().fws_gpu_validate_utf8(ctx.h, _ptr(base), _ptr(dev_descs), n,
                                                               _ptr(ok), _stream_handle(stream)))


# ------------------------------------------------------------ workloads
GEN_FIXED, GEN_MIXED, GEN_FRAGMENTED, GEN_UTF8 = 0, 1, 2, 3


def gen_batch(kind, seed=42, opcode=2, n_frames=0, payload_min=0, payload_max=0, target_bytes=0,
              invalid_permille=0):
    """Synthetic client-masked frames (fws_gen_batch). Returns (wire uint8
    numpy array, FRAME_DESC array of payload regions, utf8_ok uint8 array)."""
    p = GenParams(seed=seed, kind=kind, opcode=opcode, n_frames=n_frames, payload_min=payload_min,
                  payload_max=payload_max, target_bytes=target_bytes,
                  invalid_permille=invalid_permille)
    wl, nf = C.c_uint64(0), C.c_uint64(0)
    check("fws_gen_batch", lib().fws_gen_batch(C.byref(p), None, 0, C.byref(wl), None, 0, C.byref(nf),
                                               None))
    wire = np.empty(wl.value, dtype=np.uint8)
    descs = np.zeros(nf.value, dtype=FRAME_DESC)
    ok = np.zeros(nf.value, dtype=np.uint8)
    check("fws_gen_batch", lib().fws_gen_batch(C.byref(p), wire.ctypes.data, wl.value, C.byref(wl),
                                               descs.ctypes.data, nf.value, C.byref(nf), ok.ctypes.data))
    return wire, descs, ok


# BASELINE.json configs as generator calls
def config_c2(seed=42, n_frames=65536, payload=4096):
    return gen_batch(GEN_FIXED, seed=seed, opcode=2, n_frames=n_frames, payload_min=payload)


def config_c3(seed=42, target=256 << 20):
    return gen_batch(GEN_MIXED, seed=seed, opcode=2, payload_min=64, payload_max=65536,
                     target_bytes=target)


def config_c4(seed=42, target=256 << 20):
    return gen_batch(GEN_FRAGMENTED, seed=seed, opcode=2, payload_min=4096, payload_max=1 << 20,
                     target_bytes=target)


def config_c5(seed=42, n_frames=262144, payload=16384, invalid_permille=10):
    return gen_batch(GEN_UTF8, seed=seed, n_frames=n_frames, payload_min=payload,
                     invalid_permille=invalid_permille)


# ------------------------------------------------------------ RX session
class HostArena:
    """Page-aligned host memory registered with fws_gpu_host_register: reads
    placed in it are decoded in place by RxSession / RxMux (the drop-in hook
    registers the reference's MemPool read buffers the same way)."""

    def __init__(self, nbytes):
        self.raw = np.zeros(nbytes + 8192, dtype=np.uint8)
        off = (-self.raw.ctypes.data) % 4096
        self.mem = self.raw[off:off + nbytes]
        check("fws_gpu_host_register", lib().fws_gpu_host_register(self.mem.ctypes.data, nbytes))
        self.pos = 0

    def place(self, data, align_off=0):
        """A view of the arena holding `data`, starting align_off bytes past a
        64-B boundary (the arena is reused round-robin)."""
        n = len(data)
        start = ((self.pos + 63) // 64) * 64 + align_off
        if start + n + 64 > len(self.mem):
            start = align_off
        v = self.mem[start:start + n]
        v[:] = np.frombuffer(bytes(data), dtype=np.uint8)
        self.pos = start + n
        return v

    def close(self):
        if self.mem is not None:
            lib().fws_gpu_host_unregister(self.mem.ctypes.data)
            self.mem = None


class RxSession:
    """fws_rx_session: OnRecvData (w_socket.h:543-769) over the GPU for host reads."""

    def __init__(self, ctx, is_server=True):
        h = C.c_void_p()
        check("fws_rx_session_create", lib().fws_rx_session_create(ctx.h, 1 if is_server else 0, C.byref(h)))
        self.h = h

    def feed(self, data, extra_cap=0, ev_cap=1 << 16, ctl_cap=1 << 20, arena=None, align_off=0):
        """arena: a HostArena to place the read in (decoded in place), else a fresh host copy."""
        buf = (arena.place(data, align_off) if arena is not None
               else np.frombuffer(bytes(data), dtype=np.uint8).copy())
        ev = np.zeros(ev_cap, dtype=RX_EVENT)
        ctl = np.zeros(ctl_cap, dtype=np.uint8)
        n_ev, ctl_used = C.c_uint64(0), C.c_uint64(0)
        ret = lib().fws_rx_session_feed(self.h, buf.ctypes.data if len(buf) else None, len(buf),
                                        len(buf) + extra_cap, ev.ctypes.data, ev_cap, C.byref(n_ev),
                                        ctl.ctypes.data, ctl_cap, C.byref(ctl_used))
        return ret, (buf.copy() if arena is not None else buf), ev[:n_ev.value].copy(), ctl[:ctl_used.value].copy()

    def state(self):
        st = _lib.RxState()
        check("fws_rx_session_state", lib().fws_rx_session_state(self.h, C.byref(st)))
        return st

    def close(self):
        if self.h:
            lib().fws_rx_session_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def check_sorted(ctx, dd, n, stream=None):
    """fws_gpu_check_sorted: the first descriptor index breaking the sorted /
    disjoint contract of unmask_sorted, or None (synchronises)."""
    bad = torch.empty(1, dtype=torch.int32, device=dd.device)
    st = stream if stream is not None else torch.cuda.current_stream()
    check("fws_gpu_check_sorted", lib().fws_gpu_check_sorted(ctx.h, dd.data_ptr(), n, bad.data_ptr(), st.cuda_stream))
    v = int(bad.item()) & 0xFFFFFFFF
    return None if v == 0xFFFFFFFF else v


class RxMux:
    """fws_rx_mux: the reads of many connections decoded in one round trip
    (FLoop::OneStep's shape, floop.h:661-703), each with its own carried state;
    per read the results equal RxSession.feed on that connection alone."""

    def __init__(self, ctx, n_conns):
        h = C.c_void_p()
        check("fws_rx_mux_create", lib().fws_rx_mux_create(ctx.h, n_conns, C.byref(h)))
        self.h = h
        self.n = n_conns

    def feed(self, reads, extra_cap=0, arena=None, align_off=None, between=None):
        """reads: [(conn, bytes)]. Returns [(ret, unmasked bytes, events, ctl bytes)].
        arena: a HostArena the reads are placed in (align_off(i) -> offset past a
        64-B boundary for read i), else fresh host copies. between: a callable run
        while the batch decodes (fws_rx_mux_submit, between(), fws_rx_mux_complete)
        instead of one fws_rx_mux_feed."""
        bufs = [arena.place(d, align_off(i) if align_off else 0) if arena is not None
                else np.frombuffer(bytes(d), dtype=np.uint8).copy() for i, (_, d) in enumerate(reads)]
        rr = np.zeros(len(reads), dtype=_lib.RX_READ)
        for i, ((conn, _), b) in enumerate(zip(reads, bufs)):
            rr[i] = (conn, 0, b.ctypes.data if len(b) else 0, len(b), len(b) + extra_cap)
        out = np.zeros(len(reads), dtype=_lib.RX_READ_RESULT)
        if between is None:
            check("fws_rx_mux_feed", lib().fws_rx_mux_feed(self.h, rr.ctypes.data if len(reads) else None,
                                                           len(reads), out.ctypes.data if len(reads) else None))
        else:
            check("fws_rx_mux_submit", lib().fws_rx_mux_submit(self.h, rr.ctypes.data if len(reads) else None,
                                                               len(reads)))
            between()
            check("fws_rx_mux_complete", lib().fws_rx_mux_complete(self.h, out.ctypes.data if len(reads) else None))
        res = []
        for i, b in enumerate(bufs):
            o = out[i]
            n_ev, n_ctl = int(o["n_events"]), int(o["ctl_used"])
            ev = np.zeros(n_ev, dtype=RX_EVENT)
            if n_ev:
                C.memmove(ev.ctypes.data, int(o["events"]), n_ev * RX_EVENT.itemsize)
            ctl = np.zeros(n_ctl, dtype=np.uint8)
            if n_ctl:
                C.memmove(ctl.ctypes.data, int(o["ctl"]), n_ctl)
            res.append((int(o["ret"]), b.copy() if arena is not None else b, ev, ctl))
        return res

    def submit_raw(self, rr, n):
        """fws_rx_mux_submit on a prepared RX_READ array (tests); returns the code"""
        return int(lib().fws_rx_mux_submit(self.h, rr.ctypes.data if n else None, n))

    def complete_raw(self, out):
        """fws_rx_mux_complete into a prepared RX_READ_RESULT array (tests); returns the code"""
        return int(lib().fws_rx_mux_complete(self.h, out.ctypes.data if len(out) else None))

    def reset(self, conn):
        check("fws_rx_mux_reset", lib().fws_rx_mux_reset(self.h, conn))

    def state(self, conn):
        st = _lib.RxState()
        check("fws_rx_mux_state", lib().fws_rx_mux_state(self.h, conn, C.byref(st)))
        return st

    def close(self):
        if self.h:
            lib().fws_rx_mux_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class TxSession:
    """fws_tx_session: SendFrame (w_socket.h:832-944) for host payloads of one
    connection; the frame bytes are built on the GPU."""

    def __init__(self, ctx, is_server=False):
        h = C.c_void_p()
        check("fws_tx_session_create", lib().fws_tx_session_create(ctx.h, 1 if is_server else 0, C.byref(h)))
        self.h = h

    def send(self, frames, out_cap=None):
        """frames: [(payload bytes, frame_type, last, key)]. Returns (rc, wire
        bytes, needed length); rc != 0 leaves the session state unchanged."""
        n = len(frames)
        bufs = [np.frombuffer(bytes(p), dtype=np.uint8).copy() for p, _, _, _ in frames]
        ptrs = np.array([b.ctypes.data if len(b) else 0 for b in bufs], dtype=np.uint64)
        lens = np.array([len(b) for b in bufs], dtype=np.uint64)
        types = np.array([f[1] for f in frames], dtype=np.uint32)
        last = np.array([1 if f[2] else 0 for f in frames], dtype=np.uint8)
        keys = np.array([f[3] & 0xFFFFFFFF for f in frames], dtype=np.uint32)
        cap = int(lens.sum()) + 14 * n if out_cap is None else out_cap
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        ol = C.c_uint64(0)
        rc = lib().fws_tx_session_send(self.h, ptrs.ctypes.data, lens.ctypes.data, types.ctypes.data,
                                       last.ctypes.data, keys.ctypes.data, n, out.ctypes.data, cap, C.byref(ol))
        return rc, out[:ol.value].tobytes() if rc == 0 else b"", ol.value

    def last_msg_not_fin(self):
        v = C.c_uint8(0)
        check("fws_tx_session_state", lib().fws_tx_session_state(self.h, C.byref(v)))
        return v.value

    def close(self):
        if self.h:
            lib().fws_tx_session_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def plan_mode(ctx):
    """The last descriptor plan's mode (diagnostic; synchronises): dict with
    byte_space (payloads sorted and disjoint: byte-space unmask), s0, first_po,
    last_pe, n_units."""
    out = (C.c_uint64 * 5)()
    check("fws_internal_plan_mode", lib().fws_internal_plan_mode(ctx.h, out))
    return dict(zip(("byte_space", "s0", "first_po", "last_pe", "n_units"), list(out)))


def decode_counters(ctx):
    """The last decode's counters on ctx (decode_common.h Counter; diagnostic,
    synchronises): survivors, frames, big-ST super tiles, failure flag."""
    out = (C.c_uint32 * 16)()
    check("fws_internal_decode_counters", lib().fws_internal_decode_counters(ctx.h, out, 16))
    return {"survivors": out[0], "frames": out[3], "failed": out[9] != 0, "big_super_tiles": out[12]}


class RxPipe:
    """fws_rx_pipe: batched, pipelined decode of host batches (H2D -> parse +
    unmask -> D2H on `depth` streams). Batches are pinned CPU uint8 tensors;
    each is unmasked in place once its wait() returns."""

    def __init__(self, device=0, max_batch_bytes=1 << 28, max_frames=1 << 17, depth=3, utf8=False):
        h = C.c_void_p()
        check("fws_rx_pipe_create", lib().fws_rx_pipe_create(device, max_batch_bytes, max_frames, depth,
                                                             1 if utf8 else 0, C.byref(h)))
        self.h = h
        self.max_frames = max_frames
        self.utf8 = utf8

    def submit(self, batch, n=None):
        t = C.c_uint64()
        n = batch.numel() if n is None else n
        check("fws_rx_pipe_submit", lib().fws_rx_pipe_submit(self.h, C.c_void_p(batch.data_ptr()), n, C.byref(t)))
        return t.value

    def wait(self, ticket, copy_frames=True):
        """(frames structured array, result record, utf8 flags or None)."""
        fp, up = C.c_void_p(), C.c_void_p()
        nf = C.c_uint64()
        res = np.zeros(1, dtype=DECODE_RESULT)
        check("fws_rx_pipe_wait", lib().fws_rx_pipe_wait(self.h, ticket, C.byref(fp), C.byref(nf),
                                                         C.c_void_p(res.ctypes.data), C.byref(up)))
        frames = None
        if copy_frames and nf.value:
            raw = (C.c_uint8 * (nf.value * FRAME_INFO.itemsize)).from_address(fp.value)
            frames = np.frombuffer(bytes(raw), dtype=FRAME_INFO)
        ok = None
        if self.utf8 and nf.value:
            ok = np.frombuffer(bytes((C.c_uint8 * nf.value).from_address(up.value)), dtype=np.uint8)
        return frames, res[0], ok

    def close(self):
        if self.h:
            lib().fws_rx_pipe_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def encode_frames(ctx, out, src, dev_descs, n, out_len=None, stream=None):
    """fws_gpu_encode_frames: out (device uint8, 16-B aligned) = the frames of
    dev_descs (device TX_DESC bytes) back to back. Returns the device u64 total
    tensor (~0 if out is too small); nothing synchronised."""
    if out_len is None:
        out_len = torch.empty(1, dtype=torch.int64, device=out.device)
    check("fws_gpu_encode_frames", lib().fws_gpu_encode_frames(ctx.h, _ptr(out), out.numel(), _ptr(src),
                                                               _ptr(dev_descs), n, _ptr(out_len),
                                                               _stream_handle(stream)))
    return out_len


class TxState:
    """One connection's send sequencing (fws_tx_next, SendFrame's opcode / FIN rule)."""

    def __init__(self):
        self.last_msg_not_fin = C.c_uint8(0)

    def next(self, frame_type, last):
        op, fin = C.c_uint8(), C.c_uint8()
        lib().fws_tx_next(frame_type, int(last), C.byref(self.last_msg_not_fin), C.byref(op), C.byref(fin))
        return op.value, fin.value
