// small_kernels.hip -- one-launch decode of a small read (the RX session's
// per-read path, rx_session.cpp): header parse + unmask of a stream of at
// most kSmallMax bytes by one workgroup.
//
// The multi-launch stream decode (k_scan -> k_merge -> k_link -> k_emit ->
// k_resolve -> k_unmask_stream, decode_kernels.hip / merge_kernels.hip) is
// built for HBM-sized streams; on a 4 KiB read its six launches cost ~40 us of
// dependent latency, more than the read's PCIe copies. Here the stream is
// staged in LDS with one round of 16-B loads, the header chain is walked from
// offset 0 by one lane with ParseFrameHdr's exact semantics (w_socket.h:435-524,
// loop w_socket.h:543-769; the same walk the super-tile resolve finishes its
// terminal with), and every 16-B chunk holding payload bytes is unmasked from
// LDS by the whole workgroup and stored once.
//
// k_decode_segments does the same for many connections' reads at once (one
// workgroup each, fws_rx_mux). A read with more than kSmallFrames headers
// (tiny frames) is declined:
// res->status = FWS_SMALL_DECLINED and nothing is written but the result; the
// caller then runs fws_gpu_decode_stream. Results are those of
// fws_gpu_decode_stream (fws_decode_result, fws_frame_info, bytes).
#include "decode_common.h"
#include "fws_device.h"
#include "fws_internal.h"

namespace fwsk {

constexpr uint32_t kSThreads = 1024;
constexpr uint32_t kSChunks = kSmallMax / 16;

// The one-frame read (one message per read, the drop-in hook's common case):
// the stream is one complete header whose payload reaches or passes N. Every
// wave reads the first 16 bytes itself (one broadcast load, the same bytes, so
// the same wave-uniform parse) and each thread unmasks its own chunks straight
// from memory: no LDS staging, no serial walk, no workgroup barrier. Results
// are the general path's for such a stream (one frame record, carry-out of the
// unread payload). Returns false, having written nothing, for any other stream.
__device__ __forceinline__ bool decode_one_frame(uint8_t *__restrict__ wire, uint32_t N,
                                                 fws_frame_info *__restrict__ frames, uint32_t cap,
                                                 fws_decode_result *__restrict__ res, uint8_t *out) {
    if (N < 2u || cap == 0u) return false;
    const uintptr_t base = (uintptr_t)wire;
    const u32x4 hv = gload16(base);                  // (16-B aligned: never past the page of byte N - 1)
    // (readfirstlane returns int: through uint32_t, or the low word's sign would fill the high half)
    const uint64_t lo = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(hv.y) << 32 |
                        (uint32_t)__builtin_amdgcn_readfirstlane(hv.x);
    const uint64_t hi = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(hv.w) << 32 |
                        (uint32_t)__builtin_amdgcn_readfirstlane(hv.z);
    Hdr h;
    const int rc = parse_hdr([&](int i) -> uint32_t {
        return (uint32_t)((i < 8 ? lo >> (8 * i) : hi >> (8 * (i - 8))) & 0xFFu);
    }, N, true, h);
    if (rc <= 0) return false;                       // an incomplete header or an error: the general path
    const uint64_t po = (uint64_t)rc, pe = po + h.plen;
    if (pe < N) return false;                        // more headers follow
    // the payload [po, N): full dwords take the key rotated by the payload
    // phase of a 4-aligned address, (-po) & 3; edge dwords keep their other bytes.
    // Chunks start at wave 1: wave 0 (the resident decode's poller, its last poll
    // load still in flight) has none below ~15 KiB, and the frame record and
    // result are stored by the last thread, idle then too -- a wave's loads and
    // stores retire in issue order (vmcnt), so a chunk load issued behind those
    // host-memory stores waited for their PCIe acknowledgements
    const uint32_t rk = rotr32(h.key, 8u * ((0u - (uint32_t)po) & 3u));
    const uint32_t nch = (N + 15u) >> 4;
    uint8_t *const dst = out ? out : wire;
    for (uint32_t c = (threadIdx.x + kSThreads - kWave) % kSThreads; c < nch; c += kSThreads) {
        const uint32_t x0 = 16u * c;
        if (!out && x0 + 16u <= po) continue;        // header bytes only: unchanged in place
        u32x4 v = gload16(base + x0);
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k) v[k] ^= rk & sel_bytes(x0 + 4u * k, po, N);
        if (x0 + 16u <= N) {
            gstore16((uintptr_t)dst + x0, v);
        } else {                                     // the last chunk: whole dwords, then bytes
            uint32_t j = 0;
            for (; x0 + j + 4u <= N; j += 4u) gput(reinterpret_cast<uint32_t *>(dst + x0 + j), v[j >> 2]);
            for (; x0 + j < N; ++j) gput(dst + x0 + j, (uint8_t)(v[j >> 2] >> (8u * (j & 3u))));
        }
    }
    if (threadIdx.x == kSThreads - 1u) {
        fws_frame_info fi;
        fi.hdr_off = 0; fi.payload_len = h.plen; fi.key = h.key; fi.opcode = (uint8_t)h.opcode;
        fi.fin = (uint8_t)h.fin; fi.hdr_len = (uint8_t)rc;
        fi.flags = pe > N ? (uint8_t)FWS_FRAME_TRUNCATED : (uint8_t)0;
        gput(frames, fi);
        fws_decode_result r{};
        r.status = FWS_OK;
        r.consumed = N;
        r.carry_unread = pe - N;                     // 0 when the frame ends at N
        r.n_frames = 1;
        r.n_survivors = 1;
        gput(res, r);
    }
    return true;
}

// The decode of one small read by the calling workgroup (kSThreads threads).
__device__ __forceinline__ void decode_small_wg(uint8_t *__restrict__ wire, uint32_t N,
                                                fws_frame_info *__restrict__ frames, uint32_t cap,
                                                fws_decode_result *__restrict__ res,
                                                uint64_t *tr = nullptr,     // phase clocks (service trace)
                                                uint8_t *out = nullptr) {   // else in place: every chunk to out
    __shared__ u32x4 s_buf[kSChunks + 1];
    __shared__ uint32_t s_po[kSmallFrames + 1];     // payload start of path frame f
    __shared__ uint32_t s_pe[kSmallFrames + 1];     // payload end, clipped to N
    __shared__ uint32_t s_key[kSmallFrames + 1];
    __shared__ uint32_t s_nf;
    const uint32_t tid = threadIdx.x;
    const uint32_t nch = (N + 15u) >> 4;
    const uintptr_t base = (uintptr_t)wire;
    if (decode_one_frame(wire, N, frames, cap, res, out)) {               // (wave-uniform)
        if (tr && tid == 0) tr[0] = tr[1] = wall_clock64();              // (its own chunks done)
        return;
    }

    // 1. stage: all loads of a thread in flight together (the base is 16-B
    //    aligned, so the last chunk's block never crosses a page)
    // (two rounds of four loads per thread in flight)
#pragma unroll
    for (uint32_t k0 = 0; k0 < kSChunks / kSThreads; k0 += 4u) {
        u32x4 v0, v1, v2, v3;
        const uint32_t c = tid + k0 * kSThreads;
        if (c < nch) v0 = gload16(base + 16u * c);
        if (c + kSThreads < nch) v1 = gload16(base + 16u * (c + kSThreads));
        if (c + 2u * kSThreads < nch) v2 = gload16(base + 16u * (c + 2u * kSThreads));
        if (c + 3u * kSThreads < nch) v3 = gload16(base + 16u * (c + 3u * kSThreads));
        if (c < nch) s_buf[c] = v0;
        if (c + kSThreads < nch) s_buf[c + kSThreads] = v1;
        if (c + 2u * kSThreads < nch) s_buf[c + 2u * kSThreads] = v2;
        if (c + 3u * kSThreads < nch) s_buf[c + 3u * kSThreads] = v3;
    }
    if (tid == 0) s_buf[nch] = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();
    if (tr && tid == 0) tr[0] = wall_clock64();
    const uint8_t *sb = (const uint8_t *)s_buf;
    static_assert(sizeof(s_buf) >= kSmallMax + 16u, "the header window of the last offset stays in s_buf");

    // 2. the header chain from offset 0 (wave 0, uniformly: each lane loads one
    //    byte of the 16-byte header window, parse_hdr reads them by readlane --
    //    one LDS round per header instead of a chain of dependent byte loads;
    //    the terminal walk of merge_kernels.hip resolve_path, from the stream start)
    if (tid < kWave) {
        const uint32_t lane = tid;
        fws_decode_result r{};
        r.status = FWS_OK;
        uint64_t pos = 0;
        uint32_t nf = 0;
        bool declined = false;
        while (pos < N) {
            Hdr h;
            const uint32_t q = (uint32_t)pos;
            const uint32_t bl = sb[q + (lane & 15u)];        // (in bounds: s_buf has a chunk past N)
            const int rc = parse_hdr([&](int i) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)bl, i); },
                                     N - q, true, h);
            if (rc < 0) { r.status = rc; r.err_off = q; break; }
            if (rc == 0) break;                               // incomplete trailing header
            if (nf == kSmallFrames) { declined = true; break; }
            const uint64_t po = q + (uint32_t)rc;
            const uint64_t pe = po + h.plen;
            if (lane == 0) {
                s_po[nf] = (uint32_t)po;
                s_pe[nf] = (uint32_t)(pe < N ? pe : N);
                s_key[nf] = h.key;
            }
            if (nf < cap && lane == 0) {
                fws_frame_info fi;
                fi.hdr_off = q; fi.payload_len = h.plen; fi.key = h.key; fi.opcode = (uint8_t)h.opcode;
                fi.fin = (uint8_t)h.fin; fi.hdr_len = (uint8_t)rc;
                fi.flags = pe > N ? (uint8_t)FWS_FRAME_TRUNCATED : (uint8_t)0;
                gput(frames + nf, fi);
            }
            ++nf;
            pos = pe;
        }
        if (declined) {
            r = fws_decode_result{};
            r.status = FWS_SMALL_DECLINED;
            nf = 0;
        } else {
            if (r.status == FWS_OK) {
                if (pos > N) { r.carry_unread = pos - N; r.consumed = N; }
                else if (pos < N) { r.carry_hdr_len = (uint32_t)(N - pos); r.consumed = pos; }
                else r.consumed = N;
            } else {
                r.consumed = r.err_off;
            }
            if (nf > cap && r.status == FWS_OK) r.status = FWS_ERR_CAPACITY;
            r.n_frames = nf;
            r.n_survivors = nf;
        }
        if (lane == 0) {
            s_nf = nf < cap ? nf : cap;                      // the frames listed are the ones unmasked
            gput(res, r);
        }
    }
    __syncthreads();
    if (tr && tid == 0) tr[1] = wall_clock64();

    // 3. unmask: every chunk holding payload bytes, from LDS, one store each
    // (with `out`: every chunk, to out)
    const uint32_t nf = s_nf;
    if (nf == 0 && !out) return;
    for (uint32_t c = tid; c < nch; c += kSThreads) {
        const uint32_t lo = 16u * c, hi = lo + 16u;
        // last frame whose payload starts at or before lo (or frame 0)
        uint32_t a = 0, b = nf ? nf - 1u : 0u;
        while (a < b) {
            const uint32_t m = (a + b + 1u) >> 1;
            if (s_po[m] <= lo) a = m; else b = m - 1u;
        }
        u32x4 v = s_buf[c];
        bool touched = false;
        for (uint32_t f = a; f < nf && s_po[f] < hi; ++f) {   // (none when nf == 0)
            const uint32_t po = s_po[f], pe = s_pe[f];
            if (pe <= lo) continue;
            touched = true;
            const uint32_t key = s_key[f];
#pragma unroll
            for (uint32_t w = 0; w < 4u; ++w) {
                const uint32_t x = lo + 4u * w;               // dword of bytes [x, x + 4)
                uint32_t m = 0;
#pragma unroll
                for (uint32_t j = 0; j < 4u; ++j) {
                    const uint32_t y = x + j;
                    if (y >= po && y < pe) m |= ((key >> (8u * ((y - po) & 3u))) & 0xFFu) << (8u * j);
                }
                v[w] ^= m;
            }
        }
        if (!touched && !out) continue;
        uint8_t *const dst = out ? out : wire;
        if (hi <= N) {
            gstore16((uintptr_t)dst + lo, v);
        } else {
            for (uint32_t j = 0; lo + j < N; ++j) gput(dst + lo + j, (uint8_t)(v[j >> 2] >> (8u * (j & 3u))));
        }
    }
}

__global__ __launch_bounds__(kSThreads) void k_decode_small(uint8_t *__restrict__ wire, uint32_t N,
                                                            fws_frame_info *__restrict__ frames, uint32_t cap,
                                                            fws_decode_result *__restrict__ res) {
    decode_small_wg(wire, N, frames, cap, res);
}

// fws_rx_mux (rx_session.cpp): the reads of many connections in one launch,
// one workgroup per read (segment). A segment is the continuation of the
// connection's frame in progress (unmasked with its carried, rotated key,
// w_socket.h:607-617) followed by its header stream (staged header bytes +
// the rest of the read), decoded as above.
__device__ __forceinline__ void decode_segment(uint8_t *__restrict__ batch, const fws_seg_desc &d,
                                               fws_frame_info *__restrict__ frames,
                                               fws_decode_result *__restrict__ res, uint64_t *tr = nullptr,
                                               uint8_t *out = nullptr) {   // else in place (offsets as batch's)
    const uint32_t tid = threadIdx.x;
    // continuation: 16-B aligned start, so every 4-byte group uses the key as is.
    // Offsets are taken modulo 2^64: a read decoded in place (registered host
    // memory, rx_session.cpp) is addressed relative to the batch base too.
    uint8_t *const cont = reinterpret_cast<uint8_t *>(reinterpret_cast<uintptr_t>(batch) + d.cont_off);
    uint8_t *const ocont = out ? out + d.cont_off : cont;
    for (uint32_t c = tid; 16u * c < d.u; c += kSThreads) {
        const uint32_t lo = 16u * c;
        if (lo + 16u <= d.u) {
            u32x4 v = gload16(reinterpret_cast<uintptr_t>(cont + lo));
            v ^= u32x4{d.key, d.key, d.key, d.key};
            gstore16(reinterpret_cast<uintptr_t>(ocont + lo), v);
        } else {
            for (uint32_t j = lo; j < d.u; ++j) gput(ocont + j, (uint8_t)(gget(cont + j) ^ (uint8_t)(d.key >> (8u * (j & 3u)))));
        }
    }
    if (d.L)
        decode_small_wg(reinterpret_cast<uint8_t *>(reinterpret_cast<uintptr_t>(batch) + d.hs_off), d.L,
                        frames + d.fbase, d.fcap, res, tr, out ? out + d.hs_off : nullptr);
}

// Completion for a host that polls instead of synchronizing the stream (the
// launch + hipStreamSynchronize round trip is ~3.5 us longer than a kernel
// storing a flag the host spins on; tools/rtt_probe.hip): every wave drains its
// stores, the workgroup meets, and one lane releases at system scope and
// stores `seq` to the flag in host memory. With a counter (several
// workgroups), each workgroup releases and counts; the one completing the
// count (target = the launch's workgroups) stores 0 back and then the flag, so
// every launch starts from 0 whatever an earlier launch's host-side status said
// (a monotonic count drifted for good after one misreported launch;
// launches on the mux's one stream never overlap).
__device__ __forceinline__ void host_done(uint32_t *ctr, uint32_t target, uint32_t *flag, uint32_t seq) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x != 0 || !flag) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");                  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (ctr) {
        const uint32_t v = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1u;
        if (v != target) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");
        __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // (a global-space store: a flat one would hold the caller's next barrier
    // until the host acknowledged it)
    __hip_atomic_store((__attribute__((address_space(1))) uint32_t *)(uintptr_t)flag, seq, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kSThreads) void k_decode_segments(uint8_t *__restrict__ batch,
                                                               const fws_seg_desc *__restrict__ segs,
                                                               fws_frame_info *__restrict__ frames,
                                                               fws_decode_result *__restrict__ res, uint32_t *ctr,
                                                               uint32_t target, uint32_t *flag, uint32_t seq) {
    decode_segment(batch, segs[blockIdx.x], frames, res + blockIdx.x);
    host_done(ctr, target, flag, seq);
}

// One read of one connection (fws_rx_session's staged path): the segment
// descriptor travels as a kernel argument, so the launch needs no metadata
// copy; frames and result go straight to the session's pinned landing block.
__global__ __launch_bounds__(kSThreads) void k_decode_one(uint8_t *__restrict__ batch, fws_seg_desc d,
                                                          fws_frame_info *__restrict__ frames,
                                                          fws_decode_result *__restrict__ res, uint32_t *flag,
                                                          uint32_t seq) {
    decode_segment(batch, d, frames, res);
    host_done(nullptr, 0u, flag, seq);
}

// ------------------------------------------------------------ persistent service
// fws_rx_service (fws_internal.h): block 0 is the poller (wave 0: one
// system-scope load of the whole mailbox line per poll) and decodes the
// one-segment requests itself (a session's read: no hop through device memory,
// no completion counter); blocks 1..workers decode the larger ones, segments
// w, w + workers, ... each; they count in dv->ctr and the last one stores the
// request's flag (host_done). Host memory the request names (descriptors, reads in place,
// frame records) is read after a system-scope acquire by each worker, so no L2
// line of an earlier request is reused; the flag follows a system-scope release.
__device__ __forceinline__ uint64_t svc_load64(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// phase clocks of the one-segment requests (fws_internal_rx_service_trace):
// [0] requests, [1..5] summed ticks from the request's detection to the
// acquire, the staged read, the header walk, the unmask, the flag store;
// [6] to every wave's stores drained (before the completion's release)
__device__ unsigned long long g_svc_trace[8];

__global__ __launch_bounds__(kSThreads) void k_rx_service(fws_svc_mail *mail, const fws_svc_mail *poll,
                                                          fws_svc_dev *dv, uint32_t seq0, uint32_t workers,
                                                          uint64_t linger, uint64_t life, uint32_t trace) {
    __shared__ uint32_t s_cmd[3];
    __shared__ fws_svc_req s_req;
    if (blockIdx.x == 0) {
        // the poller's workgroup: wave 0 polls, every lane i < 16 loading word i
        // of the mailbox line; a one-segment request (a session's read) is
        // decoded here by the whole workgroup, a larger one is handed to the
        // workers through dv
        const uint32_t lane = threadIdx.x & (kWave - 1u);
        const bool poller = threadIdx.x < kWave;
        constexpr uint32_t kWords = sizeof(fws_svc_mail) / 8;               // 16
        constexpr uint32_t kReqW = sizeof(fws_svc_req) / 8, kTagW = offsetof(fws_svc_mail, tag) / 8;
        static_assert(offsetof(fws_svc_req, nseg) % 8 == 0 && offsetof(fws_svc_req, kind) % 8 == 0,
                      "nseg / kind: the low half of a word");
        const uint64_t *const src = reinterpret_cast<const uint64_t *>(poll) + (lane < kWords ? lane : 0u);
        uint64_t *const dst = reinterpret_cast<uint64_t *>(&dv->req) + (lane >= 1u && lane <= kReqW ? lane - 1u : 0u);
        uint64_t *const ldst = reinterpret_cast<uint64_t *>(&s_req) + (lane >= 1u && lane <= kReqW ? lane - 1u : 0u);
        uint32_t last = seq0;
        const uint64_t t0 = wall_clock64();
        uint64_t tl = t0, tq[4] = {0, 0, 0, 0}, tf = 0;
        for (;;) {
            if (poller) {
                uint32_t cmd = 1u;                                          // 0: decode s_req here, 1: exit
                // two polls in flight: the next line load is issued before this one is
                // checked (a load older than the last request it saw is ignored: seqs
                // only grow)
                uint64_t wv = svc_load64(src);                              // one load instruction, 16 words
                for (;;) {
                    const uint64_t wn = svc_load64(src);
                    const uint32_t sq = (uint32_t)__builtin_amdgcn_readlane((uint32_t)wv, 0) >> 1 |
                                        (uint32_t)__builtin_amdgcn_readlane((uint32_t)(wv >> 32), 0) << 31;
                    if ((int32_t)(sq - last) > 0) {
                        const uint32_t tag = (uint32_t)__builtin_amdgcn_readlane((uint32_t)wv, kTagW);
                        if (tag != sq) {                                    // the request's half was read first: again
                            wv = wn;
                            continue;
                        }
                        tl = wall_clock64();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");       // system scope, after the state
                        if (trace) tf = wall_clock64();
                        last = sq;
                        const bool quit = (uint32_t)__builtin_amdgcn_readlane(
                                              (uint32_t)wv, 1u + (uint32_t)(offsetof(fws_svc_req, kind) / 8)) == 1u;
                        const uint32_t nseg = (uint32_t)__builtin_amdgcn_readlane(
                            (uint32_t)wv, 1u + (uint32_t)(offsetof(fws_svc_req, nseg) / 8));
                        if (quit) {                                         // stop and tell the workers
                            if (lane == 0) {
                                __hip_atomic_store(&mail->state, (uint64_t)sq << 1, __ATOMIC_RELEASE,
                                                   __HIP_MEMORY_SCOPE_SYSTEM);
                                __hip_atomic_store(&dv->quit, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                            }
                            break;
                        }
                        if (nseg == 1u) {                                   // this workgroup decodes it
                            if (lane >= 1u && lane <= kReqW) *ldst = wv;
                            cmd = 0u;
                            break;
                        }
                        if (lane >= 1u && lane <= kReqW) *dst = wv;         // the request into device memory
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                        if (lane == 0)
                            __hip_atomic_store(&dv->seqn, (uint64_t)nseg << 32 | sq, __ATOMIC_RELEASE,
                                               __HIP_MEMORY_SCOPE_AGENT);
                        wv = wn;
                        continue;
                    }
                    const uint64_t now = wall_clock64();
                    if (now - tl > linger || now - t0 > life) {
                        uint32_t stopped = 0;
                        if (lane == 0) {
                            uint64_t exp = ((uint64_t)last << 1) | 1u;
                            stopped = __hip_atomic_compare_exchange_strong(&mail->state, &exp, (uint64_t)last << 1,
                                                                           __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE,
                                                                           __HIP_MEMORY_SCOPE_SYSTEM) ? 1u : 0u;
                            if (stopped)
                                __hip_atomic_store(&dv->quit, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                        }
                        if (__builtin_amdgcn_readlane(stopped, 0)) break;
                        wv = wn;
                        continue;                                           // a request came in meanwhile
                    }
                    __builtin_amdgcn_s_sleep(1);
                    wv = wn;
                }
                if (lane == 0) s_cmd[0] = cmd;
            }
            __syncthreads();
            if (s_cmd[0]) return;
            const fws_svc_req rq = s_req;
            const fws_seg_desc d = rq.descs ? *reinterpret_cast<const fws_seg_desc *>(rq.descs) : rq.one;
            // a pushed read (kind 2) is decoded in the device staging and written to rq.out
            decode_segment(reinterpret_cast<uint8_t *>(rq.base), d, reinterpret_cast<fws_frame_info *>(rq.frames),
                           reinterpret_cast<fws_decode_result *>(rq.res), trace ? tq : nullptr,
                           rq.kind == 2u ? reinterpret_cast<uint8_t *>(rq.out) : nullptr);
            if (trace && threadIdx.x == 0) tq[2] = wall_clock64();
            if (trace) {                                                   // host_done's steps, clocked
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (threadIdx.x == 0) tq[3] = wall_clock64();              // every wave's stores done
            }
            host_done(nullptr, 0u, reinterpret_cast<uint32_t *>(rq.flag), rq.flag_seq);
            if (trace && threadIdx.x == 0) {                               // (thread 0 detected it: tl, tf)
                const uint64_t te = wall_clock64();
                g_svc_trace[0] += 1u;
                g_svc_trace[1] += tf - tl;
                g_svc_trace[2] += tq[0] - tl;
                g_svc_trace[3] += tq[1] - tl;
                g_svc_trace[4] += tq[2] - tl;
                g_svc_trace[5] += te - tl;
                g_svc_trace[6] += tq[3] - tl;
            }
            __syncthreads();                                               // s_req / s_cmd rewritten next round
        }
    }
    const uint32_t w = blockIdx.x - 1u;
    uint32_t wlast = seq0;
    for (;;) {
        if (threadIdx.x == 0) {
            // relaxed polls (an acquire per poll invalidated this XCD's caches every
            // few hundred ns, for every worker); one fence once a request is seen,
            // system scope only on a worker that has a segment of it
            uint32_t v, q, ns = 0;
            for (;;) {
                const uint64_t sn = __hip_atomic_load(&dv->seqn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                v = (uint32_t)sn;
                if ((int32_t)(v - wlast) > 0) {
                    q = 0;
                    ns = (uint32_t)(sn >> 32);
                    break;
                }
                q = __hip_atomic_load(&dv->quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (q) break;
                __builtin_amdgcn_s_sleep(2);
            }
            if (!q && w < ns) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // request + host bytes fresh
            s_cmd[0] = v;
            s_cmd[1] = q;
            s_cmd[2] = ns;
        }
        __syncthreads();
        const uint32_t v = s_cmd[0];
        if (s_cmd[1]) return;
        if (w >= s_cmd[2]) {                                   // no segment of this request
            wlast = v;
            __syncthreads();                                   // s_cmd rewritten next round
            continue;
        }
        const fws_svc_req rq = dv->req;
        uint8_t *const base = reinterpret_cast<uint8_t *>(rq.base);
        fws_frame_info *const frames = reinterpret_cast<fws_frame_info *>(rq.frames);
        fws_decode_result *const res = reinterpret_cast<fws_decode_result *>(rq.res);
        for (uint32_t i = w; i < rq.nseg; i += workers) {
            const fws_seg_desc d = rq.descs ? reinterpret_cast<const fws_seg_desc *>(rq.descs)[i] : rq.one;
            decode_segment(base, d, frames, res + i);
            __syncthreads();                                   // LDS reused by the next segment
        }
        // only the workers with a segment count (the last of them stores the flag):
        // a round of 8 reads on 64 workers took 16.4 us with every worker counting
        const uint32_t active = rq.nseg < workers ? rq.nseg : workers;
        if (w < active) host_done(&dv->ctr, active, reinterpret_cast<uint32_t *>(rq.flag), rq.flag_seq);
        wlast = v;
        __syncthreads();                                       // s_cmd rewritten next round
    }
}

}  // namespace fwsk

int fws_launch_rx_service(fws_svc_mail *mail, const fws_svc_mail *poll, fws_svc_dev *dv, uint32_t seq0,
                          uint32_t workers, uint64_t linger_ticks, uint64_t life_ticks, uint32_t trace, hipStream_t s) {
    if (!workers) return FWS_ERR_INVALID;
    hipLaunchKernelGGL(fwsk::k_rx_service, dim3(workers + 1u), dim3(fwsk::kSThreads), 0, s, mail, poll, dv, seq0,
                       workers, linger_ticks, life_ticks, trace);
    return fws_hip_status(hipGetLastError());
}

// the service's phase clocks (fws_rx_service's trace hook): copied out, then zeroed
int fws_rx_service_trace_read(unsigned long long *out8) {
    hipError_t e = hipMemcpyFromSymbol(out8, HIP_SYMBOL(fwsk::g_svc_trace), sizeof(unsigned long long) * 8);
    if (e == hipSuccess) {
        const unsigned long long z[8] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(fwsk::g_svc_trace), z, sizeof(z));
    }
    return fws_hip_status(e);
}

int fws_launch_decode_segments(uint8_t *batch, const fws_seg_desc *segs, uint32_t n, fws_frame_info *frames,
                               fws_decode_result *res, hipStream_t s, uint32_t *ctr, uint32_t target, uint32_t *flag,
                               uint32_t seq) {
    if (!n) return 0;
    hipLaunchKernelGGL(fwsk::k_decode_segments, dim3(n), dim3(fwsk::kSThreads), 0, s, batch, segs, frames, res, ctr,
                       target, flag, seq);
    return fws_hip_status(hipGetLastError());
}

int fws_launch_decode_one(uint8_t *batch, const fws_seg_desc &d, fws_frame_info *frames, fws_decode_result *res,
                          hipStream_t s, uint32_t *flag, uint32_t seq) {
    if (d.L > kSmallMax || !res || (d.fcap && !frames)) return FWS_ERR_INVALID;
    hipLaunchKernelGGL(fwsk::k_decode_one, dim3(1), dim3(fwsk::kSThreads), 0, s, batch, d, frames, res, flag, seq);
    return fws_hip_status(hipGetLastError());
}

int fws_launch_decode_small(uint8_t *wire, uint64_t N, fws_frame_info *frames, uint32_t cap,
                            fws_decode_result *res, hipStream_t s) {
    if (N > kSmallMax || ((uintptr_t)wire & 15u) || (N && !wire) || !res || (cap && !frames))
        return FWS_ERR_INVALID;
    hipLaunchKernelGGL(fwsk::k_decode_small, dim3(1), dim3(fwsk::kSThreads), 0, s, wire, (uint32_t)N, frames, cap,
                       res);
    return fws_hip_status(hipGetLastError());
}
