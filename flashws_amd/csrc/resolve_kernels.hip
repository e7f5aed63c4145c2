// resolve_kernels.hip -- second half of fws_gpu_decode_stream: from the scan's
// per-tile survivors (k_scan, decode_kernels.hip) to the frame list, the
// payload descriptors and the unmask plan, in ONE cooperative launch.
//
// The phases are the serial frame loop of WSocket::OnRecvData
// (net/w_socket.h:543-769) restated as parallel passes over survivors; each
// pass needs the previous one's results device-wide, so the launch is a
// persistent grid (one workgroup per CU) separated by a grid barrier. That
// replaces ~30 dependent kernel launches -- each costing the ~5 us launch /
// end-of-kernel floor -- with one launch and cheap barriers.
//
//   1  tile prefix    tile_base = exclusive prefix of tile_count; S = total
//   2  compact        survivors from tile slots / spill into dense, offset-
//                     sorted arrays; leaf ranks -> indices
//   3  link           J0: a non-leaf -> its leaf; a leaf -> the survivor at
//                     its exit offset (END / DEAD / INCOMPLETE terminals)
//   4  jump           J_k = J_{k-1} o J_{k-1}, k < K (pointer doubling)
//   5  entry          per tile, binary lifting from the root: the tile's first
//                     true header; the path's last node and terminal
//   6  walk           per tile: follow the true chain, flag + count frames
//   7  frame prefix   fbase = exclusive prefix of the per-tile frame counts
//   8  emit           fws_frame_info + fws_frame_desc in stream order
//   9  finish         terminal -> fws_decode_result; a protocol error is
//                     located by re-walking from the last good header with
//                     ParseFrameHdr's rules (w_socket.h:435-524)
//  10  plan           stream-space unit map of the emitted frames for
//                     k_unmask_stream (unmask_kernels.hip)
#include "decode_common.h"

namespace fwsk {

constexpr int kRThreads = 1024;                   // k_resolve workgroup
constexpr uint64_t kBarrierTimeoutTicks = 5000000;  // 50 ms of the 100 MHz wall clock

struct ResolveParams {
    const uint8_t *wire;
    uint64_t N;
    uint32_t n_tiles;
    uint32_t K;                                   // doubling levels
    const fws_frame_info *stage_info;
    const uint32_t *stage_leaf;
    const fws_frame_info *spill_info;
    const uint32_t *spill_leaf;
    const uint32_t *tile_spill;
    const uint32_t *tile_count;
    uint32_t *tile_base;
    uint32_t *tile_entry;
    uint32_t *tile_frames;
    uint32_t *fbase;
    fws_frame_info *surv_info;
    uint32_t *surv_leaf;
    uint32_t *jump;                               // [K][s_cap]
    uint8_t *on_path;
    uint32_t *counters;
    uint64_t *bsums;                              // one per workgroup
    uint64_t s_cap;
    fws_frame_info *frames;
    uint32_t cap;
    fws_frame_desc *descs;
    uint32_t desc_cap;
    fws_decode_result *res;
    uint64_t *cbase;                              // unmask plan (fws_plan_ws)
    uint32_t *unit_first;
    uint64_t *plan_total;
    uint64_t unit_cap;
    uint32_t gate;                                // 1: run only if the super-tile resolve fell back
    uint32_t *zero_next;                          // the next call's counter set (zeroed here)
    uint8_t *utf8_ok;                             // optional: preset per frame (TEXT, FIN, complete)
};

__device__ __forceinline__ void put_frame(const ResolveParams &P, uint32_t f, const fws_frame_info &fi) {
    P.frames[f] = fi;
    if (P.utf8_ok)
        P.utf8_ok[f] = fi.opcode == 1u && fi.fin && !(fi.flags & FWS_FRAME_TRUNCATED) &&
                       fi.hdr_off + fi.hdr_len + fi.payload_len <= P.N;
}

// Grid barrier of a cooperative launch. Arrivals only grow within a launch
// (reset by the counters memset before k_scan), so generation g is complete
// when gridDim.x * g workgroups have arrived. A barrier that does not complete
// within kBarrierTimeoutTicks (workgroups not co-resident) sets overflow bit 1
// and lets every later barrier fall through, so the launch always ends.
struct GridBarrier {
    uint32_t *arrive;
    uint32_t *gen;
    uint32_t *fault;
    uint32_t g = 0;

    // Thread 0 of each workgroup: release fence (write back this XCD's L2 so
    // other XCDs see the phase's writes), arrive, poll the generation with
    // relaxed device-scope loads (an acquire load per poll would invalidate
    // L2 every iteration), then one acquire fence.
    __device__ void sync() {
        __syncthreads();
        ++g;
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            const uint32_t prev = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (prev + 1u == gridDim.x * g) {
                __hip_atomic_store(gen, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                const uint64_t t0 = wall_clock64();
                while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < g) {
                    if (__hip_atomic_load(fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 2u) break;
                    if (wall_clock64() - t0 > kBarrierTimeoutTicks) {
                        __hip_atomic_fetch_or(fault, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        __syncthreads();
    }
};

template <typename T>
__device__ __forceinline__ T block_sum(T v, T *sred) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) sred[w] = v;
    __syncthreads();
    T t = 0;
#pragma unroll
    for (int i = 0; i < kRThreads / 64; ++i) t += sred[i];
    __syncthreads();
    return t;
}

template <typename T>
__device__ __forceinline__ T block_excl(T v, T *sred, T *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    T inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) sred[w] = inc;
    __syncthreads();
    T off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kRThreads / 64; ++i) {
        off += (i < w) ? sred[i] : T(0);
        tot += sred[i];
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

// Device-wide exclusive prefix of val(i), i < n, in two passes around one
// grid barrier: workgroup b owns the contiguous range [lo, hi). out(i, prefix)
// receives each element's prefix; returns the grand total (every thread).
template <typename T, typename Val, typename Out>
__device__ __forceinline__ T grid_excl_scan(uint64_t n, Val val, Out out, uint64_t *bsums, T *sred,
                                            GridBarrier &bar) {
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    const uint64_t per = (n + nb - 1) / nb;
    const uint64_t lo = (uint64_t)b * per < n ? (uint64_t)b * per : n;
    const uint64_t hi = lo + per < n ? lo + per : n;
    T s = 0;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += kRThreads) s += val(i);
    s = block_sum<T>(s, sred);
    if (threadIdx.x == 0) bsums[b] = (uint64_t)s;
    bar.sync();
    T pre = 0, total = 0;
    for (uint32_t i = threadIdx.x; i < nb; i += kRThreads) {
        const T x = (T)bsums[i];
        if (i < b) pre += x;
        total += x;
    }
    pre = block_sum<T>(pre, sred);
    total = block_sum<T>(total, sred);
    T run = pre;
    for (uint64_t base = lo; base < hi; base += kRThreads) {
        const uint64_t i = base + threadIdx.x;
        const T v = i < hi ? val(i) : T(0);
        T tot;
        const T e = block_excl<T>(v, sred, &tot);
        if (i < hi) out(i, run + e, v);
        run += tot;
    }
    return total;
}

__global__ __launch_bounds__(kRThreads) void k_resolve(ResolveParams P) {
    __shared__ uint32_t sred32[kRThreads / 64];
    GridBarrier bar{P.counters + kCntBarArrive, P.counters + kCntBarGen, P.counters + kCntOverflow};
    uint32_t *const C = P.counters;
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint64_t gid = (uint64_t)blockIdx.x * kRThreads + tid, G = (uint64_t)gridDim.x * kRThreads;
    const uint64_t gwave = gid >> 6, nwaves = G >> 6;
    const uint32_t n_tiles = P.n_tiles;
    if (blockIdx.x == 0 && threadIdx.x < kCntStride) P.zero_next[threadIdx.x] = 0u;
    if (P.gate && C[kCntFallback] == 0) return;   // merge_kernels.hip resolved this stream

    // 1  tile prefix (+ per-tile / global defaults)
    if (gid == 0) C[kCntRoot] = kNone;
    for (uint64_t t = gid; t < n_tiles; t += G) P.tile_entry[t] = kNone;
    const uint32_t S = grid_excl_scan<uint32_t>(
        n_tiles, [&](uint64_t t) { return P.tile_count[t]; },
        [&](uint64_t t, uint32_t pre, uint32_t) { P.tile_base[t] = pre; }, P.bsums, sred32, bar);
    if (gid == 0) {
        C[kCntSurv] = S;
        if (S > P.s_cap) atomicOr(&C[kCntOverflow], 1u);
    }
    bar.sync();
    const bool ok = !(__hip_atomic_load(&C[kCntOverflow], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1u) &&
                    S <= P.s_cap;           // same value in every workgroup

    if (ok && n_tiles) {
        // 2  compact: one wave per tile
        for (uint64_t t = gwave; t < n_tiles; t += nwaves) {
            const uint32_t n = P.tile_count[t], b = P.tile_base[t], sp = P.tile_spill[t];
            const fws_frame_info *si = sp == kNone ? P.stage_info + t * kSlots : P.spill_info + sp;
            const uint32_t *sl = sp == kNone ? P.stage_leaf + t * kSlots : P.spill_leaf + sp;
            for (uint32_t r = lane; r < n; r += 64) {
                P.surv_info[b + r] = si[r];
                P.surv_leaf[b + r] = b + sl[r];
                P.on_path[b + r] = 0;
            }
        }
        bar.sync();

        // 3  link
        for (uint64_t i = gid; i < S; i += G) {
            const fws_frame_info fi = P.surv_info[i];
            const uint32_t lf = P.surv_leaf[i];
            uint32_t j;
            if (lf != i) {
                j = lf;                                      // in-tile: the chain's leaf
            } else if (fi.hdr_len == 0) {
                j = kTermIncomplete;
            } else {
                const uint64_t x = exit_of(fi);
                j = kTermEnd;
                if (x < P.N) {                               // survivor at offset x, or DEAD
                    const uint32_t tt = (uint32_t)(x / kTile);
                    uint32_t lo = P.tile_base[tt], n = P.tile_count[tt];
                    j = kTermDead;
                    while (n > 0) {
                        const uint32_t half = n >> 1;
                        const uint64_t o = P.surv_info[lo + half].hdr_off;
                        if (o == x) { j = lo + half; break; }
                        if (o < x) { lo += half + 1; n -= half + 1; } else { n = half; }
                    }
                }
            }
            P.jump[i] = j;
            if (fi.hdr_off == 0) C[kCntRoot] = (uint32_t)i;
        }
        bar.sync();

        // 4  pointer doubling
        for (uint32_t k = 1; k < P.K; ++k) {
            const uint32_t *Jp = P.jump + (uint64_t)(k - 1) * P.s_cap;
            uint32_t *Jn = P.jump + (uint64_t)k * P.s_cap;
            for (uint64_t i = gid; i < S; i += G) {
                const uint32_t a = Jp[i];
                Jn[i] = is_term(a) ? a : Jp[a];
            }
            bar.sync();
        }

        // 5  entry: the last path node before the tile (headers strictly
        //    increase along the path), then its successor if inside the tile
        const uint32_t root = C[kCntRoot];
        for (uint64_t t = gid; t <= n_tiles; t += G) {
            if (root == kNone) {
                if (t == n_tiles) { C[kCntTerm] = kTermDead; C[kCntLast] = kNone; }
                continue;
            }
            uint32_t cur = root;
            if (t == n_tiles) {
                for (int k = (int)P.K - 1; k >= 0; --k) {
                    const uint32_t y = P.jump[(uint64_t)k * P.s_cap + cur];
                    if (!is_term(y)) cur = y;
                }
                C[kCntLast] = cur;
                C[kCntTerm] = P.jump[cur];
                continue;
            }
            if (t == 0) { P.tile_entry[0] = root; continue; }
            const uint64_t T0 = t * kTile;
            for (int k = (int)P.K - 1; k >= 0; --k) {
                const uint32_t y = P.jump[(uint64_t)k * P.s_cap + cur];
                if (!is_term(y) && P.surv_info[y].hdr_off < T0) cur = y;
            }
            const uint32_t y = P.jump[cur];
            if (!is_term(y) && P.surv_info[y].hdr_off < T0 + kTile) P.tile_entry[t] = y;
        }
        bar.sync();

        // 6  walk the true chain of each tile through its sorted survivors
        for (uint64_t t = gid; t < n_tiles; t += G) {
            uint32_t e = P.tile_entry[t], cnt = 0;
            if (e != kNone) {
                const uint32_t end = P.tile_base[t] + P.tile_count[t];
                for (uint32_t i = e;;) {
                    const fws_frame_info fi = P.surv_info[i];
                    if (fi.hdr_len) { P.on_path[i] = 1; ++cnt; }
                    if (P.surv_leaf[i] == i) break;
                    const uint64_t x = exit_of(fi);
                    uint32_t j = i + 1;
                    while (j < end && P.surv_info[j].hdr_off < x) ++j;
                    if (j >= end || P.surv_info[j].hdr_off != x) break;   // not for a live chain
                    i = j;
                }
            }
            P.tile_frames[t] = cnt;
        }
        bar.sync();

        // 7  frame prefix
        const uint32_t nf = grid_excl_scan<uint32_t>(
            n_tiles, [&](uint64_t t) { return P.tile_frames[t]; },
            [&](uint64_t t, uint32_t pre, uint32_t) { P.fbase[t] = pre; }, P.bsums, sred32, bar);
        if (gid == 0) C[kCntFrames] = nf;
        bar.sync();

        // 8  emit, one wave per tile
        for (uint64_t t = gwave; t < n_tiles; t += nwaves) {
            const uint32_t b = P.tile_base[t], n = P.tile_count[t];
            uint32_t out = P.fbase[t];
            for (uint32_t i0 = 0; i0 < n; i0 += 64) {
                const uint32_t i = b + i0 + lane;
                const bool f = (i0 + lane < n) && P.on_path[i];
                const uint64_t m = __ballot(f);
                if (f) {
                    const uint32_t o = out + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                    const fws_frame_info fi = P.surv_info[i];
                    if (o < P.cap) put_frame(P, o, fi);
                    if (o < P.desc_cap) {
                        const uint64_t po = fi.hdr_off + fi.hdr_len;
                        const uint64_t pl = (po + fi.payload_len > P.N) ? (P.N - po) : fi.payload_len;
                        P.descs[o] = fws_frame_desc{po, pl, fi.key, 0u};
                    }
                }
                out += (uint32_t)__popcll(m);
            }
        }
    } else if (gid == 0) {
        C[kCntFrames] = 0;
        C[kCntTerm] = kTermDead;
        C[kCntLast] = kNone;
    }
    bar.sync();

    // 9  finish (one thread)
    if (gid == 0) {
        fws_decode_result r{};
        r.status = FWS_OK;
        uint32_t nf = C[kCntFrames];
        r.n_survivors = S;
        const uint32_t fault = __hip_atomic_load(&C[kCntOverflow], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!ok || (fault & 2u)) {
            r.status = (fault & 2u) ? FWS_ERR_INTERNAL : FWS_ERR_CAPACITY;
            r.n_frames = 0;
            C[kCntFrames] = 0;
            *P.res = r;
        } else {
            const uint32_t term = C[kCntTerm], last = C[kCntLast];
            const uint64_t N = P.N;
            uint64_t pos;                     // offset of the next header after the decoded chain
            if (N == 0 || last == kNone) {
                pos = 0;                      // no survivor at offset 0: walk from the start
            } else {
                const fws_frame_info fi = P.surv_info[last];
                pos = fi.hdr_len ? exit_of(fi) : fi.hdr_off;
            }
            if (N > 0 && (last == kNone || term == kTermDead)) {
                // headers from `pos` up to the failing one (ParseFrameHdr on global bytes)
                for (;;) {
                    if (pos >= N) break;
                    Hdr h;
                    const uint64_t q = pos;
                    const int rc = parse_hdr([&](int i) -> uint32_t { return P.wire[q + i]; }, N - q, true, h);
                    if (rc < 0) { r.status = rc; r.err_off = q; break; }
                    if (rc == 0) break;                       // incomplete trailing header
                    fws_frame_info fi;
                    fi.hdr_off = q; fi.payload_len = h.plen; fi.key = h.key; fi.opcode = (uint8_t)h.opcode;
                    fi.fin = (uint8_t)h.fin; fi.hdr_len = (uint8_t)rc;
                    fi.flags = (q + rc + h.plen > N) ? (uint8_t)FWS_FRAME_TRUNCATED : (uint8_t)0;
                    if (nf < P.cap) put_frame(P, nf, fi);
                    if (nf < P.desc_cap) {
                        const uint64_t po = q + rc;
                        P.descs[nf] = fws_frame_desc{po, (po + h.plen > N) ? N - po : h.plen, h.key, 0u};
                    }
                    ++nf;
                    pos = q + rc + h.plen;
                }
            }
            if (r.status == FWS_OK) {
                if (pos > N) { r.carry_unread = pos - N; r.consumed = N; }
                else if (pos < N) { r.carry_hdr_len = (uint32_t)(N - pos); r.consumed = pos; }
                else r.consumed = N;
            } else {
                r.consumed = r.err_off;
            }
            if (nf > P.cap && r.status == FWS_OK) r.status = FWS_ERR_CAPACITY;
            r.n_frames = nf;
            C[kCntFrames] = nf < P.desc_cap ? nf : P.desc_cap;
            *P.res = r;
        }
    }
    bar.sync();

    // 10  unmask plan in stream space (k_unmask_stream): frame f spans stream
    //     bytes [hdr_off_f, hdr_off_{f+1}); the last frame spans to the end
    const uint32_t n = C[kCntFrames];
    const uint64_t n_units = (P.N + 4095) / 4096 < P.unit_cap ? (P.N + 4095) / 4096 : P.unit_cap;
    for (uint64_t f = gid; f < n; f += G) {
        const uint64_t h = P.frames[f].hdr_off;
        const uint64_t e = f + 1 < n ? P.frames[f + 1].hdr_off : n_units * 4096;
        const uint64_t ue = (e + 4095) / 4096 < n_units ? (e + 4095) / 4096 : n_units;
        for (uint64_t u = (h + 4095) / 4096; u < ue; ++u) P.unit_first[u] = (uint32_t)f;
    }
}

}  // namespace fwsk

// ------------------------------------------------------------------ host side
using namespace fwsk;

int fws_launch_resolve(fws_gpu_ctx *ctx, const uint8_t *wire, uint64_t N, uint32_t n_tiles, uint32_t K,
                       fws_frame_info *frames, uint32_t cap, fws_decode_result *res, int gate, uint32_t *zero_next,
                       uint8_t *utf8_ok, hipStream_t s) {
    fws_decode_ws &d = ctx->dec;
    ResolveParams P;
    P.utf8_ok = utf8_ok;
    P.gate = gate ? 1u : 0u;
    P.zero_next = zero_next;
    P.wire = wire;
    P.N = N;
    P.n_tiles = n_tiles;
    P.K = K;
    P.stage_info = d.stage_info;
    P.stage_leaf = d.stage_leaf;
    P.spill_info = d.spill_info;
    P.spill_leaf = d.spill_leaf;
    P.tile_spill = d.tile_spill;
    P.tile_count = d.tile_count;
    P.tile_base = d.tile_base;
    P.tile_entry = d.tile_entry;
    P.tile_frames = d.tile_frames;
    P.fbase = d.fbase;
    P.surv_info = d.surv_info;
    P.surv_leaf = d.surv_leaf;
    P.jump = d.jump;
    P.on_path = d.on_path;
    P.counters = d.counters;
    P.bsums = d.rbsums;
    P.s_cap = d.max_surv;
    P.frames = frames;
    P.cap = cap;
    P.descs = d.descs;
    P.desc_cap = cap;                         // descriptors (and the unmask) cover at most cap frames
    P.res = res;
    P.cbase = ctx->plan.cbase;
    P.unit_first = ctx->plan.unit_first;
    P.plan_total = ctx->plan.total;
    P.unit_cap = ctx->plan.unit_cap;
    // A plain launch: one workgroup per CU is co-resident on an otherwise idle
    // device, and GridBarrier times out (FWS_ERR_INTERNAL in the result, never
    // a hang) if workgroups of other streams' kernels keep some of them out.
    // hipLaunchCooperativeKernel would guarantee residency but goes through the
    // runtime's cooperative queue: ~12 us of cross-queue waits before and after
    // the launch, paid by every decode although the common path returns at once.
    hipLaunchKernelGGL(k_resolve, dim3(d.resolve_grid), dim3(kRThreads), 0, s, P);
    return fws_hip_status(hipGetLastError());
}
