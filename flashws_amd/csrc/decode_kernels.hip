// decode_kernels.hip -- fused header parse + unmask of a raw server-side wire
// stream on gfx950 (fws_gpu_decode_stream). Replaces the serial frame loop of
// WSocket::OnRecvData (net/w_socket.h:543-769) for a device-resident buffer.
//
// Frame boundaries are a serial dependency (header i+1's offset comes from
// header i's length), so the stream is parsed speculatively and in parallel:
//
//  k_scan   one workgroup per 16 KiB tile staged in LDS. Every byte offset is
//           parsed as a header (ParseFrameHdr semantics, w_socket.h:435-524);
//           valid headers point at the next header offset. Pointer jumping in
//           LDS resolves every chain to the last header before the tile end
//           (its "leaf") or to DEAD (an invalid header). Offsets whose chain
//           survives are "survivors": every true header is one, most random
//           payload offsets are not (~2% pass one parse, few survive a chain).
//  k_link   survivor graph: a non-leaf points at its leaf; a leaf points at
//           the survivor at its exit offset in a later tile (binary search),
//           or at a terminal (END, DEAD = invalid header, INCOMPLETE header).
//  k_jump   pointer doubling tables J_k = J_{k-1} o J_{k-1} (K-1 launches,
//           K = ceil(log2(path bound)); the path visits <= 2 nodes per tile).
//  k_mark   one workgroup expands the root's path top-down through J_k and
//           records each tile's entry header.
//  k_walk / k_tile_scan / k_emit
//           per tile: follow the true chain from its entry through the tile's
//           survivors, then write frames (fws_frame_info) and payload regions
//           (fws_frame_desc) in stream order.
//  k_finish terminal handling (error walk for protocol errors, carry-out).
// The payload regions then go through the descriptor-mode plan + k_unmask
// (unmask_kernels.hip). HBM traffic: one read of the stream here, one read +
// write of the payloads in k_unmask; everything else touches metadata only.
#include "fws_device.h"
#include "fws_internal.h"

namespace fwsk {

constexpr uint32_t kTile = 16384;            // bytes per scan tile
constexpr uint32_t kHalo = 16;               // header bytes past the tile end
constexpr uint16_t kDead = 0xFFFF;
constexpr uint16_t kLeaf = 0x8000;           // kLeaf | offset: chain ends at this header
constexpr uint32_t kPerThread = kTile / kBlock;

constexpr uint32_t kNone = 0xFFFFFFFFu;           // "no node" (memset 0xFF)
constexpr uint32_t kTermEnd = 0xFFFFFFFEu;        // chain reaches / passes the stream end
constexpr uint32_t kTermDead = 0xFFFFFFFDu;       // next header offset is not a survivor
constexpr uint32_t kTermIncomplete = 0xFFFFFFFCu; // incomplete header at the stream end
__device__ __forceinline__ bool is_term(uint32_t v) { return v >= kTermIncomplete; }

enum Counter {
    kCntSurv = 0,        // survivors allocated
    kCntOverflow = 1,    // survivor / frame capacity exceeded
    kCntPath = 2,        // path nodes
    kCntFrames = 3,      // frames emitted (device frame count, read by plan/unmask)
    kCntRoot = 4,        // survivor index of the header at offset 0 (kNone if absent)
    kCntTerm = 5,        // terminal code of the path
    kCntLast = 6,        // last path node
    kCntCount = 8
};

__device__ __forceinline__ int parse_lds(const uint8_t *sbuf, uint32_t p, uint64_t avail, Hdr &h) {
    return parse_hdr([&](int i) -> uint32_t { return sbuf[p + i]; }, avail, true, h);
}

// ------------------------------------------------------------------ k_scan
__global__ __launch_bounds__(kBlock) void k_scan(const uint8_t *__restrict__ wire, uint64_t N,
                                                 fws_frame_info *__restrict__ surv_info,
                                                 uint32_t *__restrict__ surv_leaf,
                                                 uint32_t *__restrict__ tile_base,
                                                 uint32_t *__restrict__ tile_count,
                                                 uint32_t *__restrict__ counters, uint32_t s_cap) {
    __shared__ __attribute__((aligned(16))) uint8_t sbuf[kTile + kHalo];
    __shared__ uint16_t sptr[kTile];
    __shared__ uint64_t sbits[kTile / 64];
    __shared__ uint32_t spre[kTile / 64];
    __shared__ uint32_t sbase, stotal;

    const uint32_t t = blockIdx.x;
    const uint64_t t0 = uint64_t(t) * kTile;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;

    // stage the tile + halo (wire is 16-B aligned, tiles are 16-B multiples)
    for (uint32_t i = tid * 16u; i < kTile + kHalo; i += kBlock * 16u) {
        const uint64_t q = t0 + i;
        if (q + 16u <= N) {
            *reinterpret_cast<u32x4 *>(sbuf + i) = *reinterpret_cast<const u32x4 *>(wire + q);
        } else {
#pragma unroll
            for (int b = 0; b < 16; ++b) sbuf[i + b] = (q + b < N) ? wire[q + b] : 0;
        }
    }
    __syncthreads();

    // parse every offset: next-header pointer, leaf, or dead
    for (uint32_t k = 0; k < kPerThread; ++k) {
        const uint32_t p = uint32_t(tid) + k * kBlock;
        const uint64_t q = t0 + p;
        uint16_t v = kDead;
        if (q < N) {
            Hdr h;
            const int r = parse_lds(sbuf, p, N - q, h);
            if (r == 0) {
                v = kLeaf | p;                       // incomplete header at the stream end
            } else if (r > 0) {
                const uint64_t nx = q + (uint64_t)r + h.plen;
                v = (nx < t0 + kTile) ? (uint16_t)(nx - t0) : (uint16_t)(kLeaf | p);
            }
        }
        sptr[p] = v;
    }
    __syncthreads();

    // pointer jumping: every live offset ends at its leaf or dies
    for (;;) {
        int changed = 0;
        for (uint32_t k = 0; k < kPerThread; ++k) {
            const uint32_t p = uint32_t(tid) + k * kBlock;
            const uint16_t v = sptr[p];
            if (v < kTile) {
                sptr[p] = sptr[v];
                changed = 1;
            }
        }
        if (!__syncthreads_or(changed)) break;
    }

    // survivor bitmap (wave ballots over 64 consecutive offsets) and ranks
    for (uint32_t k = 0; k < kPerThread; ++k) {
        const uint32_t p = uint32_t(w) * 64u + uint32_t(lane) + k * kBlock;
        const uint64_t m = __ballot(sptr[p] != kDead);
        if (lane == 0) sbits[p >> 6] = m;
    }
    __syncthreads();
    {
        const uint32_t c = __popcll(sbits[tid]);
        uint32_t inc = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t x = __shfl_up(inc, o, 64);
            if (lane >= o) inc += x;
        }
        __shared__ uint32_t swsum[kBlock / 64];
        if (lane == 63) swsum[w] = inc;
        __syncthreads();
        uint32_t off = 0, tot = 0;
        for (int i = 0; i < kBlock / 64; ++i) {
            off += (i < w) ? swsum[i] : 0u;
            tot += swsum[i];
        }
        spre[tid] = off + inc - c;
        if (tid == 0) {
            uint32_t base = tot ? atomicAdd(&counters[kCntSurv], tot) : 0u;
            if (tot && base + tot > s_cap) {
                atomicOr(&counters[kCntOverflow], 1u);
                tot = 0;
            }
            sbase = base;
            stotal = tot;
            tile_base[t] = base;
            tile_count[t] = tot;
        }
    }
    __syncthreads();
    if (stotal == 0) return;
    const uint32_t base = sbase;

    auto rank_of = [&](uint32_t p) -> uint32_t {
        const uint64_t m = sbits[p >> 6] & ((1ull << (p & 63u)) - 1ull);
        return spre[p >> 6] + (uint32_t)__popcll(m);
    };
    for (uint32_t k = 0; k < kPerThread; ++k) {
        const uint32_t p = uint32_t(tid) + k * kBlock;
        const uint16_t v = sptr[p];
        if (v == kDead) continue;
        const uint64_t q = t0 + p;
        const uint32_t idx = base + rank_of(p);
        Hdr h;
        const int r = parse_lds(sbuf, p, N - q, h);
        fws_frame_info fi;
        fi.hdr_off = q;
        if (r > 0) {
            fi.payload_len = h.plen;
            fi.key = h.key;
            fi.opcode = (uint8_t)h.opcode;
            fi.fin = (uint8_t)h.fin;
            fi.hdr_len = (uint8_t)r;
            fi.flags = (q + (uint64_t)r + h.plen > N) ? (uint8_t)FWS_FRAME_TRUNCATED : (uint8_t)0;
        } else {                                     // incomplete trailing header
            fi.payload_len = 0;
            fi.key = 0;
            fi.opcode = 0;
            fi.fin = 0;
            fi.hdr_len = 0;
            fi.flags = 0;
        }
        surv_info[idx] = fi;
        surv_leaf[idx] = base + rank_of(v & 0x7FFFu);
    }
}

// ------------------------------------------------------------------ k_link
__device__ __forceinline__ uint64_t exit_of(const fws_frame_info &fi) {
    return fi.hdr_off + fi.hdr_len + fi.payload_len;
}

// Survivor index of the header at offset x (tile lists are sorted), or kNone.
__device__ __forceinline__ uint32_t find_survivor(const fws_frame_info *__restrict__ info,
                                                  const uint32_t *__restrict__ tile_base,
                                                  const uint32_t *__restrict__ tile_count, uint64_t x) {
    const uint32_t t = (uint32_t)(x / kTile);
    uint32_t lo = tile_base[t], n = tile_count[t];
    while (n > 0) {
        const uint32_t half = n >> 1;
        const uint64_t o = info[lo + half].hdr_off;
        if (o == x) return lo + half;
        if (o < x) { lo += half + 1; n -= half + 1; } else { n = half; }
    }
    return kNone;
}

__global__ __launch_bounds__(kBlock) void k_link(const fws_frame_info *__restrict__ info,
                                                 const uint32_t *__restrict__ leaf,
                                                 const uint32_t *__restrict__ tile_base,
                                                 const uint32_t *__restrict__ tile_count,
                                                 const uint32_t *__restrict__ counters, uint64_t N,
                                                 uint32_t *__restrict__ J0, uint32_t *__restrict__ root) {
    const uint32_t S = counters[kCntOverflow] ? 0u : counters[kCntSurv];
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < S; i += gridDim.x * kBlock) {
        const fws_frame_info fi = info[i];
        uint32_t j;
        if (leaf[i] != i) {
            j = leaf[i];                                   // in-tile: jump to the chain's leaf
        } else if (fi.hdr_len == 0) {
            j = kTermIncomplete;
        } else {
            const uint64_t x = exit_of(fi);
            j = (x >= N) ? kTermEnd : find_survivor(info, tile_base, tile_count, x);
            if (j == kNone) j = kTermDead;
        }
        J0[i] = j;
        if (fi.hdr_off == 0) *root = i;
    }
}

__global__ __launch_bounds__(kBlock) void k_jump(const uint32_t *__restrict__ Jp, uint32_t *__restrict__ Jn,
                                                 const uint32_t *__restrict__ counters) {
    const uint32_t S = counters[kCntOverflow] ? 0u : counters[kCntSurv];
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < S; i += gridDim.x * kBlock) {
        const uint32_t a = Jp[i];
        Jn[i] = is_term(a) ? a : Jp[a];
    }
}

// ------------------------------------------------------------------ k_mark
// One workgroup: path = {J^j(root)} expanded top-down; tile_entry[t] = the
// first header of tile t on the true chain.
constexpr int kMarkBlock = 1024;

__global__ __launch_bounds__(kMarkBlock) void k_mark(const uint32_t *__restrict__ J, uint64_t s_cap, int K,
                                                     const fws_frame_info *__restrict__ info,
                                                     const uint32_t *__restrict__ leaf,
                                                     uint32_t *__restrict__ path,
                                                     uint32_t *__restrict__ tile_entry,
                                                     uint32_t *__restrict__ counters,
                                                     const uint32_t *__restrict__ root_p) {
    __shared__ uint32_t sn;
    const uint32_t root = *root_p;
    const bool ok = !counters[kCntOverflow] && root != kNone;
    if (threadIdx.x == 0) {
        sn = 0;
        if (ok) { path[0] = root; sn = 1; }
    }
    __syncthreads();
    if (!ok) {
        if (threadIdx.x == 0) { counters[kCntPath] = 0; counters[kCntTerm] = kTermDead; counters[kCntLast] = kNone; }
        return;
    }
    for (int k = K - 1; k >= 0; --k) {
        const uint32_t m = sn;
        __syncthreads();
        const uint32_t *Jk = J + (uint64_t)k * s_cap;
        for (uint32_t i = threadIdx.x; i < m; i += kMarkBlock) {
            const uint32_t y = Jk[path[i]];
            if (!is_term(y)) path[atomicAdd(&sn, 1u)] = y;
        }
        __threadfence_block();
        __syncthreads();
    }
    const uint32_t n = sn;
    for (uint32_t i = threadIdx.x; i < n; i += kMarkBlock) {
        const uint32_t s = path[i];
        const uint32_t y = J[s];                        // J_0
        if (i == 0) tile_entry[info[s].hdr_off / kTile] = s;        // root
        if (leaf[s] == s && !is_term(y)) tile_entry[info[y].hdr_off / kTile] = y;
        if (is_term(y)) { counters[kCntTerm] = y; counters[kCntLast] = s; }
    }
    if (threadIdx.x == 0) counters[kCntPath] = n;
}

// ------------------------------------------------------------------ k_walk
// One thread per tile: follow the true chain from the tile's entry through the
// tile's sorted survivor list; flag the frames and count them.
__global__ __launch_bounds__(kBlock) void k_walk(const fws_frame_info *__restrict__ info,
                                                 const uint32_t *__restrict__ leaf,
                                                 const uint32_t *__restrict__ tile_base,
                                                 const uint32_t *__restrict__ tile_count,
                                                 const uint32_t *__restrict__ tile_entry, uint32_t n_tiles,
                                                 uint8_t *__restrict__ on_path, uint32_t *__restrict__ tile_frames) {
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= n_tiles) return;
    uint32_t e = tile_entry[t], cnt = 0;
    if (e != kNone) {
        const uint32_t end = tile_base[t] + tile_count[t];
        for (uint32_t i = e;;) {
            const fws_frame_info fi = info[i];
            if (fi.hdr_len) { on_path[i] = 1; ++cnt; }
            if (leaf[i] == i) break;
            const uint64_t x = exit_of(fi);
            uint32_t j = i + 1;
            while (j < end && info[j].hdr_off < x) ++j;
            if (j >= end || info[j].hdr_off != x) break;      // cannot happen for a live chain
            i = j;
        }
    }
    tile_frames[t] = cnt;
}

// Single-workgroup exclusive scan of per-tile frame counts (tiles <= 2^20).
__global__ __launch_bounds__(kMarkBlock) void k_tile_scan(const uint32_t *__restrict__ tile_frames,
                                                          uint32_t n_tiles, uint32_t *__restrict__ fbase,
                                                          uint32_t *__restrict__ counters) {
    __shared__ uint32_t swsum[kMarkBlock / 64];
    __shared__ uint32_t scarry;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) scarry = 0;
    __syncthreads();
    for (uint32_t b = 0; b < n_tiles; b += kMarkBlock) {
        const uint32_t t = b + tid;
        const uint32_t c = t < n_tiles ? tile_frames[t] : 0u;
        uint32_t inc = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t x = __shfl_up(inc, o, 64);
            if (lane >= o) inc += x;
        }
        if (lane == 63) swsum[w] = inc;
        __syncthreads();
        uint32_t off = 0, tot = 0;
        for (int i = 0; i < kMarkBlock / 64; ++i) {
            off += (i < w) ? swsum[i] : 0u;
            tot += swsum[i];
        }
        const uint32_t carry = scarry;
        if (t < n_tiles) fbase[t] = carry + off + inc - c;
        __syncthreads();
        if (tid == 0) scarry = carry + tot;
        __syncthreads();
    }
    if (tid == 0) counters[kCntFrames] = scarry;
}

// One wave per tile: write the tile's flagged frames in order.
__global__ __launch_bounds__(kBlock) void k_emit(const fws_frame_info *__restrict__ info,
                                                 const uint32_t *__restrict__ tile_base,
                                                 const uint32_t *__restrict__ tile_count,
                                                 const uint8_t *__restrict__ on_path,
                                                 const uint32_t *__restrict__ fbase, uint32_t n_tiles,
                                                 uint64_t N, fws_frame_info *__restrict__ frames, uint32_t cap,
                                                 fws_frame_desc *__restrict__ descs, uint32_t desc_cap) {
    const uint32_t t = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= n_tiles) return;
    const uint32_t b = tile_base[t], n = tile_count[t];
    uint32_t out = fbase[t];
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
        const uint32_t i = b + i0 + lane;
        const bool f = (i0 + lane < n) && on_path[i];
        const uint64_t m = __ballot(f);
        if (f) {
            const uint32_t o = out + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            const fws_frame_info fi = info[i];
            if (o < cap) frames[o] = fi;
            if (o < desc_cap) {
                const uint64_t po = fi.hdr_off + fi.hdr_len;
                const uint64_t pl = (po + fi.payload_len > N) ? (N - po) : fi.payload_len;
                descs[o] = fws_frame_desc{po, pl, fi.key, 0u};
            }
        }
        out += (uint32_t)__popcll(m);
    }
}

// ------------------------------------------------------------------ k_finish
// Single thread. Terminal of the true chain -> fws_decode_result. For a
// protocol error the headers between the last survivor and the failing one
// (same tile) are walked here, in global memory, and appended as frames.
__global__ void k_finish(const uint8_t *__restrict__ wire, uint64_t N, const fws_frame_info *__restrict__ info,
                         uint32_t *__restrict__ counters, fws_frame_info *__restrict__ frames, uint32_t cap,
                         fws_frame_desc *__restrict__ descs, uint32_t desc_cap,
                         fws_decode_result *__restrict__ res, uint32_t n_surv_cap_hit) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    fws_decode_result r{};
    r.status = FWS_OK;
    uint32_t nf = counters[kCntFrames];
    r.n_survivors = counters[kCntSurv];
    if (counters[kCntOverflow]) {
        r.status = FWS_ERR_CAPACITY;
        r.n_frames = 0;
        counters[kCntFrames] = 0;
        *res = r;
        return;
    }
    const uint32_t term = counters[kCntTerm], last = counters[kCntLast];
    uint64_t pos;            // offset of the next header after the decoded chain
    if (N == 0) {
        pos = 0;
    } else if (last == kNone) {
        pos = 0;             // no survivor at offset 0: walk from the start
    } else {
        const fws_frame_info fi = info[last];
        pos = fi.hdr_len ? exit_of(fi) : fi.hdr_off;
    }
    if (N > 0 && (last == kNone || term == kTermDead)) {
        // walk headers from `pos` (ParseFrameHdr on global bytes) until the error
        for (;;) {
            if (pos >= N) break;
            Hdr h;
            const uint64_t q = pos;
            const int rc = parse_hdr([&](int i) -> uint32_t { return wire[q + i]; }, N - q, true, h);
            if (rc < 0) { r.status = rc; r.err_off = q; break; }
            if (rc == 0) break;                       // incomplete trailing header
            fws_frame_info fi;
            fi.hdr_off = q; fi.payload_len = h.plen; fi.key = h.key; fi.opcode = (uint8_t)h.opcode;
            fi.fin = (uint8_t)h.fin; fi.hdr_len = (uint8_t)rc;
            fi.flags = (q + rc + h.plen > N) ? (uint8_t)FWS_FRAME_TRUNCATED : (uint8_t)0;
            if (nf < cap) frames[nf] = fi;
            if (nf < desc_cap) {
                const uint64_t po = q + rc;
                descs[nf] = fws_frame_desc{po, (po + h.plen > N) ? N - po : h.plen, h.key, 0u};
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
    if (nf > cap && r.status == FWS_OK) r.status = FWS_ERR_CAPACITY;
    r.n_frames = nf;
    counters[kCntFrames] = nf < desc_cap ? nf : desc_cap;
    *res = r;
    (void)n_surv_cap_hit;
}

}  // namespace fwsk

// ------------------------------------------------------------------ host side
using namespace fwsk;

static uint32_t ceil_log2(uint64_t x) {
    uint32_t k = 0;
    while ((1ull << k) < x) ++k;
    return k;
}

int fws_decode_ensure(fws_gpu_ctx *ctx, uint64_t N, uint32_t cap) {
    fws_decode_ws &d = ctx->dec;
    const uint64_t tiles = (N + kTile - 1) / kTile + 1;
    uint64_t s_cap = N / 256 + 8 * tiles + (uint64_t)cap + 64;
    if (ctx->cap_frames + 8 * tiles > s_cap) s_cap = ctx->cap_frames + 8 * tiles;
    const uint32_t levels = ceil_log2(2 * tiles + 2) + 1;
    if (tiles <= d.max_tiles && s_cap <= d.max_surv && levels <= d.levels && cap <= d.max_descs) return 0;
    const uint64_t nt = tiles > d.max_tiles ? tiles : d.max_tiles;
    const uint64_t ns = s_cap > d.max_surv ? s_cap : d.max_surv;
    const uint32_t nl = levels > d.levels ? levels : d.levels;
    const uint64_t nd = cap > d.max_descs ? cap : d.max_descs;
    auto rel = [](auto *&p) { if (p) (void)hipFree(p); p = nullptr; };
    rel(d.tile_count); rel(d.tile_base); rel(d.tile_entry); rel(d.tile_frames); rel(d.fbase);
    rel(d.surv_info); rel(d.surv_leaf); rel(d.jump); rel(d.on_path); rel(d.path); rel(d.counters);
    rel(d.descs);
    hipError_t e = hipSuccess;
    auto al = [&](auto **p, uint64_t bytes) { if (e == hipSuccess) e = hipMalloc((void **)p, bytes ? bytes : 16); };
    al(&d.tile_count, nt * 4); al(&d.tile_base, nt * 4); al(&d.tile_entry, nt * 4);
    al(&d.tile_frames, nt * 4); al(&d.fbase, nt * 4);
    al(&d.surv_info, ns * sizeof(fws_frame_info)); al(&d.surv_leaf, ns * 4);
    al(&d.jump, (uint64_t)nl * ns * 4); al(&d.on_path, ns); al(&d.path, (2 * nt + 8) * 4);
    al(&d.counters, kCntCount * 4 + 16);
    al(&d.descs, (nd + 1) * sizeof(fws_frame_desc));
    if (e != hipSuccess) return fws_hip_status(e);
    d.max_tiles = nt; d.max_surv = ns; d.levels = nl; d.max_descs = nd;
    return 0;
}

int fws_launch_decode(fws_gpu_ctx *ctx, uint8_t *wire, uint64_t N, fws_frame_info *frames, uint32_t cap,
                      fws_decode_result *res, hipStream_t s) {
    fws_decode_ws &d = ctx->dec;
    const uint32_t n_tiles = (uint32_t)((N + kTile - 1) / kTile);
    const uint32_t K = ceil_log2(2ull * n_tiles + 2) + 1;
    hipError_t e;
    if ((e = hipMemsetAsync(d.counters, 0, kCntCount * 4, s)) != hipSuccess) return fws_hip_status(e);
    // root defaults to kNone (0xFF bytes), tile entries to kNone
    if ((e = hipMemsetAsync(d.counters + kCntRoot, 0xFF, 4, s)) != hipSuccess) return fws_hip_status(e);
    if (n_tiles) {
        if ((e = hipMemsetAsync(d.tile_entry, 0xFF, (size_t)n_tiles * 4, s)) != hipSuccess) return fws_hip_status(e);
        hipLaunchKernelGGL(k_scan, dim3(n_tiles), dim3(kBlock), 0, s, wire, N, d.surv_info, d.surv_leaf,
                           d.tile_base, d.tile_count, d.counters, (uint32_t)d.max_surv);
        const int gl = 1024;
        hipLaunchKernelGGL(k_link, dim3(gl), dim3(kBlock), 0, s, d.surv_info, d.surv_leaf, d.tile_base,
                           d.tile_count, d.counters, N, d.jump, d.counters + kCntRoot);
        for (uint32_t k = 1; k < K; ++k)
            hipLaunchKernelGGL(k_jump, dim3(gl), dim3(kBlock), 0, s, d.jump + (uint64_t)(k - 1) * d.max_surv,
                               d.jump + (uint64_t)k * d.max_surv, d.counters);
        hipLaunchKernelGGL(k_mark, dim3(1), dim3(kMarkBlock), 0, s, d.jump, d.max_surv, (int)K, d.surv_info,
                           d.surv_leaf, d.path, d.tile_entry, d.counters, d.counters + kCntRoot);
        if ((e = hipMemsetAsync(d.on_path, 0, d.max_surv, s)) != hipSuccess) return fws_hip_status(e);
        hipLaunchKernelGGL(k_walk, dim3((n_tiles + kBlock - 1) / kBlock), dim3(kBlock), 0, s, d.surv_info,
                           d.surv_leaf, d.tile_base, d.tile_count, d.tile_entry, n_tiles, d.on_path,
                           d.tile_frames);
        hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(kMarkBlock), 0, s, d.tile_frames, n_tiles, d.fbase,
                           d.counters);
        hipLaunchKernelGGL(k_emit, dim3((n_tiles + 3) / 4), dim3(kBlock), 0, s, d.surv_info, d.tile_base,
                           d.tile_count, d.on_path, d.fbase, n_tiles, N, frames, cap, d.descs,
                           (uint32_t)d.max_descs);
    }
    hipLaunchKernelGGL(k_finish, dim3(1), dim3(64), 0, s, wire, N, d.surv_info, d.counters, frames, cap, d.descs,
                       (uint32_t)d.max_descs, res, 0u);
    return fws_hip_status(hipGetLastError());
}
