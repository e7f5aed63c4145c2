// decode_kernels.hip -- fused header parse + unmask of a raw server-side wire
// stream on gfx950 (fws_gpu_decode_stream). Replaces the serial frame loop of
// WSocket::OnRecvData (net/w_socket.h:543-769) for a device-resident buffer.
//
// Frame boundaries are a serial dependency (header i+1's offset comes from
// header i's length), so the stream is parsed speculatively and in parallel:
//
//  k_scan   one workgroup per 16 KiB tile staged in LDS. A two-byte test
//           drops every offset that cannot start a masked header; the rest
//           (~2% of random payload bytes) are parsed with ParseFrameHdr's
//           semantics (w_socket.h:435-524) and point at the next header.
//           Pointer jumping in LDS resolves every chain to the last header
//           before the tile end (its "leaf") or to DEAD (an invalid header).
//           Offsets whose chain survives are "survivors": every true header
//           is one, few random offsets are.
//  k_link   survivor graph: a non-leaf points at its leaf; a leaf points at
//           the survivor at its exit offset in a later tile (binary search),
//           or at a terminal (END, DEAD = invalid header, INCOMPLETE header).
//  k_jump   pointer doubling tables J_k = J_{k-1} o J_{k-1} (K-1 launches,
//           K = ceil(log2(path bound)); the path visits <= 2 nodes per tile).
//  k_entry  one thread per tile: binary lifting through J_k from the root
//           finds the tile's first true header (offsets increase along the path).
//  k_walk / k_tile_sums / k_tile_scan / k_emit
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
    kCntSpill = 7,       // survivors spilled by dense tiles
    kCntCount = 8
};

// ------------------------------------------------------------------ k_scan
// Offsets whose first two bytes cannot start a server-side header (RSV set,
// reserved opcode, MASK clear: w_socket.h:451-515) are dead on sight; only the
// rest ("candidates", ~2% of random payload bytes) are parsed in full and
// pointer-jumped. Candidate k is the k-th set bit of cbits (node index).
//
// Each thread owns kScanChunks 16-byte chunks of the tile and keeps a 32-byte
// register window (its chunk + the next one) from which the candidate test
// and every header parse read with constant byte indices: after the window
// load, the tile bytes in LDS are dead and the node table reuses them.
constexpr int kScanThreads = 512;
constexpr int kScanChunks = int(kTile / 16u) / kScanThreads;
constexpr int kScanWords = int(kTile / 64u);          // 64-offset bitmap words (256)

template <int kT>
__device__ __forceinline__ uint32_t block_excl_scan_u32(uint32_t c, uint32_t *swsum, uint32_t *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t x = __shfl_up(inc, o, 64);
        if (lane >= o) inc += x;
    }
    if (lane == 63) swsum[w] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kT / 64; ++i) {
        off += (i < w) ? swsum[i] : 0u;
        tot += swsum[i];
    }
    __syncthreads();
    *total = tot;
    return off + inc - c;
}

// Bit i set <=> offset i of the chunk passes the two-byte header test
// (RSV clear, opcode in {0,1,2,8,9,10}, MASK set), four offsets per dword:
// rsv:  (b0 & 0x70) == 0      <=> bit 7 of (b0 & 0x70) + 0x7F is clear
// op:   (b0 & 7) <= 2         <=> bit 3 of (b0 & 7) + 5 is clear
// mask: bit 7 of b1 (= byte i+1, v_alignbyte by one)
__device__ __forceinline__ uint32_t cand_bits16(const u32x4 &lo, uint32_t next_dword) {
    const uint32_t W[5] = {lo.x, lo.y, lo.z, lo.w, next_dword};
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t x = W[i];
        const uint32_t b1 = __builtin_amdgcn_alignbyte(W[i + 1], x, 1u);
        const uint32_t rsv_ok = ~((x & 0x70707070u) + 0x7F7F7F7Fu);
        const uint32_t op_ok = (~((x & 0x07070707u) + 0x05050505u)) << 4;
        const uint32_t f = rsv_ok & op_ok & b1 & 0x80808080u;
        m |= (((f >> 7) & 1u) | ((f >> 14) & 2u) | ((f >> 21) & 4u) | ((f >> 28) & 8u)) << (4 * i);
    }
    return m;
}

// Bytes b..b+15 (b < 16) of the 32-byte window lo:hi as four dwords: shift by
// 8 bytes, then 4, then v_alignbyte -- selects on named values, no indexing.
__device__ __forceinline__ void window16(const u32x4 &lo, const u32x4 &hi, uint32_t b, uint32_t out[4]) {
    const bool s8 = (b & 8u) != 0, s4 = (b & 4u) != 0;
    const uint32_t a0 = s8 ? lo.z : lo.x, a1 = s8 ? lo.w : lo.y, a2 = s8 ? hi.x : lo.z;
    const uint32_t a3 = s8 ? hi.y : lo.w, a4 = s8 ? hi.z : hi.x, a5 = s8 ? hi.w : hi.y;
    const uint32_t c0 = s4 ? a1 : a0, c1 = s4 ? a2 : a1, c2 = s4 ? a3 : a2;
    const uint32_t c3 = s4 ? a4 : a3, c4 = s4 ? a5 : a4;
    const uint32_t sh = b & 3u;
    out[0] = __builtin_amdgcn_alignbyte(c1, c0, sh);
    out[1] = __builtin_amdgcn_alignbyte(c2, c1, sh);
    out[2] = __builtin_amdgcn_alignbyte(c3, c2, sh);
    out[3] = __builtin_amdgcn_alignbyte(c4, c3, sh);
}

// parse_hdr (server side) on a register window; same codes and order of checks
// as ParseFrameHdr (w_socket.h:435-524), with the key picked by its length form
// so no byte index is dynamic (a dynamic index would spill the window).
__device__ __forceinline__ int parse_window(const u32x4 &lo, const u32x4 &hi, uint32_t b, uint64_t avail, Hdr &h) {
    uint32_t d[4];
    window16(lo, hi, b, d);
    if (avail < 2) return 0;                                       // :443-445
    const uint32_t b0 = d[0] & 0xFFu, b1 = (d[0] >> 8) & 0xFFu;
    h.opcode = b0 & 15u;
    if (!valid_opcode(h.opcode)) return FWS_ERR_OPCODE;            // :451-454
    h.fin = b0 >> 7;
    if (b0 & 112u) return FWS_ERR_RSV;                             // :466-470
    uint64_t plen = b1 & 127u;
    int n = 2;
    uint32_t key = __builtin_amdgcn_alignbyte(d[1], d[0], 2u);     // bytes 2..5
    if (plen == 126u) {                                            // :476-482
        if (avail < 4) return 0;
        plen = ((d[0] >> 8) & 0xFF00u) | (d[0] >> 24);
        n = 4;
        key = d[1];                                                // bytes 4..7
    } else if (plen == 127u) {                                     // :483-492
        if (avail < 10) return 0;
        const uint32_t hi32 = __builtin_amdgcn_alignbyte(d[1], d[0], 2u);   // bytes 2..5
        const uint32_t lo32 = __builtin_amdgcn_alignbyte(d[2], d[1], 2u);   // bytes 6..9
        plen = (uint64_t(__builtin_bswap32(hi32)) << 32) | __builtin_bswap32(lo32);
        n = 10;
        key = __builtin_amdgcn_alignbyte(d[3], d[2], 2u);          // bytes 10..13
    }
    if (plen > (1ull << 32)) return FWS_ERR_TOO_LARGE;             // :493-498
    h.plen = plen;
    if (!(b1 >> 7)) return FWS_ERR_NOT_MASKED;                     // :502-507
    if (avail < (uint64_t)n + 4u) return 0;                        // :508-511
    h.key = key;
    return n + 4;
}

constexpr uint32_t kSlots = 32;              // per-tile survivor slots before spilling

__global__ __launch_bounds__(kScanThreads) void k_scan(const uint8_t *__restrict__ wire, uint64_t N,
                                                       fws_frame_info *__restrict__ stage_info,
                                                       uint32_t *__restrict__ stage_leaf,
                                                       fws_frame_info *__restrict__ spill_info,
                                                       uint32_t *__restrict__ spill_leaf,
                                                       uint32_t *__restrict__ tile_spill,
                                                       uint32_t *__restrict__ tile_count,
                                                       uint32_t *__restrict__ counters, uint32_t s_cap) {
    // tile bytes (phase 1) and node table (phase 2+) share the same LDS
    __shared__ __attribute__((aligned(16))) union {
        uint8_t bytes[kTile + kHalo];
        uint16_t nval[kTile];                // per candidate: next candidate, kLeaf|self, kDead
    } sm;
    __shared__ uint64_t cbits[kScanWords];   // candidate offsets
    __shared__ uint32_t cpre[kScanWords];
    __shared__ uint64_t sbits[kScanWords];   // surviving candidates (by node index)
    __shared__ uint32_t spre[kScanWords];
    __shared__ uint32_t swsum[kScanThreads / 64];
    __shared__ uint32_t sbase, stotal;

    const uint32_t t = blockIdx.x;
    const uint64_t t0 = uint64_t(t) * kTile;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint8_t *sbuf = sm.bytes;

    // stage the tile + halo (wire is 16-B aligned, tiles are 16-B multiples)
    const bool interior = t0 + kTile + kHalo <= N;
    if (interior) {
        u32x4 v[kScanChunks];
#pragma unroll
        for (int j = 0; j < kScanChunks; ++j)
            v[j] = gload16(reinterpret_cast<uintptr_t>(wire + t0 + (uint64_t)(j * kScanThreads + tid) * 16u));
        u32x4 hv;
        if (tid == 0) hv = gload16(reinterpret_cast<uintptr_t>(wire + t0 + kTile));
#pragma unroll
        for (int j = 0; j < kScanChunks; ++j)
            *reinterpret_cast<u32x4 *>(sbuf + (j * kScanThreads + tid) * 16) = v[j];
        if (tid == 0) *reinterpret_cast<u32x4 *>(sbuf + kTile) = hv;
    } else {
        for (uint32_t i = tid * 16u; i < kTile + kHalo; i += kScanThreads * 16u) {
            const uint64_t q = t0 + i;
            if (q + 16u <= N) {
                *reinterpret_cast<u32x4 *>(sbuf + i) = gload16(reinterpret_cast<uintptr_t>(wire + q));
            } else {
#pragma unroll
                for (int b = 0; b < 16; ++b) sbuf[i + b] = (q + b < N) ? wire[q + b] : 0;
            }
        }
    }
    if (tid < kScanWords) sbits[tid] = 0;
    __syncthreads();

    // register windows + candidate bitmap (16 bits per chunk)
    u32x4 lo[kScanChunks], hi[kScanChunks];
    uint32_t cm[kScanChunks];
#pragma unroll
    for (int j = 0; j < kScanChunks; ++j) {
        const uint32_t c = uint32_t(j * kScanThreads + tid);
        lo[j] = *reinterpret_cast<const u32x4 *>(sbuf + c * 16u);
        hi[j] = *reinterpret_cast<const u32x4 *>(sbuf + c * 16u + 16u);
        uint32_t m = cand_bits16(lo[j], hi[j].x);
        if (!interior) {
            // offsets at or past the end: zero bytes never pass; the last byte
            // is a candidate on its own (an incomplete header, w_socket.h:443-445)
            const uint64_t q = t0 + uint64_t(c) * 16u;
            if (q >= N) m = 0;
            else if (N - q <= 16u) m = (m & ((1u << (N - q)) - 1u)) | (1u << (N - q - 1u));
        }
        cm[j] = m;
        reinterpret_cast<uint16_t *>(cbits)[c] = (uint16_t)m;
    }
    __syncthreads();
    uint32_t nc;
    {
        const uint32_t pc = tid < kScanWords ? (uint32_t)__popcll(cbits[tid]) : 0u;
        const uint32_t e = block_excl_scan_u32<kScanThreads>(pc, swsum, &nc);
        if (tid < kScanWords) cpre[tid] = e;
    }
    __syncthreads();
    auto crank = [&](uint32_t p) -> uint32_t {
        return cpre[p >> 6] + (uint32_t)__popcll(cbits[p >> 6] & ((1ull << (p & 63u)) - 1ull));
    };
    auto chunk_rank = [&](uint32_t c) -> uint32_t {     // node index of the chunk's first candidate
        return cpre[c >> 2] + (uint32_t)__popcll(cbits[c >> 2] & ((1ull << ((c & 3u) * 16u)) - 1ull));
    };

    // parse candidates from the register windows (LDS bytes are dead from here)
    uint32_t kfirst[kScanChunks];
#pragma unroll
    for (int j = 0; j < kScanChunks; ++j) {
        const uint32_t c = uint32_t(j * kScanThreads + tid);
        uint32_t bits = cm[j];
        uint32_t k = chunk_rank(c);
        kfirst[j] = k;
        while (bits) {
            const uint32_t b = (uint32_t)__ffs(bits) - 1u;
            bits &= bits - 1u;
            const uint32_t p = c * 16u + b;
            const uint64_t q = t0 + p;
            Hdr h;
            const int r = parse_window(lo[j], hi[j], b, N - q, h);
            uint16_t v = kDead;
            if (r == 0) {
                v = (uint16_t)(kLeaf | k);                // incomplete header at the stream end
            } else if (r > 0) {
                const uint64_t nx = q + (uint64_t)r + h.plen;
                if (nx < t0 + kTile) {
                    const uint32_t pn = (uint32_t)(nx - t0);
                    v = ((cbits[pn >> 6] >> (pn & 63u)) & 1ull) ? (uint16_t)crank(pn) : kDead;
                } else {
                    v = (uint16_t)(kLeaf | k);
                }
            }
            sm.nval[k] = v;
            ++k;
        }
    }
    __syncthreads();

    // pointer jumping over candidate nodes: every chain ends at its leaf or dies
    for (;;) {
        int changed = 0;
        for (uint32_t k = tid; k < nc; k += kScanThreads) {
            const uint16_t v = sm.nval[k];
            if (v < kTile) {
                sm.nval[k] = sm.nval[v];
                changed = 1;
            }
        }
        if (!__syncthreads_or(changed)) break;
    }

    // survivors by node index
    for (uint32_t k0 = uint32_t(w) * 64u; k0 < nc; k0 += kScanThreads) {
        const uint32_t k = k0 + uint32_t(lane);
        const uint64_t m = __ballot(k < nc && sm.nval[k] != kDead);
        if (lane == 0) sbits[k0 >> 6] = m;
    }
    __syncthreads();
    uint32_t ns;
    {
        const uint32_t pc = tid < kScanWords ? (uint32_t)__popcll(sbits[tid]) : 0u;
        const uint32_t e = block_excl_scan_u32<kScanThreads>(pc, swsum, &ns);
        if (tid < kScanWords) spre[tid] = e;
    }
    // survivors go to the tile's fixed slots (no shared counter); a tile with
    // more than kSlots of them (dense small frames) spills to a shared area
    if (tid == 0) {
        uint32_t spill = kNone;
        if (ns > kSlots) {
            spill = atomicAdd(&counters[kCntSpill], ns);
            if (spill + ns > s_cap) { atomicOr(&counters[kCntOverflow], 1u); ns = 0; spill = kNone; }
        }
        sbase = spill;
        stotal = ns;
        tile_count[t] = ns;
        tile_spill[t] = spill;
    }
    __syncthreads();
    if (stotal == 0) return;
    fws_frame_info *out_info = sbase == kNone ? stage_info + (uint64_t)t * kSlots : spill_info + sbase;
    uint32_t *out_leaf = sbase == kNone ? stage_leaf + (uint64_t)t * kSlots : spill_leaf + sbase;
    auto srank = [&](uint32_t k) -> uint32_t {
        return spre[k >> 6] + (uint32_t)__popcll(sbits[k >> 6] & ((1ull << (k & 63u)) - 1ull));
    };

    // write survivors in offset order
#pragma unroll
    for (int j = 0; j < kScanChunks; ++j) {
        const uint32_t c = uint32_t(j * kScanThreads + tid);
        uint32_t bits = cm[j];
        uint32_t k = kfirst[j];
        while (bits) {
            const uint32_t b = (uint32_t)__ffs(bits) - 1u;
            bits &= bits - 1u;
            const uint16_t v = sm.nval[k];
            if (v != kDead) {
                const uint64_t q = t0 + c * 16u + b;
                Hdr h;
                const int r = parse_window(lo[j], hi[j], b, N - q, h);
                fws_frame_info fi;
                fi.hdr_off = q;
                if (r > 0) {
                    fi.payload_len = h.plen;
                    fi.key = h.key;
                    fi.opcode = (uint8_t)h.opcode;
                    fi.fin = (uint8_t)h.fin;
                    fi.hdr_len = (uint8_t)r;
                    fi.flags = (q + (uint64_t)r + h.plen > N) ? (uint8_t)FWS_FRAME_TRUNCATED : (uint8_t)0;
                } else {                                 // incomplete trailing header
                    fi.payload_len = 0;
                    fi.key = 0;
                    fi.opcode = 0;
                    fi.fin = 0;
                    fi.hdr_len = 0;
                    fi.flags = 0;
                }
                const uint32_t idx = srank(k);
                out_info[idx] = fi;
                out_leaf[idx] = srank(v & 0x7FFFu);            // tile-local rank of the leaf
            }
            ++k;
        }
    }
}

// ------------------------------------------------------------------ k_compact
// One wave per tile: survivors from the tile's slots (or its spill range) to
// the dense, offset-sorted arrays at tile_base[t]; leaf ranks become indices.
__global__ __launch_bounds__(kBlock) void k_compact(const fws_frame_info *__restrict__ stage_info,
                                                    const uint32_t *__restrict__ stage_leaf,
                                                    const fws_frame_info *__restrict__ spill_info,
                                                    const uint32_t *__restrict__ spill_leaf,
                                                    const uint32_t *__restrict__ tile_spill,
                                                    const uint32_t *__restrict__ tile_count,
                                                    const uint32_t *__restrict__ tile_base, uint32_t n_tiles,
                                                    fws_frame_info *__restrict__ surv_info,
                                                    uint32_t *__restrict__ surv_leaf, uint32_t *__restrict__ counters,
                                                    uint32_t s_cap) {
    const uint32_t t = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= n_tiles) return;
    const uint32_t n = tile_count[t], b = tile_base[t], sp = tile_spill[t];
    if (b + n > s_cap) {
        if (lane == 0) atomicOr(&counters[kCntOverflow], 1u);
        return;
    }
    const fws_frame_info *si = sp == kNone ? stage_info + (uint64_t)t * kSlots : spill_info + sp;
    const uint32_t *sl = sp == kNone ? stage_leaf + (uint64_t)t * kSlots : spill_leaf + sp;
    for (uint32_t r = lane; r < n; r += 64) {
        surv_info[b + r] = si[r];
        surv_leaf[b + r] = b + sl[r];
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

// ------------------------------------------------------------------ k_entry
// One thread per tile, binary lifting over the doubling tables: the last path
// node before the tile (headers strictly increase along the path), then its
// successor is the tile's first true header if that lies inside the tile.
// Thread n_tiles finds the path's last node and terminal.
__global__ __launch_bounds__(kBlock) void k_entry(const uint32_t *__restrict__ J, uint64_t s_cap, int K,
                                                  const fws_frame_info *__restrict__ info,
                                                  const uint32_t *__restrict__ root_p, uint32_t n_tiles,
                                                  uint32_t *__restrict__ tile_entry,
                                                  uint32_t *__restrict__ counters) {
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t > n_tiles) return;
    const uint32_t root = *root_p;
    if (counters[kCntOverflow] || root == kNone) {
        if (t == n_tiles) { counters[kCntTerm] = kTermDead; counters[kCntLast] = kNone; }
        return;
    }
    if (t == n_tiles) {
        uint32_t cur = root;
        for (int k = K - 1; k >= 0; --k) {
            const uint32_t y = J[(uint64_t)k * s_cap + cur];
            if (!is_term(y)) cur = y;
        }
        counters[kCntLast] = cur;
        counters[kCntTerm] = J[cur];
        return;
    }
    if (t == 0) { tile_entry[0] = root; return; }
    const uint64_t T0 = (uint64_t)t * kTile;
    uint32_t cur = root;                                  // hdr_off 0 < T0
    for (int k = K - 1; k >= 0; --k) {
        const uint32_t y = J[(uint64_t)k * s_cap + cur];
        if (!is_term(y) && info[y].hdr_off < T0) cur = y;
    }
    const uint32_t y = J[cur];
    if (!is_term(y) && info[y].hdr_off < T0 + kTile) tile_entry[t] = y;
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

// Exclusive scan of per-tile frame counts: per-1024-tile block sums, then
// each block adds the sums of the blocks before it (few: tiles / 1024).
__global__ __launch_bounds__(kBlock) void k_tile_sums(const uint32_t *__restrict__ tile_frames, uint32_t n_tiles,
                                                      uint32_t *__restrict__ block_sums) {
    __shared__ uint32_t swsum[kBlock / 64];
    uint32_t c = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t t = blockIdx.x * 1024u + threadIdx.x * 4u + i;
        if (t < n_tiles) c += tile_frames[t];
    }
    uint32_t tot;
    block_excl_scan_u32<kBlock>(c, swsum, &tot);
    if (threadIdx.x == 0) block_sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void k_tile_scan(const uint32_t *__restrict__ tile_frames, uint32_t n_tiles,
                                                      const uint32_t *__restrict__ block_sums,
                                                      uint32_t *__restrict__ fbase, uint32_t *__restrict__ total_out) {
    __shared__ uint32_t swsum[kBlock / 64];
    uint32_t pre = 0, dummy;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += kBlock) pre += block_sums[b];
    const uint32_t pe = block_excl_scan_u32<kBlock>(pre, swsum, &dummy);
    __shared__ uint32_t sprefix;
    if (threadIdx.x == kBlock - 1) sprefix = pe + pre;
    __syncthreads();
    const uint32_t t0 = blockIdx.x * 1024u + threadIdx.x * 4u;
    uint32_t c[4], sum = 0;
    for (int i = 0; i < 4; ++i) { c[i] = (t0 + i < n_tiles) ? tile_frames[t0 + i] : 0u; sum += c[i]; }
    uint32_t tot;
    uint32_t run = sprefix + block_excl_scan_u32<kBlock>(sum, swsum, &tot);
    for (int i = 0; i < 4; ++i) {
        if (t0 + i < n_tiles) {
            fbase[t0 + i] = run;
            run += c[i];
            if (t0 + i == n_tiles - 1) *total_out = run;
        }
    }
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
    rel(d.descs); rel(d.stage_info); rel(d.stage_leaf); rel(d.spill_info); rel(d.spill_leaf); rel(d.tile_spill);
    hipError_t e = hipSuccess;
    auto al = [&](auto **p, uint64_t bytes) { if (e == hipSuccess) e = hipMalloc((void **)p, bytes ? bytes : 16); };
    al(&d.tile_count, nt * 4); al(&d.tile_base, nt * 4); al(&d.tile_entry, nt * 4);
    al(&d.tile_frames, nt * 4); al(&d.fbase, nt * 4);
    al(&d.surv_info, ns * sizeof(fws_frame_info)); al(&d.surv_leaf, ns * 4);
    al(&d.jump, (uint64_t)nl * ns * 4); al(&d.on_path, ns); al(&d.path, (2 * nt + 8) * 4);
    al(&d.counters, kCntCount * 4 + 16);
    al(&d.descs, (nd + 1) * sizeof(fws_frame_desc));
    al(&d.stage_info, nt * kSlots * sizeof(fws_frame_info)); al(&d.stage_leaf, nt * kSlots * 4);
    al(&d.spill_info, ns * sizeof(fws_frame_info)); al(&d.spill_leaf, ns * 4); al(&d.tile_spill, nt * 4);
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
        const uint32_t tb = (n_tiles + 1023) / 1024;
        hipLaunchKernelGGL(k_scan, dim3(n_tiles), dim3(kScanThreads), 0, s, wire, N, d.stage_info, d.stage_leaf,
                           d.spill_info, d.spill_leaf, d.tile_spill, d.tile_count, d.counters,
                           (uint32_t)d.max_surv);
        hipLaunchKernelGGL(k_tile_sums, dim3(tb), dim3(kBlock), 0, s, d.tile_count, n_tiles, d.path);
        hipLaunchKernelGGL(k_tile_scan, dim3(tb), dim3(kBlock), 0, s, d.tile_count, n_tiles, d.path, d.tile_base,
                           d.counters + kCntSurv);
        hipLaunchKernelGGL(k_compact, dim3((n_tiles + 3) / 4), dim3(kBlock), 0, s, d.stage_info, d.stage_leaf,
                           d.spill_info, d.spill_leaf, d.tile_spill, d.tile_count, d.tile_base, n_tiles,
                           d.surv_info, d.surv_leaf, d.counters, (uint32_t)d.max_surv);
        const int gl = 1024;
        hipLaunchKernelGGL(k_link, dim3(gl), dim3(kBlock), 0, s, d.surv_info, d.surv_leaf, d.tile_base,
                           d.tile_count, d.counters, N, d.jump, d.counters + kCntRoot);
        for (uint32_t k = 1; k < K; ++k)
            hipLaunchKernelGGL(k_jump, dim3(gl), dim3(kBlock), 0, s, d.jump + (uint64_t)(k - 1) * d.max_surv,
                               d.jump + (uint64_t)k * d.max_surv, d.counters);
        hipLaunchKernelGGL(k_entry, dim3(n_tiles / kBlock + 1), dim3(kBlock), 0, s, d.jump, d.max_surv, (int)K,
                           d.surv_info, d.counters + kCntRoot, n_tiles, d.tile_entry, d.counters);
        if ((e = hipMemsetAsync(d.on_path, 0, d.max_surv, s)) != hipSuccess) return fws_hip_status(e);
        hipLaunchKernelGGL(k_walk, dim3((n_tiles + kBlock - 1) / kBlock), dim3(kBlock), 0, s, d.surv_info,
                           d.surv_leaf, d.tile_base, d.tile_count, d.tile_entry, n_tiles, d.on_path,
                           d.tile_frames);
        hipLaunchKernelGGL(k_tile_sums, dim3(tb), dim3(kBlock), 0, s, d.tile_frames, n_tiles, d.path);
        hipLaunchKernelGGL(k_tile_scan, dim3(tb), dim3(kBlock), 0, s, d.tile_frames, n_tiles, d.path, d.fbase,
                           d.counters + kCntFrames);
        hipLaunchKernelGGL(k_emit, dim3((n_tiles + 3) / 4), dim3(kBlock), 0, s, d.surv_info, d.tile_base,
                           d.tile_count, d.on_path, d.fbase, n_tiles, N, frames, cap, d.descs,
                           (uint32_t)d.max_descs);
    }
    hipLaunchKernelGGL(k_finish, dim3(1), dim3(64), 0, s, wire, N, d.surv_info, d.counters, frames, cap, d.descs,
                       (uint32_t)d.max_descs, res, 0u);
    return fws_hip_status(hipGetLastError());
}
