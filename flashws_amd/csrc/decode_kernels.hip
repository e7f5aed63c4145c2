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
#include "decode_common.h"

namespace fwsk {

// ------------------------------------------------------------------ k_scan
// Offsets whose first two bytes cannot start a server-side header (RSV set,
// reserved opcode, MASK clear: w_socket.h:451-515) are dead on sight; only the
// rest ("candidates", ~2% of random payload bytes) are parsed in full and
// pointer-jumped. Candidate k is the k-th candidate offset of the tile (node).
//
// One wavefront owns one 2 KiB tile at a time (lane L: bytes 32L..32L+31), so
// every step is wave-synchronous: ballots, shuffles and the wave's private LDS
// area, no workgroup barrier anywhere in the scan.
constexpr int kScanWaves = 4;                          // wavefronts per workgroup
constexpr int kScanThreads = kScanWaves * 64;
constexpr uint32_t kWCap = 1024;                       // node list capacity of a sparse tile


// Bit i set <=> offset i of the chunk passes the two-byte header test
// (RSV clear, opcode in {0,1,2,8,9,10}, MASK set), four offsets per dword.
// RSV clear and (b0 & 7) <= 2 <=> (b0 & 0x77) <= 2 <=> bit 7 of
// (b0 & 0x77) + 0x7D is clear (no carry leaves the byte: 0x77 + 0x7D < 0x100);
// MASK is bit 7 of b1 (= byte i+1, v_alignbyte by one).
__device__ __forceinline__ uint32_t cand_bits16(const u32x4 &lo, uint32_t next_dword) {
    const uint32_t W[5] = {lo.x, lo.y, lo.z, lo.w, next_dword};
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t x = W[i];
        const uint32_t b1 = __builtin_amdgcn_alignbyte(W[i + 1], x, 1u);
        const uint32_t f = ~((x & 0x77777777u) + 0x7D7D7D7Du) & b1 & 0x80808080u;
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


// The chain-building part of ParseFrameHdr (w_socket.h:435-524) for an offset
// that passed the two-byte test (so RSV, opcode and MASK are valid): header
// length (> 0), 0 = incomplete (the same avail checks in the same order), or
// FWS_ERR_TOO_LARGE; payload length and key. Window d = bytes p..p+15.
__device__ __forceinline__ int lean_parse(const uint32_t d[4], uint64_t avail, uint64_t &plen, uint32_t &key) {
    if (avail < 2) return 0;                                       // :443-445
    const uint32_t len7 = (d[0] >> 8) & 127u;
    if (len7 < 126u) {
        plen = len7;
        key = __builtin_amdgcn_alignbyte(d[1], d[0], 2u);          // bytes 2..5
        return avail < 6 ? 0 : 6;                                  // :508-511
    }
    if (len7 == 126u) {                                            // :476-482
        if (avail < 4) return 0;
        plen = ((d[0] >> 8) & 0xFF00u) | (d[0] >> 24);
        key = d[1];                                                // bytes 4..7
        return avail < 8 ? 0 : 8;
    }
    if (avail < 10) return 0;                                      // :483-492
    const uint32_t hi32 = __builtin_amdgcn_alignbyte(d[1], d[0], 2u);
    const uint32_t lo32 = __builtin_amdgcn_alignbyte(d[2], d[1], 2u);
    plen = (uint64_t(__builtin_bswap32(hi32)) << 32) | __builtin_bswap32(lo32);
    if (plen > (1ull << 32)) return FWS_ERR_TOO_LARGE;             // :493-498
    key = __builtin_amdgcn_alignbyte(d[3], d[2], 2u);              // bytes 10..13
    return avail < 14 ? 0 : 14;
}

constexpr uint32_t kScanBlocksPerCu = 5;     // resident k_scan workgroups per CU (LDS-limited)

#ifdef FWS_SCAN_PROF
// phase clocks of k_scan summed over wavefronts (tools/prof_scan.py; build: make prof)
__device__ unsigned long long g_scan_prof[16];
#define SCAN_MARK(i)                                                                  \
    do {                                                                              \
        const uint64_t now = clock64();                                               \
        prof_acc[i] += now - prof_t;                                                  \
        prof_t = now;                                                                 \
    } while (0)
#define SCAN_COUNT(i, v) do { prof_acc[i] += (v); } while (0)
#else
#define SCAN_MARK(i) do { } while (0)
#define SCAN_COUNT(i, v) do { } while (0)
#endif

// LDS of one wavefront's tile. Sparse tiles (<= kWCap candidates, the normal
// case) use nodes[] as pos[kWCap] | nval[kWCap]; dense ones as nval[kTile].
struct ScanWaveLds {
    uint8_t bytes[kTile + kHalo];
    uint16_t nodes[2 * kWCap];
    uint32_t cm[64];                         // candidate bits of lane L's 32 offsets
    uint32_t cpre[64];                       // node index of lane L's first candidate
    uint64_t sbits[kTile / 64];              // surviving nodes
    uint32_t spre[kTile / 64];
    fws_frame_info stage[kSlots];            // survivor records before the store
    uint32_t stage_leaf[kSlots];
};
static_assert(2 * kWCap >= kTile, "dense node table must fit");
static_assert(sizeof(ScanWaveLds) % 16 == 0, "16-B aligned per-wave areas");

// LDS ordering among the lanes of one wavefront (a wave's LDS ops execute in order)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t *total) {
    const int lane = threadIdx.x & 63;
    uint32_t inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    *total = __shfl(inc, 63, 64);
    return inc - x;
}

// Persistent: wavefront gw of GW walks tiles t = gw + i * GW; each of its two
// register sets holds a tile in flight, so the HBM reads of the next two tiles
// overlap the LDS work of the current one. The 16 halo bytes (header tail past
// the tile end) come with the tile.
//
// Every tile step issues the same vector-memory sequence -- 3 stores (the
// survivor records, slot-staged in LDS, plus tile_count / tile_spill; idle
// lanes write one shared dummy record) then 3 prefetch loads (clamped to an
// in-bounds tile) -- so the compiler's in-order vmcnt waits for a register
// set count the 6 younger operations and never drain the other set.
// kPipe = false (streams shorter than one tile + halo): no prefetch.
template <bool kPipe>
__global__ __launch_bounds__(kScanThreads) __attribute__((amdgpu_waves_per_eu(5, 5))) void k_scan(const uint8_t *__restrict__ wire, uint64_t N,
                                                       uint32_t n_tiles,
                                                       fws_frame_info *__restrict__ stage_info,
                                                       uint32_t *__restrict__ stage_leaf,
                                                       fws_frame_info *__restrict__ spill_info,
                                                       uint32_t *__restrict__ spill_leaf,
                                                       uint32_t *__restrict__ tile_spill,
                                                       uint32_t *__restrict__ tile_count,
                                                       uint32_t *__restrict__ counters, uint32_t s_cap,
                                                       uint32_t *__restrict__ scan_dummy) {
    __shared__ __attribute__((aligned(16))) ScanWaveLds lds_w[kScanWaves];
    const int lane = threadIdx.x & 63;
    ScanWaveLds &W = lds_w[threadIdx.x >> 6];
    uint8_t *const B = W.bytes;
    const uint32_t gw = blockIdx.x * kScanWaves + (threadIdx.x >> 6);
    const uint32_t GW = gridDim.x * kScanWaves;
    const uint32_t L32 = uint32_t(lane) * 32u;
    const uint32_t L16 = uint32_t(lane) * 16u;
    // last tile whose bytes + halo lie inside the stream (prefetch clamp)
    const uint32_t last_inner = kPipe ? (uint32_t)((N - kHalo) / kTile) - 1u : 0u;
    // idle lanes' stores go to this wave's own 64-B line (L2-resident, no hot spot)
    fws_frame_info *const dummy_info = reinterpret_cast<fws_frame_info *>(scan_dummy + (uint64_t)gw * 16u);
    uint32_t *const dummy_word = scan_dummy + (uint64_t)gw * 16u + 8u;
#ifdef FWS_SCAN_PROF
    uint64_t prof_acc[8] = {};
    uint64_t prof_t = clock64();
    const uint64_t prof_w0 = wall_clock64(), prof_c0 = prof_t;
#endif

    auto prefetch = [&](uint32_t tt, u32x4 (&pf)[2], u32x4 &halo) {
        if (!kPipe) return;
        const uint64_t o = uint64_t(tt < last_inner ? tt : last_inner) * kTile;
        // coalesced: each load instruction reads 1 KiB contiguous (lane L: 16 B at 16L)
        pf[0] = gload16(reinterpret_cast<uintptr_t>(wire + o + L16));
        pf[1] = gload16(reinterpret_cast<uintptr_t>(wire + o + 1024u + L16));
        halo = gload16(reinterpret_cast<uintptr_t>(wire + o + kTile));
    };

    auto tile = [&](const uint32_t t, u32x4 (&pf)[2], u32x4 &halo) {
        const bool valid = t < n_tiles;                    // wave-uniform
        const uint64_t t0 = uint64_t(t) * kTile;
        uint32_t ns = 0, spill = kNone;
        if (valid) {
            const bool inner = kPipe && t <= last_inner;
            if (inner) {
                *reinterpret_cast<u32x4 *>(B + L16) = pf[0];
                *reinterpret_cast<u32x4 *>(B + 1024u + L16) = pf[1];
                if (lane == 0) *reinterpret_cast<u32x4 *>(B + kTile) = halo;
            } else {
                for (uint32_t i = uint32_t(lane) * 16u; i < kTile + kHalo; i += 64u * 16u) {
                    const uint64_t q = t0 + i;
                    if (q + 16u <= N) {
                        *reinterpret_cast<u32x4 *>(B + i) = gload16(reinterpret_cast<uintptr_t>(wire + q));
                    } else {
#pragma unroll
                        for (int b = 0; b < 16; ++b) B[i + b] = (q + b < N) ? wire[q + b] : 0;
                    }
                }
            }
            wave_sync();
            SCAN_MARK(0);

            // candidate bits of this lane's 32 offsets, node numbering by a wave scan
            uint32_t cm;
            {
                const u32x4 w0 = *reinterpret_cast<const u32x4 *>(B + L32);
                const u32x4 w1 = *reinterpret_cast<const u32x4 *>(B + L32 + 16u);
                const uint32_t nx = *reinterpret_cast<const uint32_t *>(B + L32 + 32u);
                cm = cand_bits16(w0, w1.x) | (cand_bits16(w1, nx) << 16);
                if (!inner) {
                    // offsets at or past the end: zero bytes never pass; the last byte
                    // is a candidate on its own (an incomplete header, w_socket.h:443-445)
                    const uint64_t q = t0 + L32;
                    if (q >= N) cm = 0;
                    else if (N - q <= 32u) {
                        const uint32_t r = (uint32_t)(N - q);
                        cm = (uint32_t)(cm & ((1ull << r) - 1ull)) | (1u << (r - 1u));
                    }
                }
            }
            uint32_t nc;
            const uint32_t cp = wave_excl_scan((uint32_t)__popc(cm), &nc);
            W.cm[lane] = cm;
            W.cpre[lane] = cp;
            wave_sync();
            SCAN_MARK(1);
            SCAN_COUNT(5, nc);

            // node value of the candidate at tile offset p: next node, kLeaf|k, or kDead
            auto node_value = [&](uint32_t p, uint32_t k, int r, uint64_t plen) -> uint16_t {
                if (r == 0) return (uint16_t)(kLeaf | k);      // incomplete header at the stream end
                if (r < 0) return kDead;
                const uint64_t nxo = t0 + p + (uint64_t)r + plen;
                if (nxo >= t0 + kTile || nxo >= N) return (uint16_t)(kLeaf | k);   // leaves the tile / the stream
                const uint32_t pn = (uint32_t)(nxo - t0);
                const uint32_t m = W.cm[pn >> 5];
                const uint32_t bit = pn & 31u;
                return ((m >> bit) & 1u) ? (uint16_t)(W.cpre[pn >> 5] + (uint32_t)__popc(m & ((1u << bit) - 1u)))
                                         : kDead;
            };
            auto parse_at = [&](uint32_t p, Hdr &h) -> int {   // header window from the LDS bytes
                const uint32_t a = p & ~15u;
                const u32x4 wl = *reinterpret_cast<const u32x4 *>(B + a);
                const u32x4 wh = *reinterpret_cast<const u32x4 *>(B + a + 16u);
                return parse_window(wl, wh, p & 15u, N - (t0 + p), h);
            };

            const bool sparse = nc <= kWCap;                   // wave-uniform
            // lean parse of nodes lane, lane + 64: payload length (low 32 bits), key, and
            // packed = offset | b0 << 11 | (r + 2) << 19 | (payload length >> 32) << 24
            uint32_t pl[2], ky[2], pk[2];
            uint16_t *const pos = W.nodes;
            uint16_t *const nv = sparse ? W.nodes + kWCap : W.nodes;
            if (sparse) {
                uint32_t bits = cm, k = cp;
                while (bits) {
                    const uint32_t b = (uint32_t)__ffs(bits) - 1u;
                    bits &= bits - 1u;
                    pos[k++] = (uint16_t)(L32 + b);
                }
                wave_sync();
                // nodes lane and lane + 64: lean parse, kept in registers for the emit
#pragma unroll
                for (uint32_t j = 0; j < 2; ++j) {
                    const uint32_t k = uint32_t(lane) + 64u * j;
                    if (k < nc) {
                        const uint32_t p = pos[k];
                        const uint32_t a = p & ~15u;
                        const u32x4 wl = *reinterpret_cast<const u32x4 *>(B + a);
                        const u32x4 wh = *reinterpret_cast<const u32x4 *>(B + a + 16u);
                        uint32_t d[4];
                        window16(wl, wh, p & 15u, d);
                        uint64_t plen = 0;
                        const int r = lean_parse(d, N - (t0 + p), plen, ky[j]);
                        pl[j] = (uint32_t)plen;
                        pk[j] = p | ((d[0] & 0xFFu) << 11) | (uint32_t(r + 2) << 19) | (uint32_t(plen >> 32) << 24);
                        nv[k] = node_value(p, k, r, plen);
                    }
                }
                for (uint32_t k = lane + 128u; k < nc; k += 64) {
                    const uint32_t p = pos[k];
                    Hdr h;
                    const int r = parse_at(p, h);
                    nv[k] = node_value(p, k, r, h.plen);
                }
            } else {
                uint32_t bits = cm, k = cp;
                while (bits) {
                    const uint32_t b = (uint32_t)__ffs(bits) - 1u;
                    bits &= bits - 1u;
                    Hdr h;
                    const int r = parse_at(L32 + b, h);
                    nv[k] = node_value(L32 + b, k, r, h.plen);
                    ++k;
                }
            }
            wave_sync();
            SCAN_MARK(2);

            // pointer jumping: every chain ends at its leaf or dies
            for (;;) {
                bool ch = false;
                for (uint32_t k = lane; k < nc; k += 64) {
                    const uint16_t v = nv[k];
                    if (v < kLeaf) {
                        nv[k] = nv[v];
                        ch = true;
                    }
                }
                wave_sync();
                SCAN_COUNT(6, 1u);
                if (!__any(ch)) break;
            }
            SCAN_MARK(3);

            // survivors by node index
            for (uint32_t k0 = 0; k0 < nc; k0 += 64) {
                const uint32_t k = k0 + uint32_t(lane);
                const uint64_t m = __ballot(k < nc && nv[k] != kDead);
                if (lane == 0) {
                    W.sbits[k0 >> 6] = m;
                    W.spre[k0 >> 6] = ns;
                }
                ns += (uint32_t)__popcll(m);
            }
            if (ns > kSlots) {
                // a tile with more survivors than slots (dense small frames) spills
                if (lane == 0) spill = atomicAdd(&counters[kCntSpill], ns);
                spill = __shfl(spill, 0, 64);
                if (spill + ns > s_cap) {
                    if (lane == 0) atomicOr(&counters[kCntOverflow], 1u);
                    ns = 0;
                    spill = kNone;
                }
            }
            wave_sync();
            auto srank = [&](uint32_t k) -> uint32_t {
                return W.spre[k >> 6] + (uint32_t)__popcll(W.sbits[k >> 6] & ((1ull << (k & 63u)) - 1ull));
            };
            // survivor k with leaf v: record to its LDS slot, or to the spill area
            auto put = [&](uint32_t k, uint16_t v, const fws_frame_info &fi) {
                const uint32_t idx = srank(k), leaf = srank(v & 0x7FFFu);   // tile-local ranks
                if (spill == kNone) {
                    W.stage[idx] = fi;
                    W.stage_leaf[idx] = leaf;
                } else {
                    spill_info[spill + idx] = fi;
                    spill_leaf[spill + idx] = leaf;
                }
            };
            auto record = [&](uint32_t p, int r, uint64_t plen, uint32_t key, uint32_t b0) {
                const uint64_t q = t0 + p;
                fws_frame_info fi;
                fi.hdr_off = q;
                if (r > 0) {
                    fi.payload_len = plen;
                    fi.key = key;
                    fi.opcode = (uint8_t)(b0 & 15u);
                    fi.fin = (uint8_t)(b0 >> 7);
                    fi.hdr_len = (uint8_t)r;
                    fi.flags = (q + (uint64_t)r + plen > N) ? (uint8_t)FWS_FRAME_TRUNCATED : (uint8_t)0;
                } else {                                       // incomplete trailing header
                    fi.payload_len = 0;
                    fi.key = 0;
                    fi.opcode = 0;
                    fi.fin = 0;
                    fi.hdr_len = 0;
                    fi.flags = 0;
                }
                return fi;
            };
            auto emit = [&](uint32_t k, uint32_t p, uint16_t v) {   // re-parse from the LDS bytes
                Hdr h;
                const int r = parse_at(p, h);
                put(k, v, record(p, r, h.plen, h.key, (h.fin << 7) | h.opcode));
            };
            if (ns) {
                if (sparse) {
#pragma unroll
                    for (uint32_t j = 0; j < 2; ++j) {
                        const uint32_t k = uint32_t(lane) + 64u * j;
                        if (k < nc) {
                            const uint16_t v = nv[k];
                            if (v != kDead) {
                                const uint32_t w = pk[j];
                                put(k, v, record(w & 0x7FFu, int((w >> 19) & 31u) - 2,
                                                 (uint64_t(w >> 24) << 32) | pl[j], ky[j], (w >> 11) & 0xFFu));
                            }
                        }
                    }
                    for (uint32_t k = lane + 128u; k < nc; k += 64) {
                        const uint16_t v = nv[k];
                        if (v != kDead) emit(k, pos[k], v);
                    }
                } else {
                    uint32_t bits = cm, k = cp;
                    while (bits) {
                        const uint32_t b = (uint32_t)__ffs(bits) - 1u;
                        bits &= bits - 1u;
                        const uint16_t v = nv[k];
                        if (v != kDead) emit(k, L32 + b, v);
                        ++k;
                    }
                }
            }
            wave_sync();
            SCAN_MARK(4);
            SCAN_COUNT(7, ns);
        }
        // the tile's three stores, every lane active (idle lanes -> dummy record)
        {
            const bool rec = valid && spill == kNone && uint32_t(lane) < ns;
            const uint64_t slot = (uint64_t)t * kSlots + uint32_t(lane);
            fws_frame_info fi;
            if (rec) fi = W.stage[lane];
            fws_frame_info *di = rec ? stage_info + slot : dummy_info;
            uint32_t *dw = rec ? stage_leaf + slot : dummy_word;
            uint32_t wv = rec ? W.stage_leaf[lane] : 0u;
            if (valid && lane == 62) { dw = tile_count + t; wv = ns; }
            if (valid && lane == 63) { dw = tile_spill + t; wv = spill; }
            uint32_t *di32 = reinterpret_cast<uint32_t *>(di);
            const uint32_t *f32 = reinterpret_cast<const uint32_t *>(&fi);
            *reinterpret_cast<u32x4 *>(di32) = *reinterpret_cast<const u32x4 *>(f32);
            *reinterpret_cast<uint64_t *>(di32 + 4) = *reinterpret_cast<const uint64_t *>(f32 + 4);
            *dw = wv;
        }
        prefetch(t + 2u * GW, pf, halo);
    };

    u32x4 pa[2], pah, pb[2], pbh;
    prefetch(gw, pa, pah);
    if (kPipe) {        // same younger-op count for set A on entry as on the loop back edge
        *reinterpret_cast<u32x4 *>(dummy_info) = u32x4{0, 0, 0, 0};
        *(reinterpret_cast<uint64_t *>(dummy_info) + 2) = 0;
        *dummy_word = 0;
    }
    prefetch(gw + GW, pb, pbh);
    for (uint32_t t = gw; t < n_tiles; t += 2u * GW) {
        tile(t, pa, pah);
        tile(t + GW, pb, pbh);
    }
#ifdef FWS_SCAN_PROF
    if (lane == 0) {
        for (int i = 0; i < 8; ++i) atomicAdd(&g_scan_prof[i], (unsigned long long)prof_acc[i]);
        atomicAdd(&g_scan_prof[12], (unsigned long long)(wall_clock64() - prof_w0));
        atomicAdd(&g_scan_prof[13], (unsigned long long)(clock64() - prof_c0));
    }
#endif
}

}  // namespace fwsk

// ------------------------------------------------------------------ host side
using namespace fwsk;

#ifdef FWS_SCAN_PROF
extern "C" int fws_internal_scan_prof(unsigned long long *out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(fwsk::g_scan_prof), sizeof(unsigned long long) * 16);
    if (e == hipSuccess && reset) {
        static const unsigned long long z[16] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(fwsk::g_scan_prof), z, sizeof(z));
    }
    return fws_hip_status(e);
}
#endif

// tuning / test hook: 0 = super-tile resolve (LDS tables, big-ST path for dense super
// tiles), 1 = every super tile on the big-ST path, 2 = the RX session's small-read
// kernel first (fws_gpu_decode_stream, tests only)
static int g_resolve_mode = 0;
extern "C" __attribute__((visibility("default"))) int fws_internal_set_resolve_mode(int m) {
    const int old = g_resolve_mode;
    if (m >= 0 && m <= 2) g_resolve_mode = m;
    return old;
}
int fws_resolve_mode() { return g_resolve_mode; }

static uint32_t g_scan_blocks_per_cu = 0;   // tuning override (tools/), 0 = default
extern "C" int fws_internal_set_scan_blocks_per_cu(int v) {
    g_scan_blocks_per_cu = v > 0 ? (uint32_t)v : 0u;
    return 0;
}

int fws_decode_ensure(fws_gpu_ctx *ctx, uint64_t N, uint32_t cap) {
    fws_decode_ws &d = ctx->dec;
    const uint64_t tiles = (N + kTile - 1) / kTile + 1;
    uint64_t s_cap = N / 256 + 8 * tiles + (uint64_t)cap + 64;
    if (ctx->cap_frames + 8 * tiles > s_cap) s_cap = ctx->cap_frames + 8 * tiles;
    if (tiles <= d.max_tiles && s_cap <= d.max_surv) return 0;
    const uint64_t nt = tiles > d.max_tiles ? tiles : d.max_tiles;
    const uint64_t ns = s_cap > d.max_surv ? s_cap : d.max_surv;
    auto rel = [](auto *&p) { if (p) (void)hipFree(p); p = nullptr; };
    rel(d.tile_count); rel(d.cnt_base);
    rel(d.stage_info); rel(d.stage_leaf); rel(d.spill_info); rel(d.spill_leaf); rel(d.tile_spill);
    hipError_t e = hipSuccess;
    auto al = [&](auto **p, uint64_t bytes) { if (e == hipSuccess) e = hipMalloc((void **)p, bytes ? bytes : 16); };
    al(&d.tile_count, nt * 4);
    al(&d.cnt_base, 2 * kCntStride * 4);
    d.counters = d.cnt_base;
    d.cnt_dirty = true;
    if (d.scan_grid == 0) {
        int cus = 0;
        if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device)) != hipSuccess)
            return fws_hip_status(e);
        d.scan_grid = (uint32_t)cus * (g_scan_blocks_per_cu ? g_scan_blocks_per_cu : kScanBlocksPerCu);
    }
    if (d.scan_dummy == nullptr) al(&d.scan_dummy, (uint64_t)d.scan_grid * kScanWaves * 64u);
    al(&d.stage_info, nt * kSlots * sizeof(fws_frame_info)); al(&d.stage_leaf, nt * kSlots * 4);
    al(&d.spill_info, ns * sizeof(fws_frame_info)); al(&d.spill_leaf, ns * 4); al(&d.tile_spill, nt * 4);
    // super-tile resolve: results per slot id, EXIT tails, per-ST bases, big-ST scratch
    rel(d.nres); rel(d.tails); rel(d.gnx); rel(d.tmark); rel(d.comp); rel(d.st_nodes); rel(d.st_n); rel(d.st_entry);
    rel(d.st_fbase); rel(d.bg_nx); rel(d.bg_wt); rel(d.bg_lref); rel(d.bg_ptr); rel(d.bg_sc); rel(d.bg_mark);
    const uint64_t nst = fws_merge_super_tiles(nt);
    const uint32_t tcap = fws_merge_tail_cap(nt);
    const uint64_t nn = nt * kSlots + ns;
    al(&d.nres, nn * sizeof(fws_node_res));
    al(&d.tails, (uint64_t)tcap * sizeof(fws_tail_rec)); al(&d.gnx, (uint64_t)tcap * 4); al(&d.tmark, ((uint64_t)tcap / 32 + 1) * 4);
    al(&d.comp, (uint64_t)fws_merge_comp_cap() * 4);
    al(&d.st_nodes, fws_merge_st_nodes(nt) * sizeof(fws_st_node)); al(&d.st_n, nst * 4);
    al(&d.st_entry, nst * 4); al(&d.st_fbase, nst * 4);
    al(&d.bg_nx, nn * 4); al(&d.bg_wt, nn * 4); al(&d.bg_lref, nn * 4); al(&d.bg_ptr, 2 * nn * 4);
    al(&d.bg_sc, 2 * nn * 4); al(&d.bg_mark, nn * 4);
    if (e != hipSuccess) return fws_hip_status(e);
    d.max_tiles = nt; d.max_surv = ns;
    d.max_nodes = nn; d.max_st = nst; d.tail_cap = tcap;
    return 0;
}

int fws_launch_decode(fws_gpu_ctx *ctx, uint8_t *wire, uint64_t N, fws_frame_info *frames, uint32_t cap,
                      fws_decode_result *res, uint8_t *utf8_ok, hipStream_t s) {
    fws_decode_ws &d = ctx->dec;
    const uint32_t n_tiles = (uint32_t)((N + kTile - 1) / kTile);
    hipError_t e;
    // counters: this call's set was zeroed by the previous call's k_emit launch
    d.parity ^= 1u;
    d.counters = d.cnt_base + d.parity * kCntStride;
    uint32_t *const next = d.cnt_base + (d.parity ^ 1u) * kCntStride;
    if (d.cnt_dirty) {
        if ((e = hipMemsetAsync(d.counters, 0, kCntStride * 4, s)) != hipSuccess) return fws_hip_status(e);
        d.cnt_dirty = false;
    }
    d.cnt_dirty = true;                  // until every launch of this call is queued
    if (n_tiles) {
        const uint32_t need = (n_tiles + kScanWaves - 1) / kScanWaves;
        const uint32_t sg = need < d.scan_grid ? need : d.scan_grid;
        hipLaunchKernelGGL(N >= kTile + kHalo ? k_scan<true> : k_scan<false>, dim3(sg), dim3(kScanThreads), 0, s,
                           wire, N, n_tiles, d.stage_info, d.stage_leaf, d.spill_info, d.spill_leaf, d.tile_spill,
                           d.tile_count, d.counters, (uint32_t)d.max_surv, d.scan_dummy);
        if ((e = hipGetLastError()) != hipSuccess) return fws_hip_status(e);
    }
    // super-tile resolve; g_resolve_mode 1 sends every super tile down the big-ST
    // path (tests), mode 2 decodes as mode 0 here. Slot ids are 32-bit.
    if (N >= (1ull << 39)) return FWS_ERR_CAPACITY;
    const int r = fws_launch_merge(ctx, wire, N, n_tiles, frames, cap, res, utf8_ok, g_resolve_mode == 1, next, s);
    if (r == 0) d.cnt_dirty = false;
    return r;
}
