// decode_kernels.hip -- first half of fws_gpu_decode_stream on gfx950: the
// speculative header scan of a raw server-side wire stream. Replaces the
// serial frame loop of WSocket::OnRecvData (net/w_socket.h:543-769) for a
// device-resident buffer.
//
// Frame boundaries are a serial dependency (header i+1's offset comes from
// header i's length), so every 2 KiB tile is parsed speculatively: which
// offsets could start a header whose chain of headers reaches the tile end?
// Those are the tile's "survivors" (every true header is one; a few random
// offsets are), and merge_kernels.hip links them into the true path.
//
//  k_scan        one wavefront per tile at a time (persistent, two tiles of
//                prefetch in registers). Per tile:
//                 - candidate bits: the two-byte test (RSV clear, valid opcode,
//                   MASK set; w_socket.h:451-515) passes ~2.3 % of payload bytes;
//                 - nodes, one per lane: every candidate when there are <= 64
//                   (the common case, ~48 on random payload); else first the
//                   first hop -- a candidate with a 7-bit length whose next
//                   header offset falls inside the tile on a non-candidate byte
//                   is dead (97-98 % of them) -- and the rest ("live", <= 64);
//                 - per node: full parse (ParseFrameHdr semantics,
//                   w_socket.h:435-524), next node, pointer jumping in
//                   registers (ds_bpermute) to the chain's leaf (the last
//                   header before the tile end) or DEAD;
//                 - survivors by ballot, ranked in offset order, records stored
//                   from the lanes (8 slots per tile, a spill run past that).
//                A tile with more than 256 candidates or 64 live nodes (frames
//                under ~32 B) is marked in tile_count (kDenseTile); k_merge
//                scans it with dense_tile() (scan_common.h: every candidate a
//                node in LDS tables, no per-tile limit).
// HBM traffic: one read of the stream; records are ~1 survivor per KiB.
#include "scan_common.h"

namespace fwsk {

// FWS_ABL / FWS_ABL_NOHALO / FWS_ABL_NOSTORE: ablation builds for timing only
// (make exp; tools/scan_ablation.py), never the product library
#ifndef FWS_ABL
#define FWS_ABL 0
#endif
#ifndef FWS_SCAN_NT
#define FWS_SCAN_NT 0
#endif
constexpr bool kScanNT = FWS_SCAN_NT != 0;   // nontemporal stream loads
constexpr uint32_t kSets = 2;                // tiles in flight per wavefront (register sets; 3 sets
                                             //   at 6 waves per SIMD measured slower)
#ifndef FWS_SCAN_DMA
#define FWS_SCAN_DMA 0                           // A/B build (make exp): tiles staged by LDS-DMA
#endif
// FWS_SCAN_DMA: the next tiles land in LDS by global_load_lds_dwordx4 (two LDS
// tile buffers per wave instead of two register sets; 5.8 KB of LDS per wave,
// so 6 workgroups per CU fit, or the first-hop tables would have to shrink)
constexpr uint32_t kScanBlocksPerCu = FWS_SCAN_DMA ? 6 : 8;   // resident k_scan workgroups per CU
#ifndef FWS_SCAN_EARLY_PF
#define FWS_SCAN_EARLY_PF 0                     // A/B builds: 1 = refill a set as soon as its tile is in LDS
#endif
// 0: a register set is refilled after its tile's stores; 1: as soon as its tile
// is staged in LDS (its loads get the tile's work time too) -- measured slower
// on C2 / C3 (0.1858-0.1861 vs 0.1812-0.1815 ms, two in flight 0.171-0.173 vs
// 0.163-0.164), 1 % faster on the C5 stream (profiles/r05/ab_scan_pf.txt)
constexpr bool kEarlyPf = FWS_SCAN_EARLY_PF != 0;

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

// LDS of one k_scan wavefront
struct ScanLds {
    uint8_t bytes[kTile + kHaloX];
#if FWS_SCAN_DMA
    uint8_t bytes2[kTile + kHaloX];          // the other register set's tile (LDS-DMA)
#endif
    uint32_t cm[64];                         // candidate bits of lane L's 32 offsets
    uint32_t lm[64];                         // live bits of lane L's 32 offsets
    uint32_t lpre[64];                       // node index of lane L's first live offset (first
                                             //   candidate when every candidate is a node)
    uint16_t pos[kCandCap];                  // candidate offsets (lane-major; cand_bits32p's order in a lane)
    uint16_t lpos[kLiveCap];                 // live offsets, in offset order
};
static_assert(sizeof(ScanLds) % 16 == 0, "16-B aligned per-wave areas");

// Persistent: wavefront gw of GW walks tiles t = gw + i * GW; each of its two
// register sets holds a tile in flight, so the HBM reads of the next two tiles
// overlap the work on the current one. The 16 halo bytes (header tail past the
// tile end) come with the tile.
//
// Every tile step issues the same vector-memory sequence -- 3 stores (record
// head and tail, tile_count / tile_spill; idle lanes write the wave's dummy
// line) then 3 prefetch loads (clamped to an in-bounds tile) -- so the
// compiler's in-order vmcnt waits for a register set count the younger
// operations and never drain the other set. Only a tile with more than 8
// survivors reserves its spill run with an atomic (and waits for it).
// kPipe = false (streams shorter than one tile + halo): no prefetch.
template <bool kPipe>
__global__ __launch_bounds__(kScanThreads) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_scan(const uint8_t *__restrict__ wire, uint64_t N,
                                                       uint32_t n_tiles,
                                                       fws_frame_info *__restrict__ stage_info,
                                                       fws_frame_info *__restrict__ spill_info,
                                                       uint32_t *__restrict__ tile_spill,
                                                       uint32_t *__restrict__ tile_count,
                                                       uint32_t *__restrict__ counters, uint32_t s_cap,
                                                       uint32_t *__restrict__ scan_dummy) {
    __shared__ __attribute__((aligned(16))) ScanLds lds_w[kScanWaves];
    const uint32_t lane = threadIdx.x & 63;
    ScanLds &W = lds_w[threadIdx.x >> 6];
#if FWS_SCAN_DMA
    uint8_t *B = W.bytes;                    // the buffer of the set in hand
#else
    uint8_t *const B = W.bytes;
#endif
    // wave-uniform: readfirstlane keeps the tile index and every tile-level
    // address in SGPRs (threadIdx.x >> 6 alone is a VGPR to the compiler)
    const uint32_t gw = __builtin_amdgcn_readfirstlane(blockIdx.x * kScanWaves + (threadIdx.x >> 6));
    const uint32_t GW = gridDim.x * kScanWaves;
    const uint32_t L32 = lane * 32u;
    const uint32_t L16 = lane * 16u;
    // last tile whose bytes + halo lie inside the stream (prefetch clamp)
    const uint32_t last_inner = kPipe ? (uint32_t)((N - kHaloX) / kTile) - 1u : 0u;
    // idle lanes' stores go to this wave's own 64-B line (L2-resident, no hot spot)
    fws_frame_info *const dummy_info = reinterpret_cast<fws_frame_info *>(scan_dummy + (uint64_t)gw * 16u);
    uint32_t *const dummy_cnt = scan_dummy + (uint64_t)gw * 16u + 8u;
#ifdef FWS_SCAN_PROF
    uint64_t prof_acc[8] = {};
    uint64_t prof_t = clock64();
    const uint64_t prof_w0 = wall_clock64(), prof_c0 = prof_t;
#endif

    auto prefetch = [&](uint32_t tt, u32x4 (&pf)[2], u32x4 &halo) {
        if (!kPipe) return;
        const uint64_t o = uint64_t(tt < last_inner ? tt : last_inner) * kTile;
#if FWS_SCAN_DMA
        // into B (this set's buffer: its tile is done with it): lane L's 16 B land at
        // M0 + 16 L; three DMA instructions, the halo on lanes 0..8 only
        (void)pf;
        (void)halo;
        const uint32_t lb =
            __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t *)B);
        const uint8_t *g0 = wire + o + L16;
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g0), "s"(lb) : "memory");
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g0 + 1024u), "s"(lb + 1024u) : "memory");
        if (L16 < kHaloX)
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                         "s_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(g0 + kTile), "s"(lb + kTile) : "memory");
        return;
#endif
        // coalesced: each load instruction reads 1 KiB contiguous (lane L: 16 B at 16L)
        pf[0] = gload16<kScanNT>(reinterpret_cast<uintptr_t>(wire + o + L16));
        pf[1] = gload16<kScanNT>(reinterpret_cast<uintptr_t>(wire + o + 1024u + L16));
#if FWS_ABL_NOHALO
        halo = pf[0];
#else
        halo = gload16<kScanNT>(reinterpret_cast<uintptr_t>(wire + o + kTile + (L16 < kHaloX ? L16 : 0u)));
#endif
    };

    auto tile = [&](const uint32_t t, u32x4 (&pf)[2], u32x4 &halo) {
        const bool valid = t < n_tiles;                    // wave-uniform
        const uint64_t t0 = uint64_t(t) * kTile;
        // stream bytes from the tile start, saturated at 1 MiB (scalar): every
        // per-node bound below is then 32-bit (exits past the tile + halo are
        // leaves whatever their exact offset)
        const uint32_t rem = valid ? (N - t0 > (1u << 20) ? (1u << 20) : (uint32_t)(N - t0)) : 0u;
        uint32_t ns = 0, srank = 0, spill = kNone;
        bool rec = false;
        fws_frame_info fi;
        fi.hdr_off = 0; fi.payload_len = 0; fi.key = 0;
        fi.opcode = 0; fi.fin = 0; fi.hdr_len = 0; fi.flags = 0;
        if (valid) {
            const bool inner = kPipe && t <= last_inner;
            W.lm[lane] = 0u;
#if FWS_SCAN_DMA
            // this set's DMA into B has landed: after its three instructions came the
            // other set's step, 3 stores and 3 DMA instructions (in-order completion;
            // also before the bounds-checked path below writes B itself)
            if (kPipe) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
#endif
            if (inner) {
#if FWS_SCAN_DMA
#else
                *reinterpret_cast<u32x4 *>(B + L16) = pf[0];
                *reinterpret_cast<u32x4 *>(B + 1024u + L16) = pf[1];
                if (L16 < kHaloX) *reinterpret_cast<u32x4 *>(B + kTile + L16) = halo;
#endif
            } else {
                for (uint32_t i = lane * 16u; i < kTile + kHaloX; i += 64u * 16u) {
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
            if (kEarlyPf) prefetch(t + kSets * GW, pf, halo);   // pf is in LDS now: refill it
#if FWS_ABL == 1      // ablation (exp builds, timing only): stage the tile, nothing else
            {
                const uint32_t v = *reinterpret_cast<const uint32_t *>(B + L32);
                ns = (uint32_t)__popcll(__ballot(v == 0x12345678u));
            }
#else
            // candidate bits of this lane's 32 offsets, candidate numbering by a wave scan
            uint32_t cm;
            {
                const u32x4 w0 = *reinterpret_cast<const u32x4 *>(B + L32);
                const u32x4 w1 = *reinterpret_cast<const u32x4 *>(B + L32 + 16u);
                const uint32_t nx = *reinterpret_cast<const uint32_t *>(B + L32 + 32u);
                cm = cand_bits32p(w0, w1, nx);
                if (!inner) {
                    // bytes past the end are zero in LDS and never pass (MASK clear at
                    // the next byte); the last byte is a candidate on its own (an
                    // incomplete header, w_socket.h:443-445)
                    const uint64_t q = t0 + L32;
                    if (q < N && N - q <= 32u) cm |= 1u << cand_pbit((uint32_t)(N - q) - 1u);
                }
            }
            uint32_t nc;
            const uint32_t cp = wave_excl_scan_dpp((uint32_t)__popc(cm), &nc);
            W.cm[lane] = cm;
            bool dense = nc > kCandCap;                        // wave-uniform
            SCAN_MARK(1);
            SCAN_COUNT(5, nc);
#if FWS_ABL == 2      // ablation: candidate bits and their scan only
            ns = nc;
            dense = false;
            if (false) {
#else
            if (!dense) {
#endif
                {
                    uint32_t bits = cm, k = cp;
                    while (bits) {
                        const uint32_t b = (uint32_t)__ffs(bits) - 1u;
                        bits &= bits - 1u;
                        W.pos[k++] = (uint16_t)(L32 + cand_off(b));
                    }
                }
                // up to 64 candidates (the common case): every candidate is a node, one
                // per lane, numbered as listed (lane-major, permuted bit order within a
                // lane); else the first hop below prunes them to the live nodes first
                const bool direct = nc <= 64u;                 // wave-uniform
                if (direct) W.lpre[lane] = cp;
                wave_sync();
                uint32_t M = nc;
                if (!direct) {
                    // first hop: a candidate whose next header offset (7-bit length form,
                    // header complete) is inside the tile and fails the two-byte test is dead
                    M = 0;
                    for (uint32_t k0 = 0; k0 < nc; k0 += 64u) {
                        const uint32_t k = k0 + lane;
                        bool live = false;
                        uint32_t p = 0;
                        if (k < nc) {
                            p = W.pos[k];
                            live = true;
                            const uint32_t len7 = B[p + 1u] & 127u;
                            if (len7 < 126u && p + 6u <= rem) {
                                const uint32_t nx = p + 6u + len7;
                                if (nx < kTile && nx < rem) live = (W.cm[nx >> 5] >> cand_pbit(nx & 31u)) & 1u;
                            }
                        }
                        if (live) atomicOr(&W.lm[p >> 5], 1u << (p & 31u));
                        M += (uint32_t)__popcll(__ballot(live));
                    }
                    dense = M > kLiveCap;
                    if (!dense) {
                        // live nodes in offset order: lane L lists its own (in-order bits)
                        wave_sync();
                        uint32_t mt;
                        uint32_t lbits = W.lm[lane];
                        uint32_t li = wave_excl_scan_dpp((uint32_t)__popc(lbits), &mt);
                        W.lpre[lane] = li;
                        while (lbits) {
                            const uint32_t b = (uint32_t)__ffs(lbits) - 1u;
                            lbits &= lbits - 1u;
                            W.lpos[li++] = (uint16_t)(L32 + b);
                        }
                        wave_sync();
                    }
                }
                SCAN_MARK(2);
                SCAN_COUNT(6, M);
                if (!dense) {
                    // node `lane`: full parse, next node (lane index), leaf or dead
                    const bool act = lane < M;
                    const uint32_t p = act ? (direct ? W.pos[lane] : W.lpos[lane]) : 0u;
                    const uint32_t a = p & ~15u;
                    const u32x4 wl = *reinterpret_cast<const u32x4 *>(B + a);
                    const u32x4 wh = *reinterpret_cast<const u32x4 *>(B + a + 16u);
                    uint32_t d[4];
                    window16(wl, wh, p & 15u, d);
                    uint64_t plen = 0;
                    uint32_t key = 0;
                    const int r = act ? lean_parse(d, rem - p, plen, key) : -1;   // (p < rem)
                    uint32_t ptr = kDeadLane;
                    if (r == 0) {
                        ptr = lane;                            // incomplete header at the stream end
                    } else if (r > 0) {
                        // the exit, tile-relative, with the length saturated at 64 KiB
                        const uint32_t hx = p + (uint32_t)r + (plen > 0xFFFFu ? 0x10000u : (uint32_t)plen);
                        if (hx >= kTile || hx >= rem) {
                            ptr = lane;                        // leaves the tile / the stream
                            // unless its exit, in the halo, is no header
                            if (hx + 2u <= rem && hx + 1u < kTile + kHaloX) {
                                const uint32_t e0 = B[hx], e1 = B[hx + 1u];
                                if ((e0 & 0x77u) > 2u || !(e1 & 0x80u)) ptr = kDeadLane;
                            }
                        } else {
                            // the node at the exit: a candidate (direct) or live bit, ranked
                            const uint32_t nx = hx;
                            const uint32_t m = direct ? W.cm[nx >> 5] : W.lm[nx >> 5];
                            const uint32_t bit = direct ? cand_pbit(nx & 31u) : nx & 31u;
                            if ((m >> bit) & 1u) ptr = W.lpre[nx >> 5] + (uint32_t)__popc(m & ((1u << bit) - 1u));
                        }
                    }
                    // pointer jumping in registers: every chain ends at its leaf (a
                    // lane pointing at itself) or dies
                    for (;;) {
                        const uint32_t q = lane_read(ptr, ptr < 64u ? ptr : lane);
                        const uint32_t np = ptr < 64u ? q : ptr;
                        const bool ch = np != ptr;
                        ptr = np;
                        SCAN_COUNT(7, 1u);
                        if (!__any(ch)) break;
                    }
                    // survivors and their ranks in offset order (lane order for live
                    // nodes; direct nodes are permuted within a 32-byte block: count)
                    const bool surv = act && ptr < 64u;
                    const uint64_t sm = __ballot(surv);
                    ns = (uint32_t)__popcll(sm);
                    if (direct) {
                        srank = 0;
                        for (uint64_t mm = sm; mm; mm &= mm - 1u) {
                            const uint32_t pq = (uint32_t)__builtin_amdgcn_readlane((int)p, (int)__builtin_ctzll(mm));
                            srank += pq < p ? 1u : 0u;
                        }
                    } else {
                        srank = mbcnt64(sm);
                    }
                    if (ns > kSlots) {
                        // more survivors than slots (frames under ~250 B): a spill run
                        if (lane == 0) {
                            const uint32_t rs = spill_region_size(s_cap), rg = gw % kSpillRegions;
                            const uint32_t off = atomicAdd(&counters[kCntRegion0 + rg * kRegionStride], ns);
                            spill = (off <= rs && rs - off >= ns) ? rg * rs + off : spill_shared(counters, s_cap, ns);
                        }
                        spill = __shfl(spill, 0, 64);
                        if (spill == kNone) ns = 0;
                    }
                    rec = surv && ns != 0;
                    fi.hdr_off = t0 + p;
                    if (r > 0) {
                        const uint32_t b0 = d[0] & 0xFFu;
                        fi.payload_len = plen;
                        fi.key = key;
                        fi.opcode = (uint8_t)(b0 & 15u);
                        fi.fin = (uint8_t)(b0 >> 7);
                        fi.hdr_len = (uint8_t)r;
                        fi.flags = (p + (uint64_t)r + plen > N - t0) ? (uint8_t)FWS_FRAME_TRUNCATED : (uint8_t)0;
                    }
                }
            }
            if (dense) {
                // left to dense_tile() in k_merge (frames under ~32 B)
                ns = kDenseTile;
                rec = false;
                if (lane == 0) atomicAdd(&counters[kCntScanDense], 1u);
            }
#endif
            SCAN_MARK(3);
        }
        // the tile's three stores, every lane active (idle lanes -> the dummy line)
#if FWS_ABL_NOSTORE
        if (ns == 0x7FFFFFFFu)
#endif
        {
            fws_frame_info *di = !rec ? dummy_info
                                      : spill == kNone ? stage_info + (uint64_t)t * kSlots + srank
                                                       : spill_info + (uint64_t)spill + srank;
            uint32_t *dc = dummy_cnt;
            uint32_t cv = 0;
            if (valid && lane == 0) { dc = tile_count + t; cv = ns; }
            if (valid && lane == 1) { dc = tile_spill + t; cv = spill; }
            uint32_t *di32 = reinterpret_cast<uint32_t *>(di);
            const uint32_t *f32 = reinterpret_cast<const uint32_t *>(&fi);
            *reinterpret_cast<u32x4 *>(di32) = *reinterpret_cast<const u32x4 *>(f32);
            *reinterpret_cast<uint64_t *>(di32 + 4) = *reinterpret_cast<const uint64_t *>(f32 + 4);
            *dc = cv;
        }
        if (!kEarlyPf || !valid) prefetch(t + kSets * GW, pf, halo);
    };

    auto dummy_stores = [&]() {   // same younger-op count for a set on entry as on the loop back edge
        if (!kPipe) return;
        asm volatile("" ::: "memory");             // keep the four stores between two prefetches
        *reinterpret_cast<u32x4 *>(dummy_info) = u32x4{0, 0, 0, 0};
        *(reinterpret_cast<uint64_t *>(dummy_info) + 2) = 0;
        *dummy_cnt = 0;
        asm volatile("" ::: "memory");
    };
    u32x4 pa[2], pah, pb[2], pbh;
#if FWS_SCAN_DMA
    B = W.bytes;
    prefetch(gw, pa, pah);
    dummy_stores();
    B = W.bytes2;
    prefetch(gw + GW, pb, pbh);
    for (uint32_t t = gw; t < n_tiles; t += 2u * GW) {
        B = W.bytes;
        tile(t, pa, pah);
        B = W.bytes2;
        tile(t + GW, pb, pbh);
    }
#else
    prefetch(gw, pa, pah);
    dummy_stores();
    prefetch(gw + GW, pb, pbh);
    for (uint32_t t = gw; t < n_tiles; t += 2u * GW) {
        tile(t, pa, pah);
        tile(t + GW, pb, pbh);
    }
#endif
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

// timing hook (tools/scan_ablation.py): k_scan alone over a device stream
extern "C" __attribute__((visibility("default"))) int fws_internal_scan_only(fws_gpu_ctx *ctx, const uint8_t *wire,
                                                                         uint64_t N, hipStream_t s) {
    fws_decode_ws &d = ctx->dec;
    const int r = fws_decode_ensure(ctx, N, 16);
    if (r) return r;
    const uint32_t n_tiles = (uint32_t)((N + kTile - 1) / kTile);
    if (!n_tiles || N < kTile + kHaloX) return FWS_ERR_INVALID;
    const uint32_t need = (n_tiles + kScanWaves - 1) / kScanWaves;
    const uint32_t sg = need < d.scan_grid ? need : d.scan_grid;
    // its own zeroed counter set (set 0) every call, so the spill offsets and
    // kCntScanDense start clean; the next decode zeroes the set it uses
    hipError_t e = hipMemsetAsync(d.cnt_base, 0, kCntStride * 4, s);
    if (e != hipSuccess) return fws_hip_status(e);
    d.cnt_dirty = true;
    hipLaunchKernelGGL(k_scan<true>, dim3(sg), dim3(kScanThreads), 0, s, wire, N, n_tiles, d.stage_info, d.spill_info,
                       d.tile_spill, d.tile_count, d.cnt_base, (uint32_t)d.max_surv, d.scan_dummy);
    return fws_hip_status(hipGetLastError());
}

int fws_decode_ensure(fws_gpu_ctx *ctx, uint64_t N, uint32_t cap) {
    fws_decode_ws &d = ctx->dec;
    const uint64_t tiles = (N + kTile - 1) / kTile + 1;
    // spill capacity: every frame a survivor twice over (half of it is split in
    // kSpillRegions regions, decode_common.h), plus random survivors
    uint64_t s_cap = N / 256 + 8 * tiles + 2 * (uint64_t)cap + 64;
    if (2 * ctx->cap_frames + 8 * tiles > s_cap) s_cap = 2 * ctx->cap_frames + 8 * tiles;
    if (s_cap > 0xF0000000ull) s_cap = 0xF0000000ull;   // 32-bit slot ids
    if (tiles <= d.max_tiles && s_cap <= d.max_surv) return 0;
    const uint64_t nt = tiles > d.max_tiles ? tiles : d.max_tiles;
    const uint64_t ns = s_cap > d.max_surv ? s_cap : d.max_surv;
    auto rel = [](auto *&p) { if (p) (void)hipFree(p); p = nullptr; };
    rel(d.tile_count); rel(d.cnt_base);
    rel(d.stage_info); rel(d.spill_info); rel(d.tile_spill);
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
    al(&d.stage_info, nt * kSlots * sizeof(fws_frame_info));
    al(&d.spill_info, ns * sizeof(fws_frame_info)); al(&d.tile_spill, nt * 4);
    // super-tile resolve: results per slot id, EXIT tails, per-ST bases, big-ST scratch
    rel(d.nres); rel(d.tails); rel(d.gnx); rel(d.tpk); rel(d.tmark); rel(d.comp); rel(d.st_nodes); rel(d.st_n); rel(d.st_nt); rel(d.st_entry);
    rel(d.st_fbase); rel(d.bg_nx); rel(d.bg_wt); rel(d.bg_lref); rel(d.bg_ptr); rel(d.bg_sc); rel(d.bg_mark);
    const uint64_t nst = fws_merge_super_tiles_cap(nt);
    const uint32_t tcap = fws_merge_tail_cap(nt);
    const uint64_t nn = nt * kSlots + ns;
    al(&d.nres, nn * sizeof(fws_node_res));
    al(&d.tails, (uint64_t)tcap * sizeof(fws_tail_rec)); al(&d.gnx, (uint64_t)tcap * 4); al(&d.tpk, (uint64_t)tcap * 16); al(&d.tmark, ((uint64_t)tcap / 32 + 1) * 4);
    al(&d.comp, (uint64_t)fws_merge_comp_cap() * 4);
    al(&d.st_nodes, fws_merge_st_nodes(nt) * sizeof(fws_st_node)); al(&d.st_n, nst * 4); al(&d.st_nt, nst * 4);
    al(&d.st_entry, nst * 4); al(&d.st_fbase, nst * 4);
    al(&d.bg_nx, nn * 4); al(&d.bg_wt, nn * 4); al(&d.bg_lref, nn * 4); al(&d.bg_ptr, 2 * nn * 4);
    al(&d.bg_sc, 2 * nn * 4); al(&d.bg_mark, nn * 4);
    if (e != hipSuccess) return fws_hip_status(e);
    d.max_tiles = nt; d.max_surv = ns;
    d.max_nodes = nn; d.max_st = nst; d.tail_cap = tcap;
    return 0;
}

// The decode's first half: this call's counter set (zeroed by the previous
// call's k_emit, or here when a call did not finish its launches) and k_scan.
int fws_launch_decode_scan(fws_gpu_ctx *ctx, uint8_t *wire, uint64_t N, hipStream_t s) {
    fws_decode_ws &d = ctx->dec;
    const uint32_t n_tiles = (uint32_t)((N + kTile - 1) / kTile);
    hipError_t e;
    d.parity ^= 1u;
    d.counters = d.cnt_base + d.parity * kCntStride;
    if (d.cnt_dirty) {
        if ((e = hipMemsetAsync(d.counters, 0, kCntStride * 4, s)) != hipSuccess) return fws_hip_status(e);
        d.cnt_dirty = false;
    }
    d.cnt_dirty = true;                  // until every launch of this call is queued
    if (n_tiles) {
        const uint32_t need = (n_tiles + kScanWaves - 1) / kScanWaves;
        const uint32_t sg = need < d.scan_grid ? need : d.scan_grid;
        hipLaunchKernelGGL(N >= kTile + kHaloX ? k_scan<true> : k_scan<false>, dim3(sg), dim3(kScanThreads), 0, s,
                           wire, N, n_tiles, d.stage_info, d.spill_info, d.tile_spill, d.tile_count, d.counters,
                           (uint32_t)d.max_surv, d.scan_dummy);
        if ((e = hipGetLastError()) != hipSuccess) return fws_hip_status(e);
    }
    return 0;
}

// The second half, on the counter set the scan used (k_emit zeroes the other
// set for the context's next call): the super-tile resolve. g_resolve_mode 1
// sends every super tile down the big-ST path (tests), mode 2 decodes as mode 0
// here. Slot ids are 32-bit.
int fws_launch_decode_resolve(fws_gpu_ctx *ctx, uint8_t *wire, uint64_t N, fws_frame_info *frames, uint32_t cap,
                              fws_decode_result *res, uint8_t *utf8_ok, hipStream_t s) {
    fws_decode_ws &d = ctx->dec;
    const uint32_t n_tiles = (uint32_t)((N + kTile - 1) / kTile);
    uint32_t *const next = d.cnt_base + (d.parity ^ 1u) * kCntStride;
    if (N >= (1ull << 39)) return FWS_ERR_CAPACITY;
    const int r = fws_launch_merge(ctx, wire, N, n_tiles, frames, cap, res, utf8_ok, g_resolve_mode == 1, next, s);
    if (r == 0) d.cnt_dirty = false;
    return r;
}

int fws_launch_decode(fws_gpu_ctx *ctx, uint8_t *wire, uint64_t N, fws_frame_info *frames, uint32_t cap,
                      fws_decode_result *res, uint8_t *utf8_ok, hipStream_t s) {
    const int r = fws_launch_decode_scan(ctx, wire, N, s);
    return r ? r : fws_launch_decode_resolve(ctx, wire, N, frames, cap, res, utf8_ok, s);
}
