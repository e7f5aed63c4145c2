// stream_kernels.hip -- one-launch fws_gpu_decode_stream on gfx950: the header
// scan, the chain resolve, the frame list and the unmask of a server-side wire
// stream in ONE persistent launch. Replaces the serial frame loop of
// WSocket::OnRecvData (net/w_socket.h:543-769: ParseFrameHdr :435-524, the
// unmask WSMaskBytesFast at :586 / :614, the key rotation of a continuing frame
// :750-764) for a device-resident buffer. The multi-launch path
// (decode_kernels.hip + merge_kernels.hip + k_unmask_stream) stays as its
// fallback and runs only where this kernel declines.
//
// Why one launch: the multi-launch path is a scan (VALU-bound, ~4 TB/s of
// reads), three latency-bound resolve launches, then the unmask (HBM-bound);
// each phase idles the resource the next one needs. Here every workgroup holds
// two SCANNER wavefronts and two UNMASKER wavefronts, paired: a scanner parses
// a 32 KiB super tile (ST) while its partner resolves and unmasks the ST the
// scanner finished before, so every CU runs VALU-heavy parsing beside
// HBM-heavy unmasking, and the resolve is a per-ST handshake through
// epoch-tagged 8-B granules instead of launches.
//
// Per ST k (tickets in stream order):
//  scanner   the 16 tiles of 2 KiB (k_scan's tile body, scan_common.h), then
//            the in-ST link: each survivor's chain in the ST ends at a tail that
//            EXITs the ST, reaches the stream END, is an incomplete header (INC)
//            or is DEAD (its exit is no header); pointer jumping in LDS gives
//            each survivor its tail and the frames up to it. Publishes P_k = the
//            distinct exits of the EXIT tails (usually one: the true chain's).
//  unmasker  (1) guess the entry E_k from P_{k-1}: the one exit of ST k-1 that
//            lands on a live survivor of k (or, landing on none, the one exit that
//            passes over k); publish C_k = {exit of E_k's chain, its frames, its
//            last header} -- C_k depends on P_{k-1} only, so no chain of waits
//            runs through the STs; (2) verify: E_k must be C_{k-1}'s exit; by
//            induction from offset 0 a verified prefix is the true chain;
//            (3) decoupled look-back over (verified, frames) aggregates: the
//            frame base of ST k and the proof that every ST before it verified;
//            (4) the frame records and the unmask of the ST's 32 KiB, re-read
//            from HBM, 16-B chunks, key phase from each payload's start.
// Anything it cannot finish exactly (a tile with more than 16 survivors or 256
// candidates, more than 128 survivors or 8 exits in an ST, an ambiguous entry
// whose predecessor failed, a verification mismatch -- a protocol error on the
// true chain makes one --, more frames than `cap`, a wait that gave up) marks
// the ST failed: the look-back then fails every later ST, and the multi-launch
// path (launched after, gated on kCntFFail) decodes the whole stream again and
// unmasks the STs not marked done (headers are never modified, so it sees the
// same chain).
//
// Handed-off words are 8-B granules {tag = call epoch, 40-bit value} written
// with relaxed agent-scope atomics (sc1) and polled with sc1 loads
// (MI355X_MICROARCH.md "Valid forms", R2 granules): nothing is zeroed per call.
// Every wait is on a lower ticket (held by a running wavefront) and bounded.
#include "scan_common.h"

namespace fwsk {

constexpr uint32_t kXS = kFusedStBytes;                     // 32 KiB super tile
constexpr uint32_t kXTiles = kXS / kTile;                   // 16
constexpr uint32_t kXPairs = 2;                             // scanner / unmasker pairs per workgroup
constexpr uint32_t kXThreads = 2 * kXPairs * 64;
constexpr uint32_t kXBlocksPerCu = 6;                      // 80 VGPRs: 6 waves per SIMD
constexpr uint32_t kXTileCap = 16;                          // survivors per tile
constexpr uint32_t kXCap = 128;                             // survivors per ST
constexpr uint32_t kXExCap = 8;                             // distinct EXIT exits per ST
constexpr uint32_t kXFar = 0xFFFFFFFFu;                     // ST-relative exit past 4 GiB
constexpr uint8_t kXLeaf = 0xFF;                            // lk: the chain leaves the tile
constexpr uint8_t kXTerm = 0xFE;                            // lk: a tail (after the in-ST link)
constexpr uint32_t kXSpin = 1u << 15;                       // bounded waits (polls ~1-2 us apart)
enum : uint8_t { kKExit = 0, kKEnd = 1, kKInc = 2, kKDead = 3, kKNone = 4 };

// granule regions (SoA over STs), then kXExCap exit words per ST
enum XRegion : uint32_t {
    kQP = 0,         // P_k: distinct exits published (kXExCap + 1: failed)
    kQCX = 1,        // C_k: the exit of E_k's chain (the next entry), or kVFail
    kQCN = 2,        //      frames of E_k's chain in the ST
    kQCT = 3,        //      header of the last frame up to that exit (kNoTail: none)
    kQA = 4,         // A_k: frames of the ST when verified, else kVFail
    kQI = 5,         // I_k: frames up to and including the ST when the prefix verified, else kVFail
    kQDone = 6,      // the ST's bytes were unmasked here (fws_launch_unmask_stream skips them)
    kXRegions = 7
};
constexpr uint32_t kXPubWords = kXRegions + kXExCap;
constexpr uint64_t kV40 = (1ull << 40) - 1;
constexpr uint64_t kVFail = kV40;
constexpr uint64_t kNoTail = kV40 - 1;

__device__ __forceinline__ uint64_t gr(uint32_t tag, uint64_t v) { return ((uint64_t)tag << 40) | (v & kV40); }
__device__ __forceinline__ bool gok(uint64_t g, uint32_t tag) { return (uint32_t)(g >> 40) == tag; }
__device__ __forceinline__ uint64_t gval(uint64_t g) { return g & kV40; }
__device__ __forceinline__ void gput(uint64_t *p, uint64_t g) {
    __hip_atomic_store(p, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t gget(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t cget(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
// a wave-uniform 64-bit value into SGPRs
__device__ __forceinline__ uint64_t rfl64(uint64_t v) { return ((uint64_t)rfl((uint32_t)(v >> 32)) << 32) | rfl((uint32_t)v); }

struct XParams {
    uint8_t *wire;
    uint64_t N;
    uint32_t n_st;
    uint32_t tag;                                   // call epoch, 1..2^24-1
    fws_frame_info *frames;
    uint32_t cap;
    fws_decode_result *res;
    uint32_t *C;                                    // the call's counter set (decode_common.h)
    uint64_t *pub;
    uint64_t stride;                                // fmax_st
    uint64_t *trace;                                // test hook: per-ST clocks (kXTraceW words), or null

    __device__ __forceinline__ uint64_t *R(uint32_t r) const { return pub + (uint64_t)r * stride; }
    __device__ __forceinline__ uint64_t *ex(uint32_t k) const {
        return pub + (uint64_t)kXRegions * stride + (uint64_t)k * kXExCap;
    }
    __device__ __forceinline__ uint64_t end_of(uint64_t k) const {
        const uint64_t e = (k + 1) * kXS;
        return e < N ? e : N;
    }
    // an ST before k has failed (kCntFFail holds ~(first failing ST))
    __device__ __forceinline__ bool failed_before(uint32_t k) const {
        const uint32_t f = rfl(cget(&C[kCntFFail]));
        return f != 0u && ~f < k;
    }
    // every granule of ST k failed (scanner-side failure or a skipped ST)
    __device__ __forceinline__ void fail_all(uint32_t k) const {
        gput(R(kQP) + k, gr(tag, kXExCap + 1u));
        gput(R(kQCX) + k, gr(tag, kVFail));
        gput(R(kQA) + k, gr(tag, kVFail));
        gput(R(kQI) + k, gr(tag, kVFail));
        atomicMax(&C[kCntFFail], ~k);
    }
};

// FWS_STREAM_TRACE builds (make -C flashws_amd/csrc prof; tools/prof_stream.py):
// trace[k * kXTraceW + i] = wall clock (100 MHz) at
// 0 scan start, 1 scan end, 2 P published, 3 unmasker start, 4 C published,
// 5 verified, 6 look-back done, 7 unmask end; 8 look-back window, 9 spins
constexpr uint32_t kXTraceW = 10;
#ifdef FWS_STREAM_TRACE
#define XT(k, i, v) do { if (P.trace && lane == 0) P.trace[(uint64_t)(k) * kXTraceW + (i)] = (v); } while (0)
#else
#define XT(k, i, v) do { } while (0)
#endif

// one ST's survivors, slot order = offset order (tiles in order, ranks by offset)
struct XTable {
    uint16_t off[kXCap];                            // ST-relative header offset
    uint8_t hl[kXCap];                              // header length; 0: incomplete header at the stream end
    uint8_t lk[kXCap];                              // next survivor on the chain, kXLeaf / kXTerm
    uint32_t xo[kXCap];                             // own frame's exit, ST-relative (kXFar: past 4 GiB)
    uint32_t pw[kXCap];                             // tail slot | frames before it << 8 (after jumping)
    uint8_t kind[kXCap];                            // how a tail ends (kKExit .. kKDead)
    uint32_t n;                                     // survivors
    uint32_t k;                                     // the ST
    uint32_t state;                                 // 0 empty, 1 full, 2 the scanner is done
};
// one scanner wavefront's tile scratch (k_scan's ScanLds)
struct XScanW {
    uint8_t bytes[kTile + kHaloX];
    uint32_t cm[64];
    uint32_t lm[64];
    uint32_t lpre[64];
    uint16_t pos[kCandCap];
    uint16_t lpos[kLiveCap];
};
// one unmasker wavefront's scratch: the chain's slots, the ST's payload regions
struct XUnW {
    uint8_t list[kXCap];
    uint32_t lo[kXCap + 1];                         // region [lo, hi) ST-relative, key rotated
    uint32_t hi[kXCap + 1];                         //   for 4-aligned ST-relative offsets
    uint32_t rk[kXCap + 1];
};
struct XLds {
    XTable tab[kXPairs][2];
    XScanW sw[kXPairs];
    XUnW uw[kXPairs];
};
static_assert(sizeof(XScanW) % 16 == 0, "16-B aligned tile bytes");

// survivor slot at ST-relative offset o, or kXCap (binary search over the sorted offsets)
__device__ __forceinline__ uint32_t x_lookup(const XTable &T, uint32_t n, uint32_t o) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (T.off[mid] < o) lo = mid + 1u; else hi = mid;
    }
    return (lo < n && T.off[lo] == o) ? lo : kXCap;
}

// Tile t of ST st0 by one wavefront: k_scan's tile body (decode_kernels.hip),
// the survivors appended to T in offset order with their in-tile next survivor.
// pf / halo hold the tile's bytes when `inner` (else staged bytewise). Returns
// true (wave-uniform) when the tile is too dense for this path.
__device__ __forceinline__ bool x_scan_tile(XScanW &W, XTable &T, const uint8_t *__restrict__ wire, uint64_t N, uint64_t st0,
                            uint32_t t, bool inner, const u32x4 (&pf)[2], const u32x4 &halo) {
    const uint32_t lane = threadIdx.x & 63;
    uint8_t *const B = W.bytes;
    const uint64_t t0 = st0 + (uint64_t)t * kTile;
    if (t0 >= N) return false;
    const uint32_t L32 = lane * 32u, L16 = lane * 16u;
    W.lm[lane] = 0u;
    if (inner) {
        *reinterpret_cast<u32x4 *>(B + L16) = pf[0];
        *reinterpret_cast<u32x4 *>(B + 1024u + L16) = pf[1];
        if (L16 < kHaloX) *reinterpret_cast<u32x4 *>(B + kTile + L16) = halo;
    } else {
        for (uint32_t i = L16; i < kTile + kHaloX; i += 64u * 16u) {
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
    uint32_t cm;
    {
        const u32x4 w0 = *reinterpret_cast<const u32x4 *>(B + L32);
        const u32x4 w1 = *reinterpret_cast<const u32x4 *>(B + L32 + 16u);
        const uint32_t nx = *reinterpret_cast<const uint32_t *>(B + L32 + 32u);
        cm = cand_bits32p(w0, w1, nx);
        if (!inner) {
            // bytes past the end are zero in LDS and never pass; the last byte is a
            // candidate on its own (an incomplete header, w_socket.h:443-445)
            const uint64_t q = t0 + L32;
            if (q < N && N - q <= 32u) cm |= 1u << cand_pbit((uint32_t)(N - q) - 1u);
        }
    }
    uint32_t nc;
    const uint32_t cp = wave_excl_scan_dpp((uint32_t)__popc(cm), &nc);
    W.cm[lane] = cm;
    if (nc > kCandCap) return true;
    {
        uint32_t bits = cm, k = cp;
        while (bits) {
            const uint32_t b = (uint32_t)__ffs(bits) - 1u;
            bits &= bits - 1u;
            W.pos[k++] = (uint16_t)(L32 + cand_off(b));
        }
    }
    const bool direct = nc <= 64u;
    if (direct) W.lpre[lane] = cp;
    wave_sync();
    uint32_t M = nc;
    if (!direct) {
        // first hop: a candidate whose next header offset (7-bit length form, header
        // complete) is inside the tile and fails the two-byte test is dead
        M = 0;
        for (uint32_t k0 = 0; k0 < nc; k0 += 64u) {
            const uint32_t k = k0 + lane;
            bool live = false;
            uint32_t p = 0;
            if (k < nc) {
                p = W.pos[k];
                live = true;
                const uint32_t len7 = B[p + 1u] & 127u;
                if (len7 < 126u && t0 + p + 6u <= N) {
                    const uint32_t nx = p + 6u + len7;
                    if (nx < kTile && t0 + nx < N) live = (W.cm[nx >> 5] >> cand_pbit(nx & 31u)) & 1u;
                }
            }
            if (live) atomicOr(&W.lm[p >> 5], 1u << (p & 31u));
            M += (uint32_t)__popcll(__ballot(live));
        }
        if (M > kLiveCap) return true;
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
    // node `lane`: full parse, next node (lane index), leaf or dead
    const bool act = lane < M;
    const uint32_t p = act ? (direct ? W.pos[lane] : W.lpos[lane]) : 0u;
    const uint32_t a = p & ~15u;
    uint32_t d[4];
    window16(*reinterpret_cast<const u32x4 *>(B + a), *reinterpret_cast<const u32x4 *>(B + a + 16u), p & 15u, d);
    uint64_t plen = 0;
    uint32_t key = 0;
    const int r = act ? lean_parse(d, N - (t0 + p), plen, key) : -1;
    uint32_t ptr = kDeadLane;
    if (r == 0) {
        ptr = lane;                                  // incomplete header at the stream end
    } else if (r > 0) {
        const uint64_t nxo = t0 + p + (uint64_t)r + plen;
        if (nxo >= t0 + kTile || nxo >= N) {
            ptr = lane;                              // leaves the tile / the stream
            const uint64_t hx = nxo - t0;            // unless its exit, in the halo, is no header
            if (nxo + 2u <= N && hx + 1u < kTile + kHaloX) {
                const uint32_t e0 = B[hx], e1 = B[hx + 1u];
                if ((e0 & 0x77u) > 2u || !(e1 & 0x80u)) ptr = kDeadLane;
            }
        } else {
            const uint32_t nx = (uint32_t)(nxo - t0);
            const uint32_t m = direct ? W.cm[nx >> 5] : W.lm[nx >> 5];
            const uint32_t bit = direct ? cand_pbit(nx & 31u) : nx & 31u;
            if ((m >> bit) & 1u) ptr = W.lpre[nx >> 5] + (uint32_t)__popc(m & ((1u << bit) - 1u));
        }
    }
    const uint32_t ptr0 = ptr;
    for (;;) {                                       // pointer jumping: leaf or dead
        const uint32_t q = lane_read(ptr, ptr < 64u ? ptr : lane);
        const uint32_t np = ptr < 64u ? q : ptr;
        const bool ch = np != ptr;
        ptr = np;
        if (!__any(ch)) break;
    }
    const bool surv = act && ptr < 64u;
    const uint64_t sm = __ballot(surv);
    const uint32_t ns = (uint32_t)__popcll(sm);
    const uint32_t base = T.n;
    if (ns > kXTileCap || base + ns > kXCap) return true;
    uint32_t srank;
    if (direct) {
        srank = 0;
        for (uint64_t mm = sm; mm; mm &= mm - 1u) {
            const uint32_t pq = (uint32_t)__builtin_amdgcn_readlane((int)p, (int)__builtin_ctzll(mm));
            srank += pq < p ? 1u : 0u;
        }
    } else {
        srank = mbcnt64(sm);
    }
    const uint32_t slot = base + srank;
    // a survivor's next node survives too: its slot is the next survivor on the chain
    const uint32_t nslot = lane_read(slot, ptr0 < 64u ? ptr0 : lane);
    if (surv) {
        const uint32_t o = t * kTile + p;
        T.off[slot] = (uint16_t)o;
        T.hl[slot] = (uint8_t)(r > 0 ? r : 0);
        T.lk[slot] = ptr0 == lane ? kXLeaf : (uint8_t)nslot;
        const uint64_t x = r > 0 ? (uint64_t)o + (uint64_t)r + plen : (uint64_t)o;
        T.xo[slot] = x >= kXFar ? kXFar : (uint32_t)x;
    }
    wave_sync();
    if (lane == 0) T.n = base + ns;
    wave_sync();
    return false;
}

// The scanner wavefront of pair `pr`: tickets in stream order, 16 tiles each
// (two tiles of loads in flight), the in-ST link, P_k, the table to the partner.
__device__ __forceinline__ void x_scanner(const XParams &P, XLds &S, uint32_t pr) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t N = P.N;
    const uint32_t tag = P.tag;
    const uintptr_t wb = reinterpret_cast<uintptr_t>(P.wire);
    uint32_t *const C = P.C;
    XScanW &W = S.sw[pr];
    uint32_t buf = 0;
    for (;;) {
        uint32_t k = 0;
        if (lane == 0) k = atomicAdd(&C[kCntFTicket], 1u);
        k = rfl(k);
        XTable &T = S.tab[pr][buf];
        // the partner frees the buffer (it holds at most one ST of ours besides this one)
        while (__hip_atomic_load(&T.state, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u)
            __builtin_amdgcn_s_sleep(2);
        if (k >= P.n_st) {
            if (lane == 0) __hip_atomic_store(&T.state, 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            return;
        }
        if (P.failed_before(k)) {
            if (lane == 0) P.fail_all(k);
            continue;
        }
        XT(k, 0, wall_clock64());
        const uint64_t st0 = (uint64_t)k * kXS;
        const uint64_t stE = P.end_of(k);
        const uint32_t len = (uint32_t)(stE - st0);
        if (lane == 0) T.n = 0;
        wave_sync();
        // tiles whose bytes + halo lie inside the stream come through registers
        const uint64_t last_inner = N >= kTile + kHaloX ? (N - kHaloX) / kTile - 1u : ~0ull;
        auto inner_tile = [&](uint32_t t) { return last_inner != ~0ull && st0 / kTile + t <= last_inner; };
        auto prefetch = [&](uint32_t t, u32x4 (&pf)[2], u32x4 &halo) {
            const uint64_t o = st0 + (uint64_t)(t < kXTiles ? t : kXTiles - 1u) * kTile;
            if (t >= kXTiles || !inner_tile(t)) return;
            pf[0] = gload16(wb + o + lane * 16u);
            pf[1] = gload16(wb + o + 1024u + lane * 16u);
            halo = gload16(wb + o + kTile + (lane * 16u < kHaloX ? lane * 16u : 0u));
        };
        // one tile of loads in flight per scanner (the unmaskers beside it keep most
        // of the CU's HBM requests in flight)
        u32x4 pa[2], pah;
        prefetch(0, pa, pah);
        bool bad = false;
        for (uint32_t t = 0; t < kXTiles && !bad; ++t) {
            const bool in = inner_tile(t);
            u32x4 cur[2] = {pa[0], pa[1]}, ch = pah;
            prefetch(t + 1, pa, pah);
            bad = x_scan_tile(W, T, P.wire, N, st0, t, in, cur, ch);
        }
        XT(k, 1, wall_clock64());
        const uint32_t n = T.n;
        // the in-ST link: a tile leaf's exit lands on a survivor of a later tile, or the
        // chain ends here (EXIT the ST, the stream END, INC, DEAD)
        bool far_bad = false;
        for (uint32_t s = lane; s < n && !bad; s += 64u) {
            uint8_t kd = kKNone;
            uint32_t pw;
            if (T.hl[s] == 0) {
                kd = kKInc;
            } else if (T.lk[s] == kXLeaf) {
                const uint32_t x = T.xo[s];
                if (x == kXFar) {
                    if (st0 + kXFar < N) far_bad = true;   // an exit past 4 GiB inside the stream
                    kd = kKEnd;
                } else if (st0 + x >= N) {
                    kd = kKEnd;
                } else if (x >= len) {
                    kd = kKExit;
                } else {
                    const uint32_t u = x_lookup(T, n, x);
                    if (u < kXCap) T.lk[s] = (uint8_t)u;
                    else kd = kKDead;
                }
            }
            if (kd != kKNone) {
                T.lk[s] = kXTerm;
                pw = s;
            } else {
                pw = (uint32_t)T.lk[s] | (1u << 8);
            }
            T.kind[s] = kd;
            T.pw[s] = pw;
        }
        bad = bad || __any(far_bad);
        wave_sync();
        if (!bad) {
            for (;;) {                               // pointer jumping in place
                bool ch = false;
                for (uint32_t s = lane; s < n; s += 64u) {
                    const uint32_t w = T.pw[s], q = w & 0xFFu;
                    if (q == s) continue;
                    const uint32_t w2 = T.pw[q], q2 = w2 & 0xFFu;
                    if (q2 == q) continue;
                    T.pw[s] = q2 | (((w >> 8) + (w2 >> 8)) << 8);
                    ch = true;
                }
                wave_sync();
                if (!__any(ch)) break;
            }
        }
        // P_k: the distinct exits of EXIT tails
        uint32_t nex = 0;
        if (!bad) {
            uint64_t e0 = 0, e1 = 0;
            bool x0 = false, x1 = false;
            if (lane < n && T.kind[lane] == kKExit) { x0 = true; e0 = st0 + T.xo[lane]; }
            if (lane + 64u < n && T.kind[lane + 64u] == kKExit) { x1 = true; e1 = st0 + T.xo[lane + 64u]; }
            uint64_t exv = 0;                        // lane i < nex holds distinct exit i
            for (int h = 0; h < 2 && !bad; ++h) {
                const uint64_t e = h ? e1 : e0;
                for (uint64_t m = __ballot(h ? x1 : x0); m; m &= m - 1u) {
                    const uint64_t v = rl64(e, (uint32_t)__builtin_ctzll(m));
                    if (__any(lane < nex && exv == v)) continue;
                    if (nex == kXExCap) { bad = true; break; }
                    if (lane == nex) exv = v;
                    ++nex;
                }
            }
            if (!bad && lane < nex) gput(P.ex(k) + lane, gr(tag, exv));
        }
        if (bad) {
            if (lane == 0) P.fail_all(k);
            continue;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
            gput(P.R(kQP) + k, gr(tag, nex));
            atomicAdd(&C[kCntFSurv], n);
            T.k = k;
            XT(k, 2, wall_clock64());
            __hip_atomic_store(&T.state, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        buf ^= 1u;
    }
}

// poll one granule of the current epoch (bounded); kVFail on a timeout
__device__ __forceinline__ uint64_t x_wait(const XParams &P, const uint64_t *p, uint32_t k, bool &timeout) {
    uint64_t g = rfl64(gget(p));
    for (uint32_t sp = 0; !gok(g, P.tag); ++sp) {
        if (sp >= kXSpin || P.failed_before(k)) {
            timeout = true;
            return kVFail;
        }
        __builtin_amdgcn_s_sleep(1);
        g = rfl64(gget(p));
    }
    return gval(g);
}

// region mask of the 16-B chunk at ST-relative offset c: bytes in [lo, hi) get rk
__device__ __forceinline__ u32x4 x_mask(uint32_t c, uint32_t lo, uint32_t hi, uint32_t rk) {
    u32x4 m;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        const uint32_t w = c + 4u * i;
        uint32_t s = 0u;
        if (w + 4u > lo && w < hi) {
            const uint32_t a = lo > w ? lo - w : 0u, b = hi < w + 4u ? w + 4u - hi : 0u;
            s = (0xFFFFFFFFu << (8u * a)) & (0xFFFFFFFFu >> (8u * b));
        }
        m[i] = rk & s;
    }
    return m;
}

// The unmasker wavefront of pair `pr`: the partner's STs in its ticket order.
__device__ __forceinline__ void x_unmasker(const XParams &P, XLds &S, uint32_t pr) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t N = P.N;
    const uint32_t tag = P.tag;
    const uintptr_t wb = reinterpret_cast<uintptr_t>(P.wire);
    uint32_t *const C = P.C;
    XUnW &U = S.uw[pr];
    uint32_t buf = 0;
    for (;;) {
        XTable &T = S.tab[pr][buf];
        uint32_t st;
        for (;;) {
            st = __hip_atomic_load(&T.state, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (st != 0u) break;
            __builtin_amdgcn_s_sleep(2);
        }
        st = rfl(st);
        if (st == 2u) return;
        const uint32_t k = rfl(T.k);
        const uint32_t n = rfl(T.n);
        const uint64_t st0 = (uint64_t)k * kXS;
        const uint64_t stE = P.end_of(k);
        const uint32_t len = (uint32_t)(stE - st0);
        XT(k, 3, wall_clock64());
        bool fail = false, tmo = false;
        // ---- (1) the entry guess from P_{k-1}
        uint32_t E = kXCap;                           // entry slot
        bool pass = false, ambig = false;
        uint64_t Xg = 0;                              // passing exit (pass)
        if (k == 0) {
            if (n > 0 && T.off[0] == 0) E = 0;
            else fail = true;                        // no chain from offset 0 (an error at 0)
        } else {
            const uint64_t np = x_wait(P, P.R(kQP) + (k - 1u), k, tmo);
            if (tmo || np > kXExCap) {
                fail = true;
            } else {
                uint64_t x = 0;
                bool live = false, beyond = false;
                uint32_t u = kXCap;
                if (lane < np) {
                    const uint64_t *src = P.ex(k - 1u) + lane;
                    uint64_t g = gget(src);
                    for (uint32_t sp = 0; !gok(g, tag) && sp < 64u; ++sp) g = gget(src);   // published before P
                    if (!gok(g, tag)) tmo = true;
                    x = gval(g);
                    if (x >= stE) {
                        beyond = true;
                    } else if (x >= st0) {
                        u = x_lookup(T, n, (uint32_t)(x - st0));
                        live = u < kXCap && T.kind[T.pw[u] & 0xFFu] != kKDead;
                    }
                }
                if (__any(tmo)) fail = true;
                const uint64_t lm = __ballot(live), bm = __ballot(beyond);
                if (__popcll(lm) == 1) {
                    E = rfl(lane_read(u, (uint32_t)__builtin_ctzll(lm)));
                } else if (lm == 0 && __popcll(bm) == 1) {
                    pass = true;
                    Xg = rl64(x, (uint32_t)__builtin_ctzll(bm));
                } else {
                    ambig = true;
                }
            }
        }
        // C_{k-1}, when this ST needs it before publishing its own (a passing or
        // ambiguous entry): the true state entering k if k-1 verified
        uint64_t pX = 0, pT = kNoTail;
        bool have_prev = false;
        auto load_prev = [&]() {
            if (have_prev || k == 0) return;
            pX = x_wait(P, P.R(kQCX) + (k - 1u), k, tmo);
            if (!tmo && pX != kVFail) pT = x_wait(P, P.R(kQCT) + (k - 1u), k, tmo);
            have_prev = true;
            if (tmo || pX == kVFail) fail = true;
        };
        if (!fail && (pass || ambig)) {
            load_prev();
            if (!fail) {
                if (pX >= stE) {
                    pass = true;                     // k lies inside one frame's payload
                    ambig = false;
                    Xg = pX;
                } else {
                    pass = ambig = false;
                    const uint32_t u = pX >= st0 ? x_lookup(T, n, (uint32_t)(pX - st0)) : kXCap;
                    if (u < kXCap) E = u;
                    else fail = true;                // the chain lands on no header: an error
                }
            }
        }
        // ---- (2) C_k from the guess
        uint64_t X = 0, cnt = 0, tailh = kNoTail;
        bool inc_end = false;
        if (!fail) {
            if (pass) {
                load_prev();
                X = Xg;
                cnt = 0;
                tailh = pT;
            } else {
                const uint32_t w = rfl(T.pw[E]), Tl = w & 0xFFu;
                const uint32_t kd = rfl(T.kind[Tl]), txo = rfl(T.xo[Tl]), toff = rfl(T.off[Tl]);
                cnt = (w >> 8) + (kd == kKExit || kd == kKEnd ? 1u : 0u);
                if (kd == kKExit) {
                    X = st0 + txo;
                    tailh = st0 + toff;
                } else if (kd == kKEnd) {
                    if (txo == kXFar) fail = true;
                    X = st0 + txo;
                    tailh = st0 + toff;
                } else if (kd == kKInc) {
                    inc_end = true;
                    X = st0 + toff;
                    if (stE != N) fail = true;
                    // the last frame before the incomplete header: the chain's frame before it
                    tailh = kNoTail;
                } else {
                    fail = true;                     // a protocol error on the chain
                }
            }
        }
        if (lane == 0) {
            if (fail) {
                gput(P.R(kQCX) + k, gr(tag, kVFail));
            } else {
                gput(P.R(kQCN) + k, gr(tag, cnt));
                gput(P.R(kQCT) + k, gr(tag, tailh));
                gput(P.R(kQCX) + k, gr(tag, X));
            }
        }
        XT(k, 4, wall_clock64());
        // ---- (3) verify against C_{k-1}
        bool ok = !fail;
        if (ok && k > 0) {
            load_prev();
            if (fail) ok = false;
            else if (pass) ok = pX == X || pX == Xg;
            else ok = pX == st0 + rfl(T.off[E]);
        }
        if (ok && k > 0 && pT == kNoTail && !pass && rfl(T.off[E]) != 0) ok = false;   // bytes before E need a frame
        XT(k, 5, wall_clock64());
        if (lane == 0) gput(P.R(kQA) + k, gr(tag, ok ? cnt : kVFail));
        // ---- (4) decoupled look-back: frames before k, every ST before verified
        uint64_t base = 0;
        uint32_t win = 0;
        if (ok && k > 0) {
            const uint64_t *IA = P.R(kQA), *II = P.R(kQI);
            int64_t j0 = (int64_t)k - 1;
            uint64_t acc = 0;
            bool done = false;
            for (uint32_t sp = 0; !done;) {
                const int64_t j = j0 - (int64_t)lane;
                uint64_t gi = 0, ga = 0;
                bool hi = false, ha = false;
                if (j >= 0) {
                    gi = gget(II + j);
                    ga = gget(IA + j);
                    hi = gok(gi, tag);
                    ha = gok(ga, tag);
                } else {
                    hi = true;                        // before the stream: inclusive 0
                    gi = gr(tag, 0u);
                }
                const uint64_t im = __ballot(hi);
                const uint32_t l = im ? (uint32_t)__builtin_ctzll(im) : 64u;   // nearest inclusive
                const uint64_t below = l < 64u ? ((1ull << l) - 1ull) : ~0ull;
                const bool need = ((1ull << lane) & below) != 0;
                if (__any(need && !ha)) {             // an aggregate not yet published: wait
                    if (++sp >= kXSpin || P.failed_before(k)) { ok = false; tmo = true; break; }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                const bool bad = (need && gval(ga) == kVFail) || (lane == l && gval(gi) == kVFail);
                if (__any(bad)) { ok = false; break; }
                // frame counts and bases are below cap (32-bit)
                const uint32_t v = need ? (uint32_t)gval(ga) : (lane == l ? (uint32_t)gval(gi) : 0u);
                uint32_t tot;
                (void)wave_excl_scan_dpp(v, &tot);
                acc += tot;
                win += l < 64u ? l : 64u;
                if (l < 64u) done = true;
                else j0 -= 64;
            }
            base = acc;
        }
        if (ok && base + cnt > P.cap) ok = false;    // more frames than the list holds
        if (lane == 0) {
            gput(P.R(kQI) + k, gr(tag, ok ? base + cnt : kVFail));
            if (!ok) atomicMax(&C[kCntFFail], ~k);
            if (tmo) atomicAdd(&C[kCntFTimeout], 1u);
        }
        XT(k, 6, wall_clock64());
        XT(k, 8, win);
        if (ok) {
            // ---- (5) the frames of the ST: the chain from E (lane 0 walks it)
            uint32_t nf = 0;
            if (!pass) {
                if (lane == 0) {
                    uint32_t s = E;
                    for (;;) {
                        if (T.hl[s]) U.list[nf++] = (uint8_t)s;
                        const uint8_t nx = T.lk[s];
                        if (nx == kXTerm) break;
                        s = nx;
                    }
                }
                nf = rfl(nf);
            }
            wave_sync();
            // the frame entering the ST (the last header before it, from C_{k-1})
            uint32_t nr = 0;
            if (k > 0 && pT != kNoTail) {
                const uint64_t q = pT;
                Hdr h;
                int r;
                if ((q & ~15ull) + 32u <= N) {
                    const uint64_t qa = q & ~15ull;
                    r = parse_window(gload16(wb + qa), gload16(wb + qa + 16u), (uint32_t)(q & 15u), N - q, h);
                } else {
                    r = parse_hdr([&](int i) -> uint32_t { return P.wire[q + i]; }, N - q, true, h);
                }
                if (r > 0) {
                    const uint64_t po = q + (uint64_t)r, pe0 = po + h.plen;
                    const uint64_t pe = pe0 < stE ? pe0 : stE;
                    if (pe > st0) {
                        if (lane == 0) {
                            U.lo[0] = po > st0 ? (uint32_t)(po - st0) : 0u;
                            U.hi[0] = (uint32_t)(pe - st0);
                            U.rk[0] = rotr32(h.key, 8u * ((0u - (uint32_t)po) & 3u));
                        }
                        nr = 1;
                    }
                }
            }
            // the ST's own frames: records (parsed again from their headers) and regions
            for (uint32_t i = lane; i < nf; i += 64u) {
                const uint32_t s = U.list[i];
                const uint64_t q = st0 + T.off[s];
                Hdr h;
                int r;
                if ((q & ~15ull) + 32u <= N) {
                    const uint64_t qa = q & ~15ull;
                    r = parse_window(gload16(wb + qa), gload16(wb + qa + 16u), (uint32_t)(q & 15u), N - q, h);
                } else {
                    r = parse_hdr([&](int b) -> uint32_t { return P.wire[q + b]; }, N - q, true, h);
                }
                fws_frame_info fi;
                fi.hdr_off = q;
                fi.payload_len = h.plen;
                fi.key = h.key;
                fi.opcode = (uint8_t)h.opcode;
                fi.fin = (uint8_t)h.fin;
                fi.hdr_len = (uint8_t)r;
                fi.flags = (q + (uint64_t)r + h.plen > N) ? (uint8_t)FWS_FRAME_TRUNCATED : (uint8_t)0;
                const uint64_t *s64 = reinterpret_cast<const uint64_t *>(&fi);
                uint64_t *d64 = reinterpret_cast<uint64_t *>(P.frames + base + i);
                d64[0] = s64[0];
                d64[1] = s64[1];
                d64[2] = s64[2];
                const uint64_t po = q + (uint64_t)r, pe0 = po + h.plen;
                const uint64_t pe = pe0 < stE ? pe0 : stE;
                U.lo[nr + i] = (uint32_t)(po - st0);
                U.hi[nr + i] = (uint32_t)(pe > po ? pe - st0 : po - st0);
                U.rk[nr + i] = rotr32(h.key, 8u * ((0u - (uint32_t)po) & 3u));
            }
            nr += nf;
            wave_sync();
            // ---- (6) the unmask of the ST's bytes: 4 KiB units, 16-B chunks, every
            // chunk one load and (if it holds payload) one store
            const uint32_t c_lane = lane * 16u;
            for (uint32_t u0 = 0; u0 < len; u0 += 4096u) {
                u32x4 v[4];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    const uint32_t c = u0 + j * 1024u + c_lane;
                    v[j] = c + 16u <= len ? gload16<true>(wb + st0 + c) : u32x4{0u, 0u, 0u, 0u};
                }
                // regions meeting the unit: the first with hi > u0 (regions are sorted)
                uint32_t lo = 0, hi = nr;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (U.hi[mid] <= u0) lo = mid + 1u; else hi = mid;
                }
                const uint32_t u1 = u0 + 4096u;
                lo = rfl(lo);
                const bool one = lo < nr && U.lo[lo] <= u0 && U.hi[lo] >= u1;   // one payload covers the unit
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    const uint32_t c = u0 + j * 1024u + c_lane;
                    u32x4 m;
                    if (one) {
                        const uint32_t rk = U.rk[lo];
                        m = u32x4{rk, rk, rk, rk};
                    } else {
                        m = u32x4{0u, 0u, 0u, 0u};
                        for (uint32_t g = lo; g < nr && U.lo[g] < u1; ++g) m |= x_mask(c, U.lo[g], U.hi[g], U.rk[g]);
                    }
                    if (c >= len || !(m.x | m.y | m.z | m.w)) continue;
                    if (c + 16u <= len) {
                        gstore16<true>(wb + st0 + c, v[j] ^ m);
                    } else {
                        const uint32_t mw[4] = {m.x, m.y, m.z, m.w};
                        for (uint32_t b = 0; c + b < len; ++b)
                            P.wire[st0 + c + b] ^= (uint8_t)(mw[b >> 2] >> (8u * (b & 3u)));
                    }
                }
            }
            XT(k, 7, wall_clock64());
            if (lane == 0) {
                gput(P.R(kQDone) + k, gr(tag, 1u));
                if (stE == N) {
                    // the result (OnRecvData's end state on this buffer)
                    const uint64_t nfr = base + cnt;
                    fws_decode_result *const rs = P.res;
                    rs->status = FWS_OK;
                    rs->n_frames = (uint32_t)nfr;
                    rs->err_off = 0;
                    if (inc_end) {
                        rs->consumed = X;
                        rs->carry_unread = 0;
                        rs->carry_hdr_len = (uint32_t)(N - X);
                    } else {
                        rs->consumed = N;
                        rs->carry_unread = X > N ? X - N : 0;
                        rs->carry_hdr_len = 0;
                    }
                    rs->n_survivors = cget(&C[kCntFSurv]);
                    __hip_atomic_store(&C[kCntFrames], (uint32_t)nfr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        wave_sync();
        if (lane == 0) __hip_atomic_store(&T.state, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        buf ^= 1u;
    }
}

__global__ __launch_bounds__(kXThreads) __attribute__((amdgpu_waves_per_eu(kXBlocksPerCu, kXBlocksPerCu))) void k_stream(XParams P) {
    __shared__ __attribute__((aligned(16))) XLds S;
    const uint32_t tid = threadIdx.x, wv = tid >> 6;
    if (blockIdx.x == 0 && tid == 0) __hip_atomic_store(&P.C[kCntFMode], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid < kXPairs * 2) S.tab[tid >> 1][tid & 1].state = 0u;
    __syncthreads();
    const uint32_t pr = wv % kXPairs;
    if (wv < kXPairs) x_scanner(P, S, pr);
    else x_unmasker(P, S, pr);
}

}  // namespace fwsk

// ------------------------------------------------------------------ host side
using namespace fwsk;

// tuning / test hook: 0 = the multi-launch path only, 1 = k_stream first for
// streams of at least kFusedMin bytes (the default), 2 = for every stream of at
// least 16 bytes (tests)
static int g_fused = 0;   // (1 once verified on the GPU)
extern "C" __attribute__((visibility("default"))) int fws_internal_set_fused(int mode) {
    const int old = g_fused;
    if (mode >= 0 && mode <= 2) g_fused = mode;
    return old;
}
// test hook: per-ST phase clocks of the last k_stream call (tools/prof_stream.py)
static int g_trace_on = 0;
static uint64_t *g_trace = nullptr;
static uint64_t g_trace_cap = 0, g_trace_n = 0;
extern "C" __attribute__((visibility("default"))) int fws_internal_fused_trace(int on) {
    g_trace_on = on != 0;
    return 0;
}
// copies min(n, STs of the last traced call) records of kXTraceW words; returns the count
extern "C" __attribute__((visibility("default"))) long long fws_internal_fused_trace_read(uint64_t *out, long long n) {
    if (!g_trace || n <= 0) return 0;
    const uint64_t m = (uint64_t)n < g_trace_n ? (uint64_t)n : g_trace_n;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpy(out, g_trace, m * kXTraceW * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return (long long)m;
}
bool fws_fused_enabled(uint64_t N) { return g_fused == 2 ? N >= 16 : g_fused == 1 && N >= kFusedMin; }

int fws_fused_ensure(fws_gpu_ctx *ctx, uint64_t N) {
    fws_decode_ws &d = ctx->dec;
    const uint64_t n_st = (N + kXS - 1) / kXS;
    if (n_st <= d.fmax_st) return 0;
    if (d.fpub) (void)hipFree(d.fpub);
    d.fpub = nullptr;
    d.fmax_st = 0;
    const uint64_t bytes = n_st * kXPubWords * sizeof(uint64_t);
    hipError_t e = hipMalloc((void **)&d.fpub, bytes);
    if (e == hipSuccess) e = hipMemset(d.fpub, 0, bytes);   // no tag is 0
    if (e != hipSuccess) return fws_hip_status(e);
    d.fmax_st = n_st;
    return 0;
}

const uint64_t *fws_fused_done(const fws_gpu_ctx *ctx) {
    return ctx->dec.fpub ? ctx->dec.fpub + (uint64_t)kQDone * ctx->dec.fmax_st : nullptr;
}

int fws_launch_fused(fws_gpu_ctx *ctx, uint8_t *wire, uint64_t N, fws_frame_info *frames, uint32_t cap,
                     fws_decode_result *res, hipStream_t s) {
    fws_decode_ws &d = ctx->dec;
    const uint64_t n_st = (N + kXS - 1) / kXS;
    if (n_st > d.fmax_st || n_st >= (1ull << 31) || N >= (1ull << 39)) return FWS_ERR_INTERNAL;
    if (d.fcus == 0) {                               // per context: its device's CU count
        int cus = 0;
        hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device);
        if (e != hipSuccess) return fws_hip_status(e);
        d.fcus = (uint32_t)cus;
    }
    d.fepoch = (d.fepoch + 1u) & 0xFFFFFFu;
    if (d.fepoch == 0) d.fepoch = 1;
    XParams P;
    P.wire = wire;
    P.N = N;
    P.n_st = (uint32_t)n_st;
    P.tag = d.fepoch;
    P.frames = frames;
    P.cap = cap;
    P.res = res;
    P.C = d.counters;
    P.pub = d.fpub;
    P.stride = d.fmax_st;
    P.trace = nullptr;
    if (g_trace_on) {
        if (g_trace_cap < n_st) {
            if (g_trace) (void)hipFree(g_trace);
            g_trace = nullptr;
            g_trace_cap = 0;
            if (hipMalloc((void **)&g_trace, n_st * kXTraceW * 8) != hipSuccess) return FWS_ERR_INTERNAL;
            g_trace_cap = n_st;
        }
        P.trace = g_trace;
        g_trace_n = n_st;
    }
    const uint64_t g = (uint64_t)d.fcus * kXBlocksPerCu;
    const uint64_t need = (n_st + kXPairs - 1) / kXPairs;
    hipLaunchKernelGGL(k_stream, dim3((unsigned)(need < g ? need : g)), dim3(kXThreads), 0, s, P);
    return fws_hip_status(hipGetLastError());
}
