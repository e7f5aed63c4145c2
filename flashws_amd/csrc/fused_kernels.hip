// fused_kernels.hip -- one-pass fws_gpu_decode_stream on gfx950: the header
// scan, the chain resolve and the unmask of a server-side wire stream in ONE
// launch that reads every stream byte from HBM once and writes it once.
// Replaces the serial frame loop of WSocket::OnRecvData (net/w_socket.h:543-769)
// for a device-resident buffer, like the multi-launch path (decode_kernels.hip
// + merge_kernels.hip + k_unmask_stream), which stays as this kernel's fallback.
//
// Why: the multi-launch path reads the stream twice (k_scan, then the unmask
// re-reads it after the resolve), and the Infinity Cache gives no reuse across
// those launches (tools/ic_probe.hip: a re-read only pays off from L2, within a
// few microseconds). Here each workgroup holds a 32 KiB super tile (ST) in LDS
// from the scan to the unmask.
//
// Per ST (ordered tickets; a persistent grid of 3 workgroups per CU, the next
// ST's bytes prefetched into registers while this one is processed):
//  L  scan the 16 tiles from LDS (the k_scan tile body: two-byte candidate
//     test, first hop, live nodes with pointer jumping in registers, now also
//     counting frames to the leaf), then link every survivor to the survivor at
//     its tile-leaf exit and pointer-jump in LDS (pointer and frame count in one
//     word): each survivor knows how its chain leaves the ST. The distinct exits
//     of live chains (own exits, typically the true one plus a few false long
//     jumps) are published; an exit landing two or more STs ahead is pushed to
//     that ST's inbox. LOCAL is published.
//  F  once every ST before this one is LOCAL (a look-back over the LOCAL and
//     FRONT words), the keys -- the previous ST's own exits that land here plus
//     this ST's inbox -- are every offset the true chain can enter this ST at.
//     Each key is resolved against this ST's survivors; the live ones (usually
//     one) form the fast table: key -> (exit, frames, last header). Published.
//  B  decoupled look-back: the nearest ST with an inclusive state (the true
//     entry of its successor, frames before it, the last header before it);
//     the fast tables of the STs between are composed in registers (an entry
//     at or past an ST's end passes it unchanged). INCL is published for this
//     ST at once.
//  U  the true frames of the ST (tile entries along the chain, then a walk per
//     tile), their fws_frame_info, the unmask of the ST's bytes from LDS (the
//     payload of the frame covering the ST start is parsed from its header) with
//     16-B stores, and the result if this is the last ST.
// Handed-off words are 8-B granules {tag = call epoch, 40-bit value}: relaxed
// agent-scope atomics (sc1) whose tag is the flag (cdna_hip_programming.md
// Guideline 16, recipe R2), so nothing is zeroed per call. Every wait is on a
// lower ticket (held by a running workgroup) and bounded.
//
// Fallback: an ST that cannot finish exactly here (a dense tile: frames under
// ~40 B; more than 32 survivors in a tile; more exits than the tables hold; a
// protocol error or an incomplete header reached by the true chain; more frames
// than `cap`; a bounded wait that gave up) publishes FAIL and writes nothing;
// every later ST then fails too (it cannot compose through it). The
// multi-launch path, launched after this kernel, returns at once unless
// kCntFFail is set, and then decodes the whole stream again (headers are never
// modified, so its scan sees the same chain) while its unmask skips the STs
// this kernel marked done.
#include "scan_common.h"

namespace fwsk {

constexpr uint32_t kFTiles = 16;                            // tiles per fused super tile
constexpr uint32_t kFS = kFTiles * kTile;                   // 32 KiB
static_assert(kFS == kFusedStBytes, "fws_internal.h names the fused super-tile size");
constexpr uint32_t kFWaves = 4;
constexpr uint32_t kFThreads = kFWaves * 64;
constexpr uint32_t kFBlocksPerCu = 3;                       // LDS: 3 x ~52 KB per CU
constexpr uint32_t kFTileCap = 32;                          // survivors per tile
constexpr uint32_t kFSlots = kFTiles * kFTileCap;           // survivor slots per ST
constexpr uint32_t kFBuf = kFS + kHaloX + 16;               // ST bytes, halo, parse-window over-read
constexpr uint32_t kFHaloLoads = (kHaloX + 16) / 16;        // 16-B halo loads (threads)
constexpr uint32_t kFLoads = kFS / (kFThreads * 16);        // 16-B loads per thread per ST
constexpr uint32_t kFExCap = 16;                            // own exits published per ST
constexpr uint32_t kFInCap = 16;                            // inbox entries per ST
constexpr uint32_t kFLive = 2;                              // live fast-table entries per ST
constexpr uint32_t kFDepth = 4;                             // fast-table keys: own exits of the STs k-4..k-1
constexpr uint32_t kPsDead = 0xFFFFu;                       // ps: the chain dies in the ST
constexpr uint32_t kXFar = 0xFFFFFFFFu;                     // fexit: beyond st0 + 4 GiB
constexpr uint16_t kIncBit = 0x8000;                        // lcnt: the leaf is an incomplete header
constexpr uint16_t kNoLink = 0xFFFF;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
constexpr uint32_t kSpinMax = 1u << 14;                     // bounded waits (~25 ms: polls are ~1.5 us)

// published granules: SoA regions of fmax_st words, then a block per ST
enum FRegion : uint32_t {
    kRLocal = 0,     // value: own exits published | kLFail
    kRFront = 1,     // every ST <= m is LOCAL
    kRInX = 2,       // INCL: entry of ST m + 1 (or kVFail)
    kRInB = 3,       //       frames before ST m + 1
    kRInT = 4,       //       header of the last frame before ST m + 1 (kNoTail: none)
    kRFt = 5,        // fast table header: live entries | kFtInc | kFtFail
    kRDone = 6,      // ST m's bytes were unmasked here (fws_launch_unmask_stream skips them)
    kRInbox = 7,     // inbox count (saturating past kFInCap: overflow)
    kFRegions = 8
};
constexpr uint32_t kBEx = 0, kBFt = kFExCap + kFInCap;   // block offsets (kFInCap words after the exits: former inbox, unused)
constexpr uint32_t kFBlk = kBFt + 4 * kFLive;                             // words per ST block
constexpr uint32_t kFPubWords = kFRegions + kFBlk;
constexpr uint64_t kV40 = (1ull << 40) - 1;
constexpr uint64_t kVFail = kV40;
constexpr uint64_t kNoTail = kV40 - 1;
constexpr uint32_t kLFail = 1u << 8;
constexpr uint32_t kFtInc = 4, kFtFail = 8;

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
__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l);
    return ((uint64_t)hi << 32) | lo;
}

struct FusedParams {
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
    uint64_t *trace;                                // test hook: per-ST clocks (kFTraceW words), or null

    __device__ __forceinline__ uint64_t *R(uint32_t r) const { return pub + (uint64_t)r * stride; }
    __device__ __forceinline__ uint64_t *blk(uint32_t m) const {
        return pub + (uint64_t)kFRegions * stride + (uint64_t)m * kFBlk;
    }
    __device__ __forceinline__ uint64_t end_of(uint64_t m) const {
        const uint64_t e = (m + 1) * kFS;
        return e < N ? e : N;
    }
    // an ST before k has failed (kCntFFail holds ~(first failing ST))
    __device__ __forceinline__ bool failed_before(uint32_t k) const {
        const uint32_t f = (uint32_t)__builtin_amdgcn_readfirstlane((int)cget(&C[kCntFFail]));
        return f != 0u && ~f < k;
    }
};

// one wavefront's tile scratch (the k_scan tile body)
struct FScanW {
    uint32_t cm[64];                                // candidate bits of lane L's 32 offsets
    uint32_t lm[64];                                // live bits
    uint32_t lpre[64];                              // live index of lane L's first live offset
    uint16_t pos[kCandCap];
    uint16_t lpos[kLiveCap];
};
// a true frame of the ST (offsets relative to the ST start)
struct FFrame {
    uint16_t hdr;
    uint8_t hl;
    uint8_t pad;
    uint32_t key;
    uint32_t pe;                                    // payload end, clipped to the ST end
};
struct FusedLds {
    uint8_t bytes[kFBuf];
    // survivor slots: tile t owns [t * kFTileCap, t * kFTileCap + n_t), offset order
    uint16_t soff[kFSlots];                         // ST-relative offset
    uint32_t fexit[kFSlots];                        // own frame's exit (ST-relative, kXFar), or the
                                                    //   header itself for an incomplete one
    uint16_t lleaf[kFSlots];                        // slot of the tile leaf of its chain
    uint16_t lcnt[kFSlots];                         // frames to the leaf inclusive | kIncBit
    uint16_t link[kFSlots];                         // slot at the leaf's exit (next tile) or kNoLink
    uint32_t ps[kFSlots];                           // in-ST pointer | frames before it << 16
    union {
        struct {
            uint32_t sbits[kFTiles][64];            // survivor offsets, per tile
            uint8_t spre[kFTiles][64];              // survivors before word w of the tile
            FScanW w[kFWaves];
        } s;
        FFrame fr[kFSlots];                         // after the resolve: the ST's true frames
    } u;
    uint32_t tcnt[kFTiles];                         // survivors per tile, later frames per tile
    uint32_t fpre[kFTiles + 1];
    int32_t fcov[kFTiles];                          // frame slot covering a tile's start, -1: head
    uint16_t tentry[kFTiles];
    uint64_t ex[kFExCap];
    uint64_t X, base, tail, hpo, hpe;
    uint32_t hkey, n_ex, fail, ticket, own_u, own_cnt, nf, inc_end, surv;
    uint64_t nx;
};
static_assert(sizeof(FusedLds) * kFBlocksPerCu <= 160u * 1024u, "fused LDS per CU");

// survivor slot at ST-relative offset o (< the ST end), or kNoSlot
__device__ __forceinline__ uint32_t f_lookup(const FusedLds &S, uint32_t o) {
    const uint32_t te = o >> 11, oo = o & (kTile - 1), wd = oo >> 5, b = oo & 31u;
    const uint32_t bits = S.u.s.sbits[te][wd];
    if (!((bits >> b) & 1u)) return kNoSlot;
    return te * kFTileCap + S.u.s.spre[te][wd] + (uint32_t)__popc(bits & ((1u << b) - 1u));
}

__device__ __forceinline__ uint32_t f_byte_sel(uint64_t w, uint64_t lo, uint64_t hi) {
    if (w + 4u <= lo || w >= hi) return 0u;
    const uint32_t s = lo > w ? (uint32_t)(lo - w) : 0u;
    const uint32_t e = hi < w + 4u ? (uint32_t)(w + 4u - hi) : 0u;
    return (0xFFFFFFFFu << (8u * s)) & (0xFFFFFFFFu >> (8u * e));
}
// key mask of the 16-B chunk at stream offset c for payload [po, pe), key k (phase 0 at po)
__device__ __forceinline__ u32x4 f_region_mask(uint64_t c, uint64_t po, uint64_t pe, uint32_t k) {
    if (pe <= c || po >= c + 16u) return u32x4{0u, 0u, 0u, 0u};
    const uint32_t rk = rotr32(k, 8u * ((uint32_t)(c - po) & 3u));
    return u32x4{rk & f_byte_sel(c, po, pe), rk & f_byte_sel(c + 4u, po, pe), rk & f_byte_sel(c + 8u, po, pe),
                 rk & f_byte_sel(c + 12u, po, pe)};
}

// Tile t of the ST (bytes in LDS): the k_scan tile body (decode_kernels.hip),
// plus frame counts to the leaf. Writes the tile's survivor slots, bitmap and
// count. Returns true (wave-uniform) when the tile is too dense for this path.
__device__ bool f_scan_tile(FusedLds &S, uint32_t t, uint64_t st0, uint64_t N) {
    const uint32_t lane = threadIdx.x & 63;
    FScanW &W = S.u.s.w[threadIdx.x >> 6];
    const uint64_t t0 = st0 + (uint64_t)t * kTile;
    const uint8_t *const B = S.bytes + t * kTile;
    const uint32_t L32 = lane * 32u;
    S.u.s.sbits[t][lane] = 0u;
    if (t0 >= N) {
        S.u.s.spre[t][lane] = 0;
        if (lane == 0) S.tcnt[t] = 0;
        return false;
    }
    W.lm[lane] = 0u;
    uint32_t cm;
    {
        const u32x4 w0 = *reinterpret_cast<const u32x4 *>(B + L32);
        const u32x4 w1 = *reinterpret_cast<const u32x4 *>(B + L32 + 16u);
        const uint32_t nx = *reinterpret_cast<const uint32_t *>(B + L32 + 32u);
        cm = cand_bits32p(w0, w1, nx);
        // bytes past the end are zero in LDS and never pass; the last byte is a
        // candidate on its own (an incomplete header, w_socket.h:443-445)
        const uint64_t q = t0 + L32;
        if (q < N && N - q <= 32u) cm |= 1u << cand_pbit((uint32_t)(N - q) - 1u);
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
    wave_sync();
    // first hop: a candidate whose next header (7-bit length, complete) is inside
    // the tile on a non-candidate byte is dead
    uint32_t M = 0;
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
    {
        uint32_t mt;
        uint32_t lbits = W.lm[lane];
        uint32_t li = wave_excl_scan_dpp((uint32_t)__popc(lbits), &mt);
        W.lpre[lane] = li;
        while (lbits) {
            const uint32_t b = (uint32_t)__ffs(lbits) - 1u;
            lbits &= lbits - 1u;
            W.lpos[li++] = (uint16_t)(L32 + b);
        }
    }
    wave_sync();
    // live node `lane`: full parse, next live node, leaf or dead; frames to the leaf
    const bool act = lane < M;
    const uint32_t p = act ? W.lpos[lane] : 0u;
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
            const uint32_t m = W.lm[nx >> 5], bit = nx & 31u;
            if ((m >> bit) & 1u) ptr = W.lpre[nx >> 5] + (uint32_t)__popc(m & ((1u << bit) - 1u));
        }
    }
    const uint32_t w = r > 0 ? 1u : 0u;              // a frame (an incomplete header counts none)
    uint32_t sum = (ptr < 64u && ptr != lane) ? w : 0u;   // frames in [node, ptr)
    for (;;) {
        const uint32_t src = ptr < 64u ? ptr : lane;
        const uint32_t q = lane_read(ptr, src);
        const uint32_t qs = lane_read(sum, src);
        const uint32_t np = ptr < 64u ? q : ptr;
        const bool ch = np != ptr;
        if (ch) sum += qs;
        ptr = np;
        if (!__any(ch)) break;
    }
    const bool surv = act && ptr < 64u;
    const uint64_t sm = __ballot(surv);
    const uint32_t ns = (uint32_t)__popcll(sm);
    if (ns > kFTileCap) return true;
    const uint32_t leaf = ptr < 64u ? ptr : lane;
    const uint32_t wl = lane_read(w, leaf);
    const uint32_t il = lane_read((act && r == 0) ? 1u : 0u, leaf);
    if (surv) {
        const uint32_t slot = t * kFTileCap + mbcnt64(sm);
        const uint32_t lrank = (uint32_t)__popcll(sm & ((1ull << leaf) - 1ull));
        const uint64_t ex = r > 0 ? (t0 + p + (uint64_t)r + plen) - st0 : (uint64_t)(t * kTile + p);
        S.soff[slot] = (uint16_t)(t * kTile + p);
        S.fexit[slot] = ex >= kXFar ? kXFar : (uint32_t)ex;
        S.lleaf[slot] = (uint16_t)(t * kFTileCap + lrank);
        S.lcnt[slot] = (uint16_t)((sum + wl) | (il ? kIncBit : 0u));
        atomicOr(&S.u.s.sbits[t][p >> 5], 1u << (p & 31u));
    }
    wave_sync();
    {
        uint32_t tot;
        const uint32_t pre = wave_excl_scan_dpp((uint32_t)__popc(S.u.s.sbits[t][lane]), &tot);
        S.u.s.spre[t][lane] = (uint8_t)pre;
    }
    if (lane == 0) S.tcnt[t] = ns;
    return false;
}

// The kFDepth STs before k have published LOCAL (their own exits are this ST's
// keys). False: one of them failed, an ST before k failed, or the wait gave up.
__device__ bool f_wait_recent(const FusedParams &P, uint32_t k, uint32_t lane, uint32_t &nspin) {
    const uint64_t *const LO = P.R(kRLocal);
    for (uint32_t spins = 0;; ++spins) {
        bool ok = true, fail = false;
        if (lane < kFDepth && k >= lane + 1u) {
            const uint64_t gl = gget(LO + (k - 1u - lane));
            ok = gok(gl, P.tag);
            fail = ok && (gval(gl) & kLFail);
        }
        nspin = spins;
        if (__any(fail)) return false;
        if (__all(ok)) return true;
        if (spins >= kSpinMax || P.failed_before(k)) return false;
        __builtin_amdgcn_s_sleep(1);
    }
}

// The state entering ST k by decoupled look-back: X (the true chain's first
// header at or after the ST start, or a passing exit), frames before it, the
// header of the last frame before it. False: not resolvable here.
__device__ bool f_lookback(const FusedParams &P, uint32_t k, uint32_t lane, uint64_t &X, uint64_t &base,
                           uint64_t &tail, uint32_t &nspin, uint32_t &win) {
    if (k == 0) {
        X = 0;
        base = 0;
        tail = kNoTail;
        return true;
    }
    const uint32_t tag = P.tag;
    const uint64_t *const IX = P.R(kRInX), *const IB = P.R(kRInB), *const IT = P.R(kRInT), *const FT = P.R(kRFt);
    // pass 1: the nearest ST with INCL (or FAIL); every fast table after it ready.
    // All four words of a lane are loaded in one batch (a load that waited for
    // another made the look-back latency grow with the window, and the window
    // with the latency).
    int64_t j = -1;
    for (uint32_t spins = 0;; ++spins) {
        bool ready = true, fail = false;
        for (int64_t w0 = (int64_t)k - 1;; w0 -= 64) {
            const int64_t m = w0 - (int64_t)lane;
            bool inc = false, f = false, ftr = false;
            const bool valid = m >= -1;
            if (m >= 0) {
                const uint64_t gx = gget(IX + m), gb = gget(IB + m), gt = gget(IT + m), h = gget(FT + m);
                if (gok(gx, tag)) {
                    if (gval(gx) == kVFail) f = true;
                    else inc = gok(gb, tag) && gok(gt, tag);
                }
                if (gok(h, tag)) {
                    if (gval(h) & kFtFail) f = true;
                    ftr = !(gval(h) & kFtInc);
                }
            } else if (m == -1) {
                inc = true;
            }
            const uint64_t im = __ballot(valid && (inc || f));
            if (im) {
                const uint32_t l = (uint32_t)__ffsll((unsigned long long)im) - 1u;
                const uint64_t below = l ? ((1ull << l) - 1ull) : 0ull;
                if (__ballot(f) & (below | (1ull << l))) fail = true;
                if (__ballot(!ftr) & below) ready = false;
                j = w0 - (int64_t)l;
                break;
            }
            if (__ballot(f)) {
                fail = true;
                break;
            }
            if (__ballot(!ftr)) ready = false;
        }
        nspin = spins;
        if (fail) return false;
        if (ready) break;
        if (spins >= kSpinMax || P.failed_before(k)) return false;
        __builtin_amdgcn_s_sleep(1);
    }
    win = (uint32_t)((int64_t)k - 1 - j);
    if (j < 0) {
        X = 0;
        base = 0;
        tail = kNoTail;
    } else {
        X = gval(gget(IX + j));
        base = gval(gget(IB + j));
        tail = gval(gget(IT + j));
    }
    // pass 2: compose the fast tables of STs j+1 .. k-1, 64 per step. Common
    // case: every ST the chain enters has one live entry and every other ST has
    // none, so the chain's STs are the non-empty ones, each entered at the exit
    // of the previous non-empty one: checked lane-parallel (each key against the
    // previous non-empty lane's exit), frames summed by a wave scan. Anything
    // else (two live entries, a key that does not match) is composed serially.
    for (int64_t c0 = j + 1; c0 <= (int64_t)k - 1; c0 += 64) {
        const int64_t m = c0 + (int64_t)lane;
        const bool in = m <= (int64_t)k - 1;
        uint64_t e[4 * kFLive];
        uint32_t nl = 0;
        if (in) {
            const uint64_t *b = P.blk((uint32_t)m) + kBFt;
            const uint64_t h = gget(FT + m);
#pragma unroll
            for (uint32_t i = 0; i < 4 * kFLive; ++i) e[i] = gget(b + i);
            nl = (uint32_t)(gval(h) & 3u);
            bool bad = false;
#pragma unroll
            for (uint32_t i = 0; i < 4 * kFLive; ++i) bad = bad || (i < 4 * nl && !gok(e[i], tag));
            for (uint32_t sp = 0; bad && sp < 4096; ++sp) {      // published before the header: rare
                bad = false;
#pragma unroll
                for (uint32_t i = 0; i < 4 * kFLive; ++i) {
                    if (i < 4 * nl && !gok(e[i], tag)) e[i] = gget(b + i);
                    bad = bad || (i < 4 * nl && !gok(e[i], tag));
                }
            }
            if (bad) nl = 3;                                    // unreadable: the serial path fails
#pragma unroll
            for (uint32_t i = 0; i < 4 * kFLive; ++i) e[i] = gval(e[i]);
        }
        const uint32_t cnt = (int64_t)k - c0 < 64 ? (uint32_t)((int64_t)k - c0) : 64u;
        const uint64_t ne = __ballot(in && nl == 1u);
        bool fast = !__any(in && nl > 1u);
        if (fast) {
            // previous non-empty lane's exit (or X entering the chunk) must be this lane's key
            uint64_t pre_lo = ne & ((1ull << lane) - 1ull);
            const uint32_t p = pre_lo ? 63u - (uint32_t)__clzll((unsigned long long)pre_lo) : 64u;
            const uint32_t src = p < 64u ? p : lane;
            const uint64_t po = ((uint64_t)lane_read((uint32_t)(e[1] >> 32), src) << 32) | lane_read((uint32_t)e[1], src);
            const uint64_t arrive = p < 64u ? po : X;
            const bool ok = !((ne >> lane) & 1ull) || e[0] == arrive;
            fast = __all(ok);
            if (fast) {
                if (ne) {
                    const uint32_t L = 63u - (uint32_t)__clzll((unsigned long long)ne);
                    const uint64_t xl = readlane64(e[1], L);
                    // the empty STs after the last non-empty one are passed: its exit must reach their end
                    if (xl < P.end_of((uint64_t)c0 + cnt - 1u) && L + 1u < cnt) fast = false;
                    else {
                        uint32_t tot;
                        (void)wave_excl_scan_dpp(((ne >> lane) & 1ull) ? (uint32_t)e[2] : 0u, &tot);
                        X = xl;
                        base += tot;
                        tail = readlane64(e[3], L);
                    }
                } else if (X < P.end_of((uint64_t)c0 + cnt - 1u)) {
                    fast = false;                               // the chain stops in an empty ST
                }
            }
        }
        if (fast) continue;
        for (uint32_t l = 0; l < cnt; ++l) {
            const uint64_t mm = (uint64_t)c0 + l;
            if (X >= P.end_of(mm)) continue;                 // the ST lies inside one frame's payload
            const uint32_t n = (uint32_t)__builtin_amdgcn_readlane((int)nl, (int)l);
            bool hit = false;
#pragma unroll
            for (uint32_t i = 0; i < kFLive; ++i) {
                const uint64_t key = readlane64(e[4 * i], l);
                if (!hit && i < n && n <= kFLive && key == X) {   // n == 3: unreadable, a miss
                    X = readlane64(e[4 * i + 1], l);
                    base += readlane64(e[4 * i + 2], l);
                    tail = readlane64(e[4 * i + 3], l);
                    hit = true;
                }
            }
            if (!hit) {
                // the entry is no key of this ST's fast table: a jump from more than
                // kFDepth STs back, or a protocol error. This ST resolves it from its
                // own tables: wait for its INCL (FAIL if the chain dies there).
                const uint64_t *px = IX + mm, *pb = IB + mm, *pt = IT + mm;
                uint64_t gx = gget(px), gb = gget(pb), gt = gget(pt);
                for (uint32_t sp = 0; !(gok(gx, tag) && gok(gb, tag) && gok(gt, tag)); ++sp) {
                    if (gok(gx, tag) && gval(gx) == kVFail) return false;
                    if (sp >= kSpinMax || P.failed_before(k)) return false;
                    __builtin_amdgcn_s_sleep(1);
                    gx = gget(px);
                    gb = gget(pb);
                    gt = gget(pt);
                }
                if (gval(gx) == kVFail) return false;
                X = gval(gx);
                base = gval(gb);
                tail = gval(gt);
            }
        }
    }
    return true;
}

// tools/prof_fused.py: trace[k * kFTraceW + i] = wall clock at phase i of ST k
// (0 start, 1 after L, 2 after F, 3 after B, 4 end), 5 = look-back window,
// 6 = lookback spins, 7 = frontier spins (wave 0 lane 0 writes)
constexpr uint32_t kFTraceW = 12;   // + 8 after load, 9 after scan, 10 after the in-ST resolve
#define FT_MARK(i, v) do { if (P.trace && tid == 0) P.trace[(uint64_t)k * kFTraceW + (i)] = (v); } while (0)

__global__ __launch_bounds__(kFThreads) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_fused(FusedParams P) {
    __shared__ __attribute__((aligned(16))) FusedLds S;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t *const C = P.C;
    const uint64_t N = P.N;
    const uint32_t tag = P.tag;
    uint8_t *const wire = P.wire;
    const uintptr_t wb = reinterpret_cast<uintptr_t>(wire);
    if (blockIdx.x == 0 && tid == 0) __hip_atomic_store(&C[kCntFMode], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    u32x4 pf[kFLoads], ph = u32x4{0u, 0u, 0u, 0u};
    auto load_st = [&](uint32_t kk) {
        if (kk >= P.n_st) return;
        const uint64_t b = (uint64_t)kk * kFS;
#pragma unroll
        for (uint32_t j = 0; j < kFLoads; ++j) {
            const uint64_t o = b + j * (kFThreads * 16u) + tid * 16u;
            pf[j] = gload16<true>(wb + (o + 16u <= N ? o : 0u));
        }
        const uint64_t o = b + kFS + tid * 16u;
        if (tid < kFHaloLoads) ph = gload16<true>(wb + (o + 16u <= N ? o : 0u));
    };
    auto store_st = [&](uint32_t kk) {
        const uint64_t b = (uint64_t)kk * kFS;
#pragma unroll
        for (uint32_t j = 0; j <= kFLoads; ++j) {
            if (j == kFLoads && tid >= kFHaloLoads) break;
            const uint32_t o = j < kFLoads ? j * (kFThreads * 16u) + tid * 16u : kFS + tid * 16u;
            const uint64_t a = b + o;
            if (a + 16u <= N) {
                *reinterpret_cast<u32x4 *>(S.bytes + o) = j < kFLoads ? pf[j] : ph;
            } else {
                for (uint32_t i = 0; i < 16u; ++i) S.bytes[o + i] = a + i < N ? wire[a + i] : (uint8_t)0;
            }
        }
    };

    // A ticket is taken only when its ST is processed at once: a ticket held
    // while the workgroup finishes an older ST delays every later ST's frontier
    // (measured: 87 us frontier waits and 230-ST look-back windows on C2).
    for (;;) {
        __syncthreads();                             // the previous ST is done with LDS
        if (tid == 0) {
            const uint32_t t = atomicAdd(&C[kCntFTicket], 1u);
            S.ticket = t;
            // decided once for the workgroup: every wave must take the same branches
            // (they hold barriers), so no thread reads the fail word on its own
            S.fail = t < P.n_st && P.failed_before(t) ? 1u : 0u;
            S.n_ex = 0;
            S.surv = 0;
        }
        __syncthreads();
        const uint32_t k = S.ticket;
        if (k >= P.n_st) break;
        FT_MARK(0, wall_clock64());
        load_st(k);
        store_st(k);
        __syncthreads();

        const uint64_t st0 = (uint64_t)k * kFS;
        const uint64_t stE = P.end_of(k);
        const uint32_t rel_end = (uint32_t)(stE - st0);
        bool pub_local = false, pub_ft = false;
        auto fail_now = [&]() {                      // wave 0: publish FAIL for every word still open
            if (lane == 0) {
                if (!pub_local) gput(P.R(kRLocal) + k, gr(tag, kLFail));
                if (!pub_ft) gput(P.R(kRFt) + k, gr(tag, kFtFail));
                gput(P.R(kRInX) + k, gr(tag, kVFail));
                atomicMax(&C[kCntFFail], ~k);
                S.fail = 1;
            }
        };

        // ---- L: scan, in-ST resolve, own exits, LOCAL
        FT_MARK(8, wall_clock64());
        bool skip = S.fail != 0;
        if (!skip) {
            for (uint32_t t = wv; t < kFTiles; t += kFWaves)
                if (f_scan_tile(S, t, st0, N) && lane == 0) S.fail = 1;
        }
        __syncthreads();
        FT_MARK(9, wall_clock64());
        skip = skip || S.fail;
        if (!skip) {
            for (uint32_t s = tid; s < kFSlots; s += kFThreads) {
                const uint32_t t = s / kFTileCap;
                if (s % kFTileCap >= S.tcnt[t]) continue;
                const uint32_t lf = S.lleaf[s];
                const uint32_t lc = S.lcnt[s];
                uint32_t v = s;                      // terminal: leaves the ST / the stream, or incomplete
                uint16_t lk = kNoLink;
                if (!(lc & kIncBit)) {
                    const uint32_t e = S.fexit[lf];
                    if (e < rel_end) {
                        const uint32_t u = f_lookup(S, e);
                        if (u != kNoSlot) {
                            lk = (uint16_t)u;
                            v = u | ((lc & 0x7FFFu) << 16);
                        } else {
                            v = kPsDead;
                        }
                    }
                }
                S.ps[s] = v;
                S.link[s] = lk;
            }
            if (tid < kFTiles) atomicAdd(&S.surv, S.tcnt[tid]);
            __syncthreads();
            // pointer jumping in place: (pointer, frames before it) move together in one word
            for (;;) {
                int changed = 0;
                for (uint32_t s = tid; s < kFSlots; s += kFThreads) {
                    if (s % kFTileCap >= S.tcnt[s / kFTileCap]) continue;
                    const uint32_t v = S.ps[s], q = v & 0xFFFFu;
                    if (q == kPsDead || q == s) continue;
                    const uint32_t v2 = S.ps[q], q2 = v2 & 0xFFFFu;
                    if (q2 == kPsDead) {
                        S.ps[s] = kPsDead;
                        changed = 1;
                    } else if (q2 != q) {
                        S.ps[s] = q2 | (((v >> 16) + (v2 >> 16)) << 16);
                        changed = 1;
                    }
                }
                if (!__syncthreads_or(changed)) break;
            }
            // own exits: leaves of terminal chains that exit the ST inside the stream
            for (uint32_t s = tid; s < kFSlots; s += kFThreads) {
                if (s % kFTileCap >= S.tcnt[s / kFTileCap]) continue;
                if ((S.ps[s] & 0xFFFFu) != s || S.lleaf[s] != s || (S.lcnt[s] & kIncBit)) continue;
                const uint32_t e = S.fexit[s];
                if (e == kXFar) {
                    if (st0 + 0xFFFFFFFFull < N) S.fail = 1;   // an exit past 4 GiB inside the stream
                    continue;
                }
                if (st0 + e < N) {
                    const uint32_t i = atomicAdd(&S.n_ex, 1u);
                    if (i < kFExCap) S.ex[i] = st0 + e;
                    else S.fail = 1;
                }
            }
            __syncthreads();
            skip = S.fail != 0;
        }
        FT_MARK(10, wall_clock64());
        if (wv == 0) {
            if (skip) {
                fail_now();
            } else {
                // LOCAL: the distinct own exits
                const uint32_t n = S.n_ex;
                const uint64_t e = lane < n ? S.ex[lane] : 0ull;
                bool dup = false;
                for (uint32_t i = 0; i < n; ++i) {
                    const uint64_t o = readlane64(e, i);
                    dup = dup || (i < lane && o == e);
                }
                const bool keep = lane < n && !dup;
                const uint64_t km = __ballot(keep);
                if (keep) gput(P.blk(k) + kBEx + mbcnt64(km), gr(tag, e));
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) {
                    atomicAdd(&C[kCntFSurv], S.surv);
                    gput(P.R(kRLocal) + k, gr(tag, (uint64_t)__popcll(km)));
                }
                pub_local = true;
            }
        }

        // ---- F: every ST before is LOCAL; the fast table over this ST's entry keys
        FT_MARK(1, wall_clock64());
        if (wv == 0 && !skip) {
            uint32_t fsp = 0;
            const bool fok = f_wait_recent(P, k, lane, fsp);
            FT_MARK(7, fsp);
            if (!fok) {
                if (lane == 0) atomicAdd(&C[kCntFTimeout], 1u);
                skip = true;
                fail_now();
            } else {
                // keys: the own exits of the kFDepth STs before that land here (lanes
                // 16 d + i: exit i of ST k - 1 - d); a longer jump is a look-back miss
                uint64_t key = 0;
                bool has = false, inc = false;
                const uint32_t d = lane >> 4, i = lane & 15u;
                if (d < kFDepth && k >= d + 1u) {
                    const uint32_t m = k - 1u - d;
                    const uint32_t np = (uint32_t)(gval(gget(P.R(kRLocal) + m)) & 0xFFu);
                    if (i < np) {
                        const uint64_t *src = P.blk(m) + kBEx + i;
                        uint64_t g = gget(src);
                        for (uint32_t sp = 0; !gok(g, tag) && sp < 4096; ++sp) g = gget(src);
                        if (gok(g, tag)) {
                            key = gval(g);
                            has = key >= st0 && key < stE;
                        } else {
                            inc = true;                // should not happen: published before LOCAL
                        }
                    }
                }
                inc = __any(inc);
                bool live = false;
                uint64_t out = 0, cnt = 0, tl = 0;
                if (has) {
                    const uint32_t u = f_lookup(S, (uint32_t)(key - st0));
                    if (u != kNoSlot) {
                        const uint32_t v = S.ps[u], T = v & 0xFFFFu;
                        if (T != kPsDead) {
                            const uint32_t lf = S.lleaf[T];
                            const uint32_t e = S.fexit[lf];
                            if ((S.lcnt[T] & kIncBit) || e == kXFar) {
                                inc = true;            // ends in an incomplete header / too far: not here
                            } else {
                                live = true;
                                out = st0 + e;
                                cnt = (v >> 16) + (S.lcnt[T] & 0x7FFFu);
                                tl = st0 + S.soff[lf];
                            }
                        }
                    }
                }
                inc = __any(inc);
                // distinct live keys (the same offset can come from two exits)
                bool dup = false;
                uint64_t lm = __ballot(live);
                for (uint64_t b = lm; b;) {
                    const uint32_t l = (uint32_t)__ffsll((unsigned long long)b) - 1u;
                    b &= b - 1ull;
                    if (l < lane && readlane64(key, l) == key) dup = true;
                }
                const bool keep = live && !dup;
                const uint64_t km = __ballot(keep);
                const uint32_t nl = (uint32_t)__popcll(km);
                if (nl > kFLive) inc = true;
                if (keep && !inc) {
                    uint64_t *const b = P.blk(k) + kBFt + 4u * mbcnt64(km);
                    gput(b + 0, gr(tag, key));
                    gput(b + 1, gr(tag, out));
                    gput(b + 2, gr(tag, cnt));
                    gput(b + 3, gr(tag, tl));
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) gput(P.R(kRFt) + k, gr(tag, inc ? (uint64_t)kFtInc : (uint64_t)nl));
                pub_ft = true;
            }
        }

        // ---- B: the state entering this ST, then this ST's INCL
        FT_MARK(2, wall_clock64());
        if (wv == 0 && !skip) {
            uint64_t X, base, tail;
            uint32_t lsp = 0, win = 0;
            bool ok = f_lookback(P, k, lane, X, base, tail, lsp, win);
            FT_MARK(6, lsp);
            FT_MARK(5, win);
            FT_MARK(3, wall_clock64());
            uint32_t u = kNoSlot, cnt = 0, inc_end = 0;
            uint64_t nx = X, ntail = tail;
            if (ok && X < stE) {
                u = f_lookup(S, (uint32_t)(X - st0));
                if (u == kNoSlot) {
                    ok = false;                          // the true chain lands on no header
                } else {
                    const uint32_t v = S.ps[u], T = v & 0xFFFFu;
                    if (T == kPsDead) {
                        ok = false;                      // a protocol error ahead on the chain
                    } else {
                        const uint32_t lf = S.lleaf[T];
                        cnt = (v >> 16) + (S.lcnt[T] & 0x7FFFu);
                        if (S.lcnt[T] & kIncBit) {
                            inc_end = 1;                 // an incomplete trailing header
                            ok = k + 1 == P.n_st;
                            nx = st0 + S.fexit[lf];
                        } else if (S.fexit[lf] == kXFar) {
                            ok = false;
                        } else {
                            nx = st0 + S.fexit[lf];
                            ntail = st0 + S.soff[lf];
                        }
                    }
                }
            }
            if (ok && base + cnt > P.cap) ok = false;   // more frames than the list holds
            if (!ok) {
                skip = true;
                fail_now();
            } else {
                if (lane == 0) {
                    gput(P.R(kRInB) + k, gr(tag, base + cnt));
                    gput(P.R(kRInT) + k, gr(tag, ntail));
                    gput(P.R(kRInX) + k, gr(tag, nx));
                    S.X = X;
                    S.base = base;
                    S.tail = tail;
                    S.own_u = u;
                    S.own_cnt = cnt;
                    S.inc_end = inc_end;
                    S.nx = nx;
                }
            }
            if (lane == 0) S.fail = skip ? 1u : 0u;
        }
        __syncthreads();
        if (S.fail) continue;

        // ---- U: the true frames, their records, the unmask from LDS
        if (tid < kFTiles) S.tentry[tid] = 0xFFFFu;
        __syncthreads();
        if (tid == 0 && S.own_u != kNoSlot) {
            for (uint32_t s = S.own_u;;) {
                S.tentry[S.soff[s] >> 11] = S.soff[s];
                const uint16_t lk = S.link[s];
                if (lk == kNoLink) break;
                s = lk;
            }
        }
        __syncthreads();
        for (uint32_t t = wv; t < kFTiles; t += kFWaves) {
            uint32_t n = 0;
            if (lane == 0 && S.tentry[t] != 0xFFFFu) {
                uint32_t pos = S.tentry[t];
                const uint32_t tend = (t + 1u) * kTile;
                for (;;) {
                    const uint64_t a = st0 + pos;
                    if (a >= N || n >= kFTileCap) break;
                    Hdr h;
                    const uint32_t al = pos & ~15u;
                    const int r = parse_window(*reinterpret_cast<const u32x4 *>(S.bytes + al),
                                               *reinterpret_cast<const u32x4 *>(S.bytes + al + 16u), pos & 15u, N - a, h);
                    if (r <= 0) break;                   // the incomplete trailing header
                    const uint64_t pe = a + (uint64_t)r + h.plen;
                    FFrame f;
                    f.hdr = (uint16_t)pos;
                    f.hl = (uint8_t)r;
                    f.pad = 0;
                    f.key = h.key;
                    f.pe = (uint32_t)((pe < stE ? pe : stE) - st0);
                    S.u.fr[t * kFTileCap + n] = f;
                    ++n;
                    if (pe >= st0 + tend) break;
                    pos = (uint32_t)(pe - st0);
                }
                S.tcnt[t] = n;
            } else if (lane == 0) {
                S.tcnt[t] = 0;
            }
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t acc = 0;
            int32_t cov = -1;
            for (uint32_t t = 0; t < kFTiles; ++t) {
                S.fpre[t] = acc;
                S.fcov[t] = cov;
                const uint32_t n = S.tcnt[t];
                if (n) cov = (int32_t)(t * kFTileCap + n - 1u);
                acc += n;
            }
            S.fpre[kFTiles] = acc;
            S.nf = acc;
            if (acc != S.own_cnt) atomicAdd(&C[kCntFTimeout], 1u << 16);   // diagnostic: never expected
            // the frame covering the ST start: its header (never modified) from the stream
            S.hpo = S.hpe = 0;
            S.hkey = 0;
            if (S.tail != kNoTail) {
                const uint64_t q = S.tail;
                Hdr h;
                int r;
                if ((q & ~15ull) + 32u <= N) {           // the header's 32-B window in two loads
                    const uint64_t qa = q & ~15ull;
                    r = parse_window(gload16(wb + qa), gload16(wb + qa + 16u), (uint32_t)(q & 15u), N - q, h);
                } else {
                    r = parse_hdr([&](int i) -> uint32_t { return wire[q + i]; }, N - q, true, h);
                }
                if (r > 0) {
                    S.hpo = q + (uint64_t)r;
                    const uint64_t pe = S.hpo + h.plen;
                    S.hpe = pe < N ? pe : N;
                    S.hkey = h.key;
                }
            }
        }
        __syncthreads();
        const uint32_t nf = S.nf;
        const uint64_t base = S.base;
        for (uint32_t f = tid; f < nf; f += kFThreads) {
            uint32_t t = 0;
            while (t + 1u < kFTiles && S.fpre[t + 1u] <= f) ++t;
            const FFrame F = S.u.fr[t * kFTileCap + (f - S.fpre[t])];
            Hdr h;
            const uint32_t al = F.hdr & ~15u;
            const uint64_t a = st0 + F.hdr;
            (void)parse_window(*reinterpret_cast<const u32x4 *>(S.bytes + al),
                               *reinterpret_cast<const u32x4 *>(S.bytes + al + 16u), F.hdr & 15u, N - a, h);
            fws_frame_info fi;
            fi.hdr_off = a;
            fi.payload_len = h.plen;
            fi.key = h.key;
            fi.opcode = (uint8_t)h.opcode;
            fi.fin = (uint8_t)h.fin;
            fi.hdr_len = F.hl;
            fi.flags = (a + F.hl + h.plen > N) ? (uint8_t)FWS_FRAME_TRUNCATED : (uint8_t)0;
            const uint64_t *s64 = reinterpret_cast<const uint64_t *>(&fi);
            if (base + f >= P.cap) continue;
            uint64_t *d64 = reinterpret_cast<uint64_t *>(P.frames + base + f);
            d64[0] = s64[0];
            d64[1] = s64[1];
            d64[2] = s64[2];
        }
        const uint64_t hpo = S.hpo, hpe = S.hpe;
        const uint32_t hkey = S.hkey;
        for (uint32_t c = tid * 16u; c < kFS; c += kFThreads * 16u) {
            const uint64_t ca = st0 + c;
            if (ca >= N) break;
            const uint32_t t = c >> 11, n = S.tcnt[t], sb = t * kFTileCap;
            uint32_t lo = 0, hi = n;                 // frames of the tile with hdr <= c
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (S.u.fr[sb + mid].hdr <= c) lo = mid + 1u; else hi = mid;
            }
            const int32_t f = lo ? (int32_t)(sb + lo - 1u) : S.fcov[t];
            u32x4 m;
            if (f < 0) {
                m = f_region_mask(ca, hpo, hpe, hkey);
            } else {
                const FFrame F = S.u.fr[f];
                m = f_region_mask(ca, st0 + F.hdr + F.hl, st0 + F.pe, F.key);
            }
            for (uint32_t i = lo; i < n; ++i) {
                const FFrame F = S.u.fr[sb + i];
                if (F.hdr >= c + 16u) break;
                m |= f_region_mask(ca, st0 + F.hdr + F.hl, st0 + F.pe, F.key);
            }
            if (m.x | m.y | m.z | m.w) {
                const u32x4 v = *reinterpret_cast<const u32x4 *>(S.bytes + c) ^ m;
                if (ca + 16u <= N) {
                    gstore16<true>(wb + ca, v);
                } else {
                    const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
                    for (uint32_t i = 0; ca + i < N; ++i) wire[ca + i] = (uint8_t)(vw[i >> 2] >> (8u * (i & 3u)));
                }
            }
        }
        FT_MARK(4, wall_clock64());
        if (tid == 0) {
            gput(P.R(kRDone) + k, gr(tag, 1u));
            if (k + 1u == P.n_st) {
                // the result (OnRecvData's end state on this buffer)
                const uint64_t nfr = base + S.own_cnt;
                fws_decode_result *const r = P.res;
                r->status = FWS_OK;
                r->n_frames = (uint32_t)nfr;
                r->err_off = 0;
                const uint64_t pos = S.nx;
                if (S.inc_end) {
                    r->consumed = pos;
                    r->carry_unread = 0;
                    r->carry_hdr_len = (uint32_t)(N - pos);
                } else {
                    r->consumed = N;
                    r->carry_unread = pos > N ? pos - N : 0;
                    r->carry_hdr_len = 0;
                }
                r->n_survivors = cget(&C[kCntFSurv]);
                __hip_atomic_store(&C[kCntFrames], (uint32_t)nfr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

}  // namespace fwsk

// ------------------------------------------------------------------ host side
using namespace fwsk;

// tuning / test hook: 0 = the multi-launch path only (default: k_fused measured
// slower), 1 = k_fused first for streams of at least kFusedMin
// bytes, 2 = for every stream of at least 16 bytes (tests)
static int g_fused = 0;
extern "C" __attribute__((visibility("default"))) int fws_internal_set_fused(int mode) {
    const int old = g_fused;
    if (mode >= 0 && mode <= 2) g_fused = mode;
    return old;
}
// test hook: per-ST phase clocks of the last k_fused (tools/prof_fused.py)
static int g_trace_on = 0;
static uint64_t *g_trace = nullptr;
static uint64_t g_trace_cap = 0, g_trace_n = 0;
extern "C" __attribute__((visibility("default"))) int fws_internal_fused_trace(int on) {
    g_trace_on = on != 0;
    return 0;
}
// copies min(n, STs of the last traced call) records of kFTraceW words; returns the count
extern "C" __attribute__((visibility("default"))) long long fws_internal_fused_trace_read(uint64_t *out, long long n) {
    if (!g_trace || n <= 0) return 0;
    const uint64_t m = (uint64_t)n < g_trace_n ? (uint64_t)n : g_trace_n;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpy(out, g_trace, m * kFTraceW * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return (long long)m;
}
bool fws_fused_enabled(uint64_t N) { return g_fused == 2 ? N >= 16 : g_fused == 1 && N >= kFusedMin; }

int fws_fused_ensure(fws_gpu_ctx *ctx, uint64_t N) {
    fws_decode_ws &d = ctx->dec;
    const uint64_t n_st = (N + kFS - 1) / kFS;
    if (n_st <= d.fmax_st) return 0;
    if (d.fpub) (void)hipFree(d.fpub);
    d.fpub = nullptr;
    d.fmax_st = 0;
    const uint64_t bytes = n_st * kFPubWords * sizeof(uint64_t);
    hipError_t e = hipMalloc((void **)&d.fpub, bytes);
    if (e == hipSuccess) e = hipMemset(d.fpub, 0, bytes);   // no tag is 0
    if (e != hipSuccess) return fws_hip_status(e);
    d.fmax_st = n_st;
    return 0;
}

const uint64_t *fws_fused_done(const fws_gpu_ctx *ctx) {
    return ctx->dec.fpub ? ctx->dec.fpub + (uint64_t)kRDone * ctx->dec.fmax_st : nullptr;
}

int fws_launch_fused(fws_gpu_ctx *ctx, uint8_t *wire, uint64_t N, fws_frame_info *frames, uint32_t cap,
                     fws_decode_result *res, hipStream_t s) {
    fws_decode_ws &d = ctx->dec;
    const uint64_t n_st = (N + kFS - 1) / kFS;
    if (n_st > d.fmax_st || n_st >= (1ull << 31)) return FWS_ERR_INTERNAL;
    if (d.fcus == 0) {                               // per context: its device's CU count
        int cus = 0;
        hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device);
        if (e != hipSuccess) return fws_hip_status(e);
        d.fcus = (uint32_t)cus;
    }
    d.fepoch = (d.fepoch + 1u) & 0xFFFFFFu;
    if (d.fepoch == 0) d.fepoch = 1;
    FusedParams P;
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
            if (hipMalloc((void **)&g_trace, n_st * kFTraceW * 8) != hipSuccess) return FWS_ERR_INTERNAL;
            g_trace_cap = n_st;
        }
        P.trace = g_trace;
        g_trace_n = n_st;
    }
    const uint64_t g = (uint64_t)d.fcus * kFBlocksPerCu;
    hipLaunchKernelGGL(k_fused, dim3((unsigned)(n_st < g ? n_st : g)), dim3(kFThreads), 0, s, P);
    return fws_hip_status(hipGetLastError());
}
