// merge_kernels.hip -- second half of fws_gpu_decode_stream: from k_scan's
// per-tile survivors to the frame list, the result and the unmask plan in
// three launches, with no grid barrier (no launch depends on co-residency).
//
// OnRecvData's frame loop (net/w_socket.h:543-769) is a chain: the next
// header starts at this header's exit (hdr_off + hdr_len + payload_len,
// w_socket.h:750-764). k_scan (decode_kernels.hip) left, per 2 KiB tile, the
// offsets whose header chain reaches the tile end ("survivors"): every true
// header plus a few random offsets.
//
//  k_merge  one workgroup per super tile (ST = 256 tiles = 512 KiB). First
//           the tiles k_scan left (kDenseTile: frames under ~32 B) are
//           scanned with dense_tile() (scan_common.h). Then it loads the ST's
//           survivors (offset order), links each to the survivor at its exit
//           inside the ST (search in the exit's tile, in LDS) and
//           pointer-jumps (Wyllie) so every survivor knows the tail of its
//           chain in the ST, the frames up to that tail, and how the chain
//           leaves the ST: EXIT (into a later ST), END (at or past the stream
//           end), DEAD (the exit is not a header: a protocol error or a false
//           chain) or INC (an incomplete header at the stream end). EXIT
//           tails go to a global list; the ST's survivors are also written as
//           one table (slot id, next, tail, frames to it) for k_emit. A super
//           tile with 2049-8192 survivors (frames of ~70-250 B) takes
//           merge_mid (the same steps in LDS, in-place jumping on one word
//           per survivor); above that, the big-ST path over global scratch.
//  k_link   one thread per EXIT tail: the survivor its exit lands on (the
//           tile's slots, one batch of loads) and next(tail) = the tail of
//           that survivor's chain; marks every next() target in a bitmap.
//  last WG  the k_link workgroup that finishes last (atomic ticket) resolves
//           the path from the header at offset 0 over the marked tails,
//           compacted into LDS. The path's tails are the greatest fixpoint of
//           K = {root's tail} U next(K): offsets strictly increase along next,
//           so a false tail has a finite chain of predecessors and drops out
//           after a few rounds (an input that keeps one alive for 64 rounds
//           is walked serially from the root instead). Each landing survivor
//           on the path is its ST's entry; a scan over the STs gives every
//           ST's first frame index. The terminal is finished with
//           ParseFrameHdr's rules (w_socket.h:435-524): error walk, carry-out,
//           fws_decode_result. Workspace limits (k_scan's survivor spill, the
//           tail list) end the decode with FWS_ERR_CAPACITY in the result.
//  k_emit   one workgroup per ST with an entry: marks the entry's chain
//           (the survivors at or after it with its tail when their frame
//           count is the entry's, else one survivor per depth -- the only one
//           at its depth or next() of the one above -- else pointer doubling)
//           and writes fws_frame_info in stream order and the unmask plan:
//           unit_first[u] = the frame whose span [hdr_off, next hdr_off)
//           holds stream byte 4 KiB * u (k_unmask_stream, unmask_kernels.hip).
//
// Every global access on these paths is metadata (about 1 survivor per KiB of
// stream); the kernels are latency-bound, so loads are issued in batches of
// independent addresses before their uses.
#include "scan_common.h"

namespace fwsk {

// tiles per super tile: kStTiles (1 MiB), halved down to kStTilesMin for a
// stream too short to give kStTarget super tiles (the host picks it per call,
// MergeParams::st_tiles; LDS tables are sized for kStTiles). Streams under
// 512 MiB (C2 / C3: 256 MiB) get 512 KiB super tiles as before; the C5 stream
// (4 GiB) gets 4,096 super tiles of 1 MiB instead of 8,192 of 512 KiB, so
// k_merge's three workgroups per CU take 6 rounds of its latency chain, not 11.
#ifndef FWS_ST_TILES
#define FWS_ST_TILES 512                                // (A/B builds: make exp EXP_DEFS=-DFWS_ST_TILES=256)
#endif
constexpr uint32_t kStTiles = FWS_ST_TILES;
#ifndef FWS_ST_TILES_MIN
#define FWS_ST_TILES_MIN 16
#endif
constexpr uint32_t kStTilesMin = FWS_ST_TILES_MIN;   // 16: the 200,000 x 64 B stream 0.0696 -> 0.067 ms (32 KiB super tiles)
constexpr uint64_t kStTarget = 512;
constexpr uint32_t kStCap = 2048;                   // survivors of one ST in LDS
constexpr int kMThreads = 512;
constexpr int kMWaves = kMThreads / 64;
constexpr uint32_t kPer = kStCap / kMThreads;       // survivors per thread: i = kPer * tid + j
constexpr uint32_t kWaveJump = 512;                 // k_merge: one wavefront pointer-jumps up to this many
constexpr uint32_t kTailRun = 16;                   // EXIT tails of one super tile in its own tail-list run
#ifndef FWS_LAND_WAVE
#define FWS_LAND_WAVE 1                               // A/B: 0 = one thread per tail, stage slots only
#endif
constexpr uint32_t kLandCap = 256;                  // k_merge: EXIT tails whose landing survivor it looks up
#ifndef FWS_LAND_WAVE_MAX
#define FWS_LAND_WAVE_MAX 24                          // A/B builds: 7 = one tail per idle wave (r04)
#endif
constexpr uint32_t kLandWaveMax = FWS_LAND_WAVE_MAX;  // up to this many: a wavefront per tail (7 idle waves)
constexpr uint32_t kTailCapMax = 1u << 18;          // LDS bitmap of the path pruning
constexpr uint32_t kCompCap = 32768;                // tails that are some tail's next (+ the root's)
constexpr uint32_t kMaxPruneRounds = 64;
constexpr uint64_t kUnit = 4096;                    // stream bytes per unmask plan unit

// in-ST next of a survivor: an LDS index, or how the chain leaves the ST
constexpr uint16_t kNxInc = 0xFFFC, kNxDead = 0xFFFD, kNxEnd = 0xFFFE, kNxExit = 0xFFFF;
constexpr uint32_t kKindExit = 0, kKindEnd = 1, kKindDead = 2, kKindInc = 3;
constexpr uint32_t kGTerm = 0xFFFFFFF0u;            // next(tail) >= kGTerm: the path ends (kGTerm | kind)
constexpr uint16_t kCTerm = 0xFFFF;

#ifdef FWS_SCAN_PROF
// phase clocks (100 MHz wall clock, summed over workgroups) for tools/prof_scan.py
__device__ unsigned long long g_merge_prof[32];
// per-workgroup timestamps (tools/prof_merge_trace.py): [workgroup % kTraceWg][mark]
constexpr uint32_t kTraceWg = 1024;
__device__ unsigned long long g_merge_trace[kTraceWg * 32];
#define MP_START(slot)                                                              \
    do {                                                                            \
        if (threadIdx.x == 0) g_merge_trace[(blockIdx.x % kTraceWg) * 32 + (slot)] = wall_clock64(); \
    } while (0)
#define MP_T0() const uint64_t mp_t0 = wall_clock64()
#define MP_INIT() uint64_t mp_t = wall_clock64()
#define MP_MARK(k)                                                                  \
    do {                                                                            \
        if (threadIdx.x == 0) {   /* a plain store: no same-address atomic queue */ \
            const uint64_t now = wall_clock64();                                    \
            g_merge_trace[(blockIdx.x % kTraceWg) * 32 + (k)] = now;                \
            mp_t = now;                                                             \
        }                                                                           \
    } while (0)
#define MP_ADD(k, v) do { } while (0)          /* same-address atomics would queue behind each other */
#define MP_SPAN(k0, k1) do { } while (0)
#define MP_VAL(k, v)                                                                \
    do {                                                                            \
        if (threadIdx.x == 0) g_merge_trace[(blockIdx.x % kTraceWg) * 32 + (k)] = (v); \
    } while (0)
#else
#define MP_VAL(k, v) do { } while (0)
#define MP_START(slot) do { } while (0)
#define MP_T0() do { } while (0)
#define MP_INIT() do { } while (0)
#define MP_MARK(k) do { } while (0)
#define MP_ADD(k, v) do { } while (0)
#define MP_SPAN(k0, k1) do { } while (0)
#endif

// fws_node_res::kind = kKind* | kBigBit (tail / ent are slot ids, not ST-local indices)
constexpr uint32_t kBigBit = 4u;
__device__ __forceinline__ uint32_t res_kind(const fws_node_res &r) { return r.kind & 3u; }

__device__ __forceinline__ uint32_t kind_of(uint16_t code) {
    return code == kNxExit ? kKindExit : code == kNxEnd ? kKindEnd : code == kNxDead ? kKindDead : kKindInc;
}

// big-ST path: in-ST next as a slot id, or how the chain leaves the ST
constexpr uint32_t kBgInc = 0xFFFFFFFCu, kBgDead = 0xFFFFFFFDu, kBgEnd = 0xFFFFFFFEu, kBgExit = 0xFFFFFFFFu;
__device__ __forceinline__ uint32_t bg_kind(uint32_t code) {
    return code == kBgExit ? kKindExit : code == kBgEnd ? kKindEnd : code == kBgDead ? kKindDead : kKindInc;
}
// relaxed agent-scope accesses: coherent in L2 across the waves of a workgroup
__device__ __forceinline__ uint32_t gld(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gst(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct MergeParams {
    const uint8_t *wire;
    uint64_t N;
    uint32_t n_tiles;
    uint32_t n_st;
    uint32_t st_tiles;                               // tiles per super tile (a power of two <= kStTiles)
    uint32_t st_shift;                               // log2 of the super tile's bytes
    const fws_frame_info *stage_info;
    const fws_frame_info *spill_info;
    uint32_t *tile_count;                            // k_merge rewrites the tiles k_scan left (kDenseTile)
    uint32_t *tile_spill;
    fws_frame_info *spill_w;                         // = spill_info, for dense_tile()
    uint32_t s_cap;                                  // spill capacity
    uint32_t spill_base;                             // n_tiles * kSlots: first slot id of the spill area
    uint32_t tail_cap;
    uint32_t *counters;
    fws_node_res *nres;
    fws_tail_rec *tails;
    uint32_t *gnx;
    uint64_t *tpk;                                   // [2 * tail_cap] tail_pack (k_link -> its last workgroup)
    uint32_t *tmark;                                 // tail-target bitmap (tail_cap / 32 + 1 words)
    uint32_t *comp;                                  // [kCompCap] compact index -> tail index
    fws_st_node *st_nodes;                           // [n_st][kStCap]
    uint32_t *st_n;
    uint32_t *st_nt;                                 // EXIT tails in the ST's own run (0: overflow area)
    uint32_t *st_entry;                              // local index of the ST's entry, or kNone
    uint32_t *st_fbase;
    fws_frame_info *frames;
    uint32_t cap;
    fws_decode_result *res;
    uint8_t *utf8_ok;                                // optional: preset per frame (TEXT, FIN, complete)
    uint32_t *unit_first;                            // unmask plan (fws_plan_ws), stream space
    uint64_t n_units;                                // ceil(N / kUnit), clamped to the plan's capacity
    uint32_t force_big;                              // test hook: every ST on the big-ST path, and the
                                                     //   path resolve on its global-table branches
    uint32_t *zero_next;                             // the next call's counter set (k_emit zeroes it)
    uint32_t *bg_nx, *bg_wt, *bg_lref, *bg_ptr, *bg_sc, *bg_mark;   // big-ST scratch [max_nodes]
    uint64_t max_nodes;

    __device__ __forceinline__ bool big(uint32_t n) const { return force_big || n > kStCap; }
    // the record of a chain's tail survivor in ST s (fws_node_res::tail of a non-EXIT kind)
    __device__ __forceinline__ uint32_t tail_sid(uint32_t s, const fws_node_res &r) const {
        return (r.kind & kBigBit) ? r.tail : st_nodes[(uint64_t)s * kStCap + r.tail].sid;
    }
    __device__ __forceinline__ const fws_frame_info *tail_rec(uint32_t s, const fws_node_res &r) const {
        return rec(tail_sid(s, r));
    }

    // slot id of survivor r of tile t (stage slots, or the tile's spill run)
    __device__ __forceinline__ uint32_t sid(uint32_t t, uint32_t sp, uint32_t r) const {
        return sp == kNone ? t * kSlots + r : spill_base + sp + r;
    }
    __device__ __forceinline__ const fws_frame_info *rec(uint32_t id) const {
        return id < spill_base ? stage_info + id : spill_info + (id - spill_base);
    }
    // slot id of the survivor at offset x (x < N), or kTermDead. A tile's <= 8
    // stage slots are read in one batch; a spilled (dense) tile is searched.
    __device__ __forceinline__ uint32_t find_node(uint64_t x) const {
        const uint32_t t = (uint32_t)(x / kTile);
        const uint32_t n = tile_count[t], sp = tile_spill[t];
        // (loading the 8 slots with the count, unconditionally, measured slower in k_link)
        if (sp == kNone) {
            uint64_t o[kSlots];
#pragma unroll
            for (uint32_t r = 0; r < kSlots; ++r) o[r] = r < n ? stage_info[t * kSlots + r].hdr_off : ~0ull;
            uint32_t hit = kTermDead;
#pragma unroll
            for (uint32_t r = 0; r < kSlots; ++r) hit = o[r] == x ? t * kSlots + r : hit;
            return hit;
        }
        uint32_t lo = 0, hi = n;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (rec(sid(t, sp, mid))->hdr_off < x) lo = mid + 1; else hi = mid;
        }
        return (lo < n && rec(sid(t, sp, lo))->hdr_off == x) ? sid(t, sp, lo) : kTermDead;
    }
    // unit_first for frame f spanning stream bytes [h, e) (e = the next frame's
    // header; the last frame < lim spans to the end of the stream)
    // a frame as written to the output: the record, and its UTF-8 flag preset
    __device__ __forceinline__ void put_frame(uint32_t f, const fws_frame_info &fi) const {
        frames[f] = fi;
        if (utf8_ok)
            utf8_ok[f] = fi.opcode == 1u && fi.fin && !(fi.flags & FWS_FRAME_TRUNCATED) &&
                         fi.hdr_off + fi.hdr_len + fi.payload_len <= N;
    }
    __device__ __forceinline__ void plan_units(uint32_t f, uint64_t h, uint64_t e, bool last) const {
        const uint64_t ue = last ? n_units : ((e + kUnit - 1) / kUnit < n_units ? (e + kUnit - 1) / kUnit : n_units);
        for (uint64_t u = (h + kUnit - 1) / kUnit; u < ue; ++u) unit_first[u] = f;
    }
};

__device__ __forceinline__ uint32_t ld_acq(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_acq64(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gst64(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    for (int i = 0; i < kMWaves; ++i) {
        off += (i < w) ? sred[i] : T(0);
        tot += sred[i];
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

// The tail list: super tile s writes its k EXIT tails to its own run
// [s * kTailRun, s * kTailRun + k) when k <= kTailRun (every C2 / C3 / C5
// super tile), else to a run of the overflow area past n_st * kTailRun, taken
// with one atomic. (One atomic per super tile on one counter word queued 513
// workgroups behind each other: k_merge 18 -> see DESIGN 4.3.) Returns the
// run's first tail index, or kNone when the overflow area is full (the decode
// ends with FWS_ERR_CAPACITY).
__device__ uint32_t reserve_tails(const MergeParams &P, uint32_t s, uint32_t k) {
    if (k <= kTailRun) {
        P.st_nt[s] = k;
        return s * kTailRun;
    }
    P.st_nt[s] = 0;
    const uint32_t fixed = P.n_st * kTailRun, room = P.tail_cap - fixed;
    const uint32_t off = atomicAdd(&P.counters[kCntTails], k);
    if (off > room || room - off < k) {
        atomicOr(&P.counters[kCntFallback], 1u);
        return kNone;
    }
    return fixed + off;
}

// ------------------------------------------------------------------ k_merge
constexpr uint32_t kDenseWaves = 4;                 // k_merge wavefronts running dense_tile()
constexpr uint32_t kMidCap = 6144;                  // big super tiles merged / emitted in LDS (else global scratch;
                                                    //   6144, not 8192: k_merge keeps 3 workgroups per CU at 512 tiles)
constexpr uint16_t kDenseTile16 = (uint16_t)kDenseTile;   // tcnt's mark (real tile counts are <= kTile)
struct MergeLds {
    uint16_t tcnt[kStTiles];                         // (u16: three workgroups per CU at 512 tiles)
    uint32_t tsp[kStTiles];
    uint32_t tbase[kStTiles];
    union {
        uint16_t boff[kMidCap];                      // mid path: tile-local offset of survivor i
        struct {                                     // LDS path: EXIT tail lref -> its exit (the
            uint64_t texit[kLandCap];                //   landing lookups) -> slot id of the survivor
            uint32_t tland[kLandCap];                //   there, kTermDead, or kNone
        };
    };
    union {
        struct {
            union {
                uint32_t off[kStCap];                // hdr_off - ST start (the exit search)
                uint32_t lref[kStCap];               // then: EXIT tail's index in the ST's tail run
            };
            uint16_t nx[kStCap];
            uint8_t wt[kStCap];                      // 1: a frame; 0: incomplete header
            uint32_t pw[kStCap];                     // Wyllie pointer (tails point to themselves) |
                                                     //   frames from i up to it (exclusive) << 16
        };
        ScanWaveLds dw[kDenseWaves];                 // first: the tiles k_scan left (dense_tile)
        uint32_t bw[kMidCap];                        // mid path: ptr | frames << 16 | kind << 29 | frame bit << 31
    };
    uint32_t red32[kMWaves];
    uint32_t n_tail, tail_base;
};
// (LDS is allocated in 512-B blocks: 54,576 B at kMidCap 8192 rounded to three
// blocks too many, and C2 / C3's 513 super tiles took a second round, +4 %)
static_assert(3u * ((sizeof(MergeLds) + 1024u + 511u) / 512u * 512u) <= 160u * 1024u,
              "three k_merge workgroups per CU (513 super tiles of C2 / C3), with 1 KB for its other LDS");
static_assert(kStTiles <= (uint32_t)kMThreads, "one thread per tile of a super tile");

// Slot id of survivor i of ST s (tile by a search of the ST's tile prefix in LDS).
__device__ __forceinline__ uint32_t st_sid(const MergeParams &P, const MergeLds &L, uint32_t t0, uint32_t i) {
    uint32_t lo = 0, hi = kStTiles;                  // last tile with tbase <= i
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (L.tbase[mid] <= i) lo = mid; else hi = mid;
    }
    return P.sid(t0 + lo, L.tsp[lo], i - L.tbase[lo]);
}

// The big-ST path of k_merge: the LDS path's steps for a super tile whose n
// survivors do not fit the LDS tables, over global scratch indexed by slot
// id. Same outputs (fws_node_res with kBigBit: tails and entries are slot
// ids; EXIT tails in the global list), no table for k_emit (it walks the
// scratch the same way).
__device__ void merge_big(const MergeParams &P, MergeLds &L, uint32_t s, uint32_t n) {
    const uint32_t tid = threadIdx.x, t0 = s * P.st_tiles;
    const uint64_t st_end = (uint64_t(s) + 1u) << P.st_shift;
    uint32_t *const p0 = P.bg_ptr, *const p1 = P.bg_ptr + P.max_nodes;
    uint32_t *const c0 = P.bg_sc, *const c1 = P.bg_sc + P.max_nodes;
    // in-ST next of every survivor: the survivor at its exit (search in the exit's tile)
    for (uint32_t i = tid; i < n; i += kMThreads) {
        const uint32_t id = st_sid(P, L, t0, i);
        const fws_frame_info r = *P.rec(id);
        const uint64_t x = exit_of(r);
        uint32_t v;
        if (!r.hdr_len) v = kBgInc;
        else if (x >= P.N) v = kBgEnd;
        else if (x >= st_end) v = kBgExit;
        else {
            v = P.find_node(x);
            if (v == kTermDead) v = kBgDead;
        }
        const uint32_t wt = r.hdr_len ? 1u : 0u;
        const bool tail = v >= kBgInc;
        gst(P.bg_nx + id, v);
        gst(P.bg_wt + id, wt);
        gst(p0 + id, tail ? id : v);
        gst(c0 + id, tail ? 0u : wt);
        if (v == kBgExit) gst(P.bg_lref + id, atomicAdd(&L.n_tail, 1u));
    }
    __syncthreads();
    if (tid == 0) L.tail_base = reserve_tails(P, s, L.n_tail);   // the ST's run of the tail list
    // pointer jumping over slot ids: every survivor -> its chain's tail, frame counts
    uint32_t *pc = p0, *pn = p1, *sc = c0, *sn = c1;
    for (;;) {
        int changed = 0;
        for (uint32_t i = tid; i < n; i += kMThreads) {
            const uint32_t id = st_sid(P, L, t0, i);
            const uint32_t p = gld(pc + id), q = gld(pc + p);
            const uint32_t a = gld(sc + id);
            if (p != q) {
                gst(pn + id, q);
                gst(sn + id, a + gld(sc + p));
                changed = 1;
            } else {
                gst(pn + id, p);
                gst(sn + id, a);
            }
        }
        uint32_t *t = pc; pc = pn; pn = t;
        t = sc; sc = sn; sn = t;
        if (!__syncthreads_or(changed)) break;
    }
    const uint32_t tb = L.tail_base;
    if (tb == kNone) return;
    for (uint32_t i = tid; i < n; i += kMThreads) {
        const uint32_t id = st_sid(P, L, t0, i);
        const uint32_t t = gld(pc + id);
        const uint32_t kind = bg_kind(gld(P.bg_nx + t));
        const uint32_t cnt = gld(sc + id) + gld(P.bg_wt + t);
        const uint32_t ref = kind == kKindExit ? tb + gld(P.bg_lref + t) : t;
        P.nres[id] = fws_node_res{ref, cnt, id, kind | kBigBit};
        if (gld(P.bg_nx + id) == kBgExit) {
            const uint64_t x = exit_of(*P.rec(id));
            P.tails[tb + gld(P.bg_lref + id)] = fws_tail_rec{x, id, kNone, (uint32_t)(x >> P.st_shift), 0u};
        }
    }
}

// A super tile with kStCap < n <= kMidCap survivors (frames of ~70 B and up):
// the big path's outputs (fws_node_res with kBigBit; bg_ptr[id] = in-ST next as
// a local index or itself for a tail, bg_wt, bg_nx = exit kind, bg_lref) with
// the chain work in LDS: the exit search over tile-local offsets (boff) and
// in-place pointer jumping on one word per survivor (a pair read or written
// as one 32-bit word stays consistent, so rounds need no second buffer).
// Global loads are issued four survivors at a time.
constexpr uint32_t kMidB = 4;
__device__ void merge_mid(const MergeParams &P, MergeLds &L, uint32_t s, uint32_t n) {
    const uint32_t tid = threadIdx.x, t0 = s * P.st_tiles;
    const uint64_t st0 = uint64_t(s) << P.st_shift, st_end = st0 + (1ull << P.st_shift);
    MP_INIT();
    // pass 1: tile-local offsets
    for (uint32_t base = tid; base < n; base += kMidB * kMThreads) {
        uint32_t id[kMidB];
        uint64_t off[kMidB];
#pragma unroll
        for (uint32_t b = 0; b < kMidB; ++b) {
            const uint32_t i = base + b * kMThreads;
            id[b] = st_sid(P, L, t0, i < n ? i : base);
        }
#pragma unroll
        for (uint32_t b = 0; b < kMidB; ++b) off[b] = P.rec(id[b])->hdr_off;
#pragma unroll
        for (uint32_t b = 0; b < kMidB; ++b) {
            const uint32_t i = base + b * kMThreads;
            if (i < n) L.boff[i] = (uint16_t)(off[b] % kTile);
        }
    }
    __syncthreads();
    MP_MARK(18);
    // pass 2: in-ST next (the survivor at the exit, searched in the exit's tile)
    for (uint32_t base = tid; base < n; base += kMidB * kMThreads) {
        uint32_t id[kMidB];
        fws_frame_info r[kMidB];
#pragma unroll
        for (uint32_t b = 0; b < kMidB; ++b) {
            const uint32_t i = base + b * kMThreads;
            id[b] = st_sid(P, L, t0, i < n ? i : base);
        }
#pragma unroll
        for (uint32_t b = 0; b < kMidB; ++b) r[b] = *P.rec(id[b]);
#pragma unroll
        for (uint32_t b = 0; b < kMidB; ++b) {
            const uint32_t i = base + b * kMThreads;
            if (i >= n) continue;
            const uint64_t x = exit_of(r[b]);
            uint32_t kind = 0, nx = i;
            bool tail = true;
            if (!r[b].hdr_len) kind = kKindInc;
            else if (x >= P.N) kind = kKindEnd;
            else if (x >= st_end) kind = kKindExit;
            else {
                const uint32_t tl = (uint32_t)((x - st0) / kTile), xo = (uint32_t)(x % kTile);
                uint32_t lo = L.tbase[tl], hi = lo + L.tcnt[tl];
                while (lo < hi) {                    // first survivor of the tile at or past xo
                    const uint32_t mid = (lo + hi) >> 1;
                    if (L.boff[mid] < xo) lo = mid + 1; else hi = mid;
                }
                if (lo < L.tbase[tl] + L.tcnt[tl] && L.boff[lo] == xo) {
                    nx = lo;
                    tail = false;
                } else {
                    kind = kKindDead;
                }
            }
            const uint32_t wt = r[b].hdr_len ? 1u : 0u;
            L.bw[i] = nx | (tail ? 0u : wt << 16) | (kind << 29) | (wt << 31);
            P.bg_ptr[id[b]] = nx;
            P.bg_wt[id[b]] = wt;
            P.bg_nx[id[b]] = tail ? kind : kNone;
            if (tail && kind == kKindExit) P.bg_lref[id[b]] = atomicAdd(&L.n_tail, 1u);
        }
    }
    __syncthreads();
    MP_MARK(19);
    if (tid == 0) L.tail_base = reserve_tails(P, s, L.n_tail);   // the ST's run of the tail list
    // pointer jumping in place: ptr and frame count move together in one word
    for (;;) {
        int changed = 0;
        for (uint32_t i = tid; i < n; i += kMThreads) {
            const uint32_t w = L.bw[i], p = w & 0xFFFFu;
            if (p == i) continue;
            const uint32_t wp = L.bw[p], q = wp & 0xFFFFu;
            if (q == p) continue;
            const uint32_t c = ((w >> 16) & 0x1FFFu) + ((wp >> 16) & 0x1FFFu);
            L.bw[i] = (w & 0xE0000000u) | q | (c << 16);
            changed = 1;
        }
        if (!__syncthreads_or(changed)) break;
    }
    MP_MARK(20);
    const uint32_t tb = L.tail_base;
    if (tb == kNone) return;
    for (uint32_t base = tid; base < n; base += kMidB * kMThreads) {
        uint32_t id[kMidB], tid_[kMidB], lr[kMidB], own[kMidB];
        uint64_t x[kMidB];
#pragma unroll
        for (uint32_t b = 0; b < kMidB; ++b) {
            const uint32_t i = base + b * kMThreads < n ? base + b * kMThreads : base;
            id[b] = st_sid(P, L, t0, i);
            tid_[b] = st_sid(P, L, t0, L.bw[i] & 0xFFFFu);
        }
#pragma unroll
        for (uint32_t b = 0; b < kMidB; ++b) {
            lr[b] = P.bg_lref[tid_[b]];
            own[b] = P.bg_lref[id[b]];
            x[b] = exit_of(*P.rec(id[b]));
        }
#pragma unroll
        for (uint32_t b = 0; b < kMidB; ++b) {
            const uint32_t i = base + b * kMThreads;
            if (i >= n) continue;
            const uint32_t w = L.bw[i], t = w & 0xFFFFu, wt_t = L.bw[t];
            const uint32_t kind = (wt_t >> 29) & 3u;
            const uint32_t cnt = ((w >> 16) & 0x1FFFu) + (wt_t >> 31);
            const uint32_t ref = kind == kKindExit ? tb + lr[b] : tid_[b];
            P.nres[id[b]] = fws_node_res{ref, cnt, id[b], kind | kBigBit};
            if (t == i && kind == kKindExit)
                P.tails[tb + own[b]] = fws_tail_rec{x[b], id[b], kNone, (uint32_t)(x[b] >> P.st_shift), 0u};
        }
    }
    __syncthreads();
    MP_MARK(21);
}

// Pointer jumping in place by one wavefront over pw[0, n), n <= 64 J: every
// survivor -> its chain's tail, with frame counts (pointer and count move
// together in one word). One synchronous round = every read of the round
// before any write; the reads are unconditional (in-bounds words past n,
// unused) so the J reads issue back to back under one wait, twice per round;
// a wave's LDS operations are ordered, so no barrier per round.
template <uint32_t J>
__device__ __forceinline__ void wave_jump(uint32_t *pw, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63;
    for (;;) {
        uint32_t w[J], wp[J];
#pragma unroll
        for (uint32_t j = 0; j < J; ++j) w[j] = pw[lane + 64u * j];
#pragma unroll
        for (uint32_t j = 0; j < J; ++j) wp[j] = pw[w[j] & (kStCap - 1u)];
        bool ch = false;
#pragma unroll
        for (uint32_t j = 0; j < J; ++j) {
            const uint32_t i = lane + 64u * j;
            if (i < n && (wp[j] & 0xFFFFu) != (w[j] & 0xFFFFu)) {
                pw[i] = (wp[j] & 0xFFFFu) | (((w[j] >> 16) + (wp[j] >> 16)) << 16);
                ch = true;
            }
        }
        wave_sync();
        if (!__any(ch)) break;
    }
}

__global__ __launch_bounds__(kMThreads) void k_merge(MergeParams P) {
    __shared__ MergeLds L;
    const uint32_t s = blockIdx.x, tid = threadIdx.x;
    uint32_t *const C = P.counters;
    MP_START(30);
    MP_T0();
    MP_INIT();
    // the tail-target bitmap k_link sets
    for (uint64_t w = (uint64_t)s * kMThreads + tid; w < P.tail_cap / 32u + 1u; w += (uint64_t)gridDim.x * kMThreads)
        P.tmark[w] = 0u;
    if (s >= P.n_st) return;
    const uint32_t t0 = s * P.st_tiles;
    const uint64_t st0 = uint64_t(s) << P.st_shift, st_end = st0 + (1ull << P.st_shift);

    // survivors per tile -> ST-local numbering
    uint32_t c = 0, sp = kNone;
    if (tid < P.st_tiles && t0 + tid < P.n_tiles) {
        c = P.tile_count[t0 + tid];
        sp = P.tile_spill[t0 + tid];
    }
    if (__syncthreads_or(c == kDenseTile)) {
        // tiles k_scan left (frames under ~32 B): dense_tile() on kDenseWaves wavefronts,
        // survivors to spill runs; the counts go back to tile_count / tile_spill for k_link
        // and k_emit (find_node)
        if (tid < kStTiles) {
            L.tcnt[tid] = (uint16_t)c;               // (kDenseTile -> kDenseTile16)
            L.tsp[tid] = sp;
        }
        __syncthreads();
        const uint32_t w = tid >> 6;
        if (w < kDenseWaves) {
            for (uint32_t i = w; i < kStTiles; i += kDenseWaves) {
                if (L.tcnt[i] != kDenseTile16) continue;         // wave-uniform
                if ((tid & 63) == 0) atomicAdd(&C[kCntDenseTiles], 1u);
                const uint64_t r = dense_tile(L.dw[w], P.wire, P.N, t0 + i, P.spill_w, C, P.s_cap);
                const uint32_t dn = (uint32_t)r, dsp = (uint32_t)(r >> 32);
                if ((tid & 63) == 0) {
                    L.tcnt[i] = (uint16_t)dn;
                    L.tsp[i] = dsp;
                    P.tile_count[t0 + i] = dn;
                    P.tile_spill[t0 + i] = dsp;
                }
            }
        }
        __syncthreads();
        if (tid < kStTiles) {
            c = L.tcnt[tid];
            sp = L.tsp[tid];
        }
        __syncthreads();
    }
    uint32_t n;
    const uint32_t b = block_excl<uint32_t>(c, L.red32, &n);
    if (tid == 0) P.st_n[s] = n;        // (the survivor total: summed by the path resolve, no hot atomic)
    if (tid < kStTiles) {
        L.tcnt[tid] = (uint16_t)c;
        L.tsp[tid] = sp;
        L.tbase[tid] = b;
    }
    if (tid == 0) L.n_tail = 0;
    const bool no_land = C[kCntScanDense] != 0;      // (k_scan's, read here: visible to this launch)
    __syncthreads();
    MP_MARK(0);
    MP_VAL(22, n);
#ifdef FWS_SCAN_PROF
    { const int nsp = __syncthreads_count(tid < P.st_tiles && sp != kNone); MP_VAL(23, (uint64_t)nsp); }
#endif
    if (P.big(n)) {
        if (tid == 0) atomicAdd(&C[kCntBig], 1u);
        if (n <= kMidCap && !P.force_big) merge_mid(P, L, s, n);
        else merge_big(P, L, s, n);
        return;
    }

    // this thread's survivors i = kPer * tid + j: slot ids, then one batch of record loads
    const uint32_t i0 = kPer * tid;
    uint32_t nid[kPer];
    fws_frame_info r[kPer];
    if (i0 < n) {
        uint32_t lo = 0, hi = kStTiles;              // last tile with tbase <= i0
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (L.tbase[mid] <= i0) lo = mid; else hi = mid;
        }
        uint32_t tl = lo;
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) {
            const uint32_t i = i0 + j;
            // (i < n: past the last survivor every later tile has tbase n, and a
            // partial last super tile has up to 255 of them to walk)
            while (i < n && tl + 1 < kStTiles && L.tbase[tl + 1] <= i) ++tl;
            // past n: a slot of this ST's first tile (a global slot 0 for every
            // thread past n of every super tile was one line all of them queued on)
            nid[j] = i < n ? P.sid(t0 + tl, L.tsp[tl], i - L.tbase[tl]) : t0 * kSlots + (j & (kSlots - 1u));
        }
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) r[j] = *P.rec(nid[j]);   // unconditional (a local dummy past n)
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) {
            const uint32_t i = i0 + j;
            if (i < n) {
                L.off[i] = (uint32_t)(r[j].hdr_off - st0);
                L.wt[i] = r[j].hdr_len ? 1 : 0;
            }
        }
    }
    __syncthreads();
    MP_MARK(1);
    // in-ST next: the survivor at the exit offset, searched in the exit's tile only
    // (the 4 searches of a thread interleaved), and the ST's node table for k_emit
    fws_st_node *const tab = P.st_nodes + (uint64_t)s * kStCap;
    uint32_t xr[kPer], sb[kPer], sl[kPer];
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
        const uint64_t x = exit_of(r[j]);
        const bool inside = i0 + j < n && r[j].hdr_len && x < P.N && x < st_end;
        xr[j] = inside ? (uint32_t)(x - st0) : 0u;
        const uint32_t tl = xr[j] / kTile;
        sb[j] = inside ? L.tbase[tl] : 0u;
        sl[j] = inside ? L.tcnt[tl] : 0u;
    }
    for (;;) {
        // the kPer searches' reads of a step issue together (unconditional, in bounds)
        uint32_t ov[kPer];
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) ov[j] = L.off[(sb[j] + (sl[j] >> 1) - (sl[j] > 1 ? 1u : 0u)) & (kStCap - 1u)];
        bool more = false;
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) {
            if (sl[j] > 1) {
                const uint32_t half = sl[j] >> 1;
                if (ov[j] < xr[j]) sb[j] += half;
                sl[j] -= half;
                more |= sl[j] > 1;
            }
        }
        if (!more) break;
    }
    uint16_t vv[kPer];
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
        const uint32_t i = i0 + j;
        vv[j] = kNxDead;
        if (i >= n) continue;
        uint16_t v;
        const uint64_t x = exit_of(r[j]);
        if (!r[j].hdr_len) v = kNxInc;
        else if (x >= P.N) v = kNxEnd;
        else if (x >= st_end) v = kNxExit;
        else v = (sl[j] == 1 && L.off[sb[j]] == xr[j]) ? (uint16_t)sb[j] : kNxDead;
        vv[j] = v;
        L.nx[i] = v;
        const bool tail = v >= kNxInc;
        L.pw[i] = tail ? i : (uint32_t)v | (uint32_t)L.wt[i] << 16;
    }
    __syncthreads();                                 // off[] dead: lref[] reuses it
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j)
        if (i0 + j < n && vv[j] == kNxExit) {
            const uint32_t k = atomicAdd(&L.n_tail, 1u);
            L.lref[i0 + j] = k;
            if (k < kLandCap) L.texit[k] = exit_of(r[j]);
        }
    __syncthreads();
    MP_MARK(2);
    // reserve the ST's run of the tail list (a wave that takes no part in the
    // jumping below, so the atomic's round trip overlaps it)
    if (tid == kMThreads - 64) L.tail_base = reserve_tails(P, s, L.n_tail);
    // the landing survivor of each EXIT tail (k_link's lookup, done here by the
    // waves the jumping below leaves idle, so its two load rounds overlap it):
    // the exit's tile count and its 8 stage slots in one round; a spilled tile
    // is left to k_link (kNone), and so is every tail of a stream with dense
    // tiles (another k_merge workgroup may be rewriting a tile's count and
    // spill offset while this one reads them)
    if (FWS_LAND_WAVE && L.n_tail <= kLandWaveMax) {
        // few tails (every dense-frame super tile): one wavefront per tail, waves
        // 1..7 taking every seventh, so a spilled exit tile (more than 8
        // survivors: frames under ~250 B) is searched too -- its lanes read the
        // spill run's offsets, one ballot -- instead of k_link's binary search
        // over it (a chain of dependent loads). The 200,000 x 64 B stream's
        // super tiles have 16 EXIT tails each (false chains leave with long
        // lengths): k_link's first phase 6.2 -> see DESIGN 4.3.
        const uint32_t wv = tid >> 6, ln = tid & 63u;
        for (uint32_t k = wv - 1u; wv >= 1u && k < L.n_tail; k += (uint32_t)kMWaves - 1u) {
            uint32_t w = kNone;
            if (!no_land) {
                const uint64_t x = L.texit[k];
                const uint32_t t = (uint32_t)(x / kTile);
                const uint32_t tc = P.tile_count[t], tsp = P.tile_spill[t];
                uint64_t o = ln < kSlots ? P.stage_info[t * kSlots + ln].hdr_off : ~0ull;   // with the counts
                uint32_t id = t * kSlots + ln;
                bool ok = true;
                if (tsp != kNone) {                  // wave-uniform
                    ok = tc <= 64u;
                    id = P.spill_base + tsp + ln;
                    o = ok && ln < tc ? P.spill_info[tsp + ln].hdr_off : ~0ull;
                } else if (ln >= tc) {
                    o = ~0ull;
                }
                const uint64_t m = __ballot(o == x);
                if (ok) w = m ? (uint32_t)__builtin_amdgcn_readlane((int)id, (int)__builtin_ctzll(m)) : kTermDead;
            }
            if (ln == 0) L.tland[k] = w;
        }
    } else if (tid >= 64 && tid - 64 < L.n_tail && tid - 64 < kLandCap) {
        const uint32_t k = tid - 64;
        uint32_t w = kNone;                          // every looked-up slot is written (kNone: k_link's)
        if (!no_land) {
            const uint64_t x = L.texit[k];
            const uint32_t t = (uint32_t)(x / kTile);
            uint64_t o[kSlots];
#pragma unroll
            for (uint32_t q = 0; q < kSlots; ++q) o[q] = P.stage_info[t * kSlots + q].hdr_off;
            const uint32_t tc = P.tile_count[t], tsp = P.tile_spill[t];
            uint32_t hit = kTermDead;
#pragma unroll
            for (uint32_t q = 0; q < kSlots; ++q) hit = (q < tc && o[q] == x) ? t * kSlots + q : hit;
            if (tsp == kNone && tc <= kSlots) w = hit;
        }
        L.tland[k] = w;
    }
    // pointer jumping in place: every survivor -> its chain's tail, with frame
    // counts (pointer and count move together in one word, so a read of a word
    // another lane is rewriting sees either pair, both consistent). Up to
    // kWaveJump survivors (every C2 / C3 super tile) one wavefront does it with
    // no workgroup barrier per round (a wave's LDS operations are ordered);
    // more take the whole workgroup.
    if (n <= kWaveJump) {
        if (tid < 64) {
            if (n <= kWaveJump / 2) wave_jump<kWaveJump / 128>(L.pw, n);
            else wave_jump<kWaveJump / 64>(L.pw, n);
        }
        __syncthreads();
    } else {
        for (;;) {
            int changed = 0;
            for (uint32_t i = tid; i < n; i += kMThreads) {
                const uint32_t w = L.pw[i];
                const uint32_t p = w & 0xFFFFu;
                const uint32_t wp = L.pw[p];
                if ((wp & 0xFFFFu) != p) {
                    L.pw[i] = (wp & 0xFFFFu) | (((w >> 16) + (wp >> 16)) << 16);
                    changed = 1;
                }
            }
            if (!__syncthreads_or(changed)) break;
        }
    }
    MP_MARK(3);
    const uint32_t tb = L.tail_base;
    if (tb == kNone) return;
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
        const uint32_t i = i0 + j;
        if (i >= n) continue;
        const uint32_t t = L.pw[i] & 0xFFFFu;
        const uint32_t kind = kind_of(L.nx[t]);
        const uint32_t cnt = (L.pw[i] >> 16) + L.wt[t];
        const uint32_t ref = kind == kKindExit ? tb + L.lref[t] : t;
        P.nres[nid[j]] = fws_node_res{ref, cnt, i, kind};
        fws_st_node nd;
        nd.sid = nid[j];
        nd.nx = vv[j];
        nd.tail = (uint16_t)t;
        nd.cnt = (uint16_t)cnt;
        nd.wt = L.wt[i];
        nd.pad0 = 0;
        nd.pad1 = 0;
        tab[i] = nd;
        if (vv[j] == kNxExit) {
            const uint64_t x = exit_of(r[j]);
            const uint32_t k = L.lref[i];
            P.tails[tb + k] = fws_tail_rec{x, nid[j], k < kLandCap ? L.tland[k] : kNone, (uint32_t)(x >> P.st_shift), 0u};
        }
        if (s == 0 && i == 0 && r[j].hdr_off == 0) {  // the root's chain, for resolve_path
            C[kCntRootSid] = nid[j];
            C[kCntRootTail] = ref;
            C[kCntRootCnt] = cnt;
            C[kCntRoot] = 2u + kind;
        }
    }
    if (s == 0 && tid == 0 && (n == 0 || r[0].hdr_off != 0)) C[kCntRoot] = 1u;
    __syncthreads();
    MP_MARK(4);
    MP_ADD(5, 1);
    MP_SPAN(6, 7);
}

// ------------------------------------------------------------- k_link + path
constexpr uint32_t kStLds = 2048;                   // ST entries / bases in LDS up to this many STs (1 GiB)
constexpr uint32_t kRegComp = 4u * kMThreads;       // marked tails whose tail_pack stays in registers

// tail_pack of EXIT tail x (k_link's thread for x -> the last workgroup, sc1):
// tpk[2x] = landing survivor as its ST's entry | frames of its chain in that ST << 32,
// tpk[2x+1] = record of the path's last header if next(x) ends the path | (ST |
// end kind << 30) << 32. A tail whose exit is no survivor: entry kNone, kind DEAD,
// the last header is the tail's own record.
struct PathLds {
    uint32_t words[kTailCapMax / 32];                // tail-target bitmap (+ the root's tail)
    uint16_t wpre[kTailCapMax / 32];                 // marked tails before each word (<= kCompCap)
    uint16_t cnx[kCompCap];                          // compact next, or kCTerm
    uint32_t kb[2][kCompCap / 32];                   // kept bitmaps (first: the compact list, mc <= kRegComp)
    uint32_t sent[kStLds];                           // per ST: entry, frame count -> base (n_st <= kStLds)
    uint32_t sfb[kStLds];
    uint32_t red32[kMWaves];
    uint32_t root, rt, crt, root_ent, root_cnt, end_kind, end_set, end_sid;
};
static_assert(sizeof(PathLds) <= 160u * 1024u, "k_link LDS");

// Batched loop over c = tid + k * kMThreads < n: the loads of up to 4
// iterations are issued before any of their uses.
template <typename Load, typename Use>
__device__ __forceinline__ void batched4(uint32_t n, Load load, Use use) {
    for (uint32_t base = threadIdx.x; base < n; base += 4u * kMThreads) {
        decltype(load(0u)) v[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {             // unconditional (index 0 past n: n > 0 here), so
            const uint32_t c = base + j * kMThreads;   // no load waits for its data before the next issues
            v[j] = load(c < n ? c : 0u);
        }
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t c = base + j * kMThreads;
            if (c < n) use(c, v[j]);
        }
    }
}

// A workspace limit was hit (k_scan's survivor spill, the tail list, the
// compacted tails): the decode ends with FWS_ERR_CAPACITY, nothing listed or
// unmasked (k_emit and the unmask see kCntFallback / zero frames).
__device__ __forceinline__ void fail_capacity(const MergeParams &P) {
    uint32_t *const C = P.counters;
    if (threadIdx.x != 0) return;
    atomicOr(&C[kCntFallback], 1u);
    C[kCntFrames] = 0;
    fws_decode_result *const r = P.res;              // field by field: no stack copy
    r->status = FWS_ERR_CAPACITY;
    r->n_frames = 0;
    r->consumed = 0;
    r->err_off = 0;
    r->carry_unread = 0;
    r->carry_hdr_len = 0;
    r->n_survivors = ld_acq(&C[kCntSurv]);
}

// The path from offset 0 over the target tails: ST entries and frame bases,
// terminal, result. Runs in the last k_link workgroup. Latency-bound: every
// global load of a phase is issued before its first use, the per-tail data
// arrives packed (tail_pack, one round of loads), and up to kStLds super tiles
// keep their entries and bases in LDS until the final stores.
__device__ void resolve_path(const MergeParams &P, PathLds &G) {
    uint32_t *const C = P.counters;
    const uint32_t tid = threadIdx.x;
    MP_INIT();
    const uint32_t n_st = P.n_st;
    const uint64_t N = P.N;
    const bool lds_st = n_st <= kStLds && !P.force_big;
    // the phase's loads, all issued up front: the flags and counts this launch
    // handed off (sc1), k_merge's record of the root, the survivors per ST
    const uint32_t fbk = ld_acq(&C[kCntFallback]), ovf = ld_acq(&C[kCntOverflow]);
    const uint32_t M = n_st * kTailRun + ld_acq(&C[kCntTails]);   // tail index space: the runs + overflow
    const uint32_t root_state = tid == 0 ? C[kCntRoot] : 0u;
    const uint32_t root_sid = tid == 0 ? C[kCntRootSid] : 0u;
    const uint32_t root_tail = tid == 0 ? C[kCntRootTail] : 0u;
    const uint32_t root_cnt = tid == 0 ? C[kCntRootCnt] : 0u;
    constexpr uint32_t kSper = 8;                    // STs per thread in a prefix pass
    uint32_t sn0[kSper];
#pragma unroll
    for (uint32_t j = 0; j < kSper; ++j) sn0[j] = tid * kSper + j < n_st ? P.st_n[tid * kSper + j] : 0u;
    if (fbk || (ovf & 1u)) {
        fail_capacity(P);                            // k_scan's spill or the tail list overflowed
        return;
    }
    if (tid == 0) {
        uint32_t root = kNone, rt = kNone;
        fws_node_res rr{0, 0, 0, 0};
        if (root_state >= 2u) {
            root = root_sid;
            rr = fws_node_res{root_tail, root_cnt, 0u, root_state - 2u};
        } else if (root_state == 0u && P.n_tiles && P.tile_count[0]) {
            const uint32_t id0 = P.sid(0, P.tile_spill[0], 0);
            if (P.rec(id0)->hdr_off == 0) root = id0;
        }
        G.end_set = 0;
        if (root != kNone) {
            if (root_state == 0u) rr = P.nres[root];
            if (res_kind(rr) == kKindExit) rt = rr.tail;
            else {                                   // the root's chain ends in ST 0
                G.end_sid = P.tail_sid(0, rr);
                G.end_kind = res_kind(rr);
                G.end_set = 1;
            }
        }
        G.root = root;
        G.rt = rt;
        G.root_ent = rr.ent;
        G.root_cnt = rr.cnt;
    }
    // ST entries and frame counts start empty
    if (lds_st) {
        for (uint32_t s = tid; s < n_st; s += kMThreads) {
            G.sent[s] = kNone;
            G.sfb[s] = 0;
        }
    } else {
        for (uint32_t s = tid; s < n_st; s += kMThreads) {
            P.st_entry[s] = kNone;
            P.st_fbase[s] = 0;
        }
    }
    __syncthreads();
    MP_MARK(10);
    const uint32_t root = G.root, rt = G.rt;
    auto set_entry = [&](uint32_t s, uint32_t ent, uint32_t cnt) {
        if (lds_st) { G.sent[s] = ent; G.sfb[s] = cnt; }
        else { P.st_entry[s] = ent; P.st_fbase[s] = cnt; }
    };

    // compact the marked tails (every next() target, plus the root's tail), in tail order
    const uint32_t words = (M + 31u) / 32u;
    const uint32_t per = (words + kMThreads - 1) / kMThreads;
    const uint32_t w0 = tid * per < words ? tid * per : words;
    const uint32_t w1 = w0 + per < words ? w0 + per : words;
    uint32_t cnt = 0;
    for (uint32_t w = w0; w < w1; ++w) {
        uint32_t v = ld_acq(&P.tmark[w]);
        if (rt != kNone && (rt >> 5) == w) v |= 1u << (rt & 31u);
        if (w == words - 1 && (M & 31u)) v &= (1u << (M & 31u)) - 1u;
        G.words[w] = v;
        cnt += (uint32_t)__popc(v);
    }
    uint32_t mc;
    uint32_t pre = block_excl<uint32_t>(cnt, G.red32, &mc);
    if (mc > kCompCap) {                             // > 32 768 STs on the path (8 GiB streams)
        fail_capacity(P);
        return;
    }
    // mc <= kRegComp: the compact list in LDS (kb, unused until the fixpoint) and
    // each thread's tail_packs in registers from here to the entries
    const bool reg = mc <= kRegComp && !P.force_big;
    uint32_t *const comp = reg ? &G.kb[0][0] : P.comp;
    for (uint32_t w = w0; w < w1; ++w) {
        G.wpre[w] = (uint16_t)pre;
        uint32_t v = G.words[w];
        while (v) {
            const uint32_t b = (uint32_t)__ffs(v) - 1u;
            v &= v - 1u;
            comp[pre++] = w * 32u + b;
        }
    }
    __syncthreads();
    MP_MARK(11);
    auto rank = [&](uint32_t x) -> uint32_t {
        return G.wpre[x >> 5] + (uint32_t)__popc(G.words[x >> 5] & ((1u << (x & 31u)) - 1u));
    };
    uint64_t pa[4] = {0, 0, 0, 0}, pb[4] = {0, 0, 0, 0};
    if (reg) {
        uint32_t g[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t c = tid + j * kMThreads;
            const uint32_t x = c < mc ? comp[c] : 0u;  // x = 0 past mc: unused loads of tail 0
            g[j] = ld_acq(&P.gnx[x]);
            pa[j] = ld_acq64(&P.tpk[2u * x]);
            pb[j] = ld_acq64(&P.tpk[2u * x + 1u]);
        }
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t c = tid + j * kMThreads;
            if (c < mc) G.cnx[c] = g[j] >= kGTerm ? kCTerm : (uint16_t)rank(g[j]);
        }
    } else {
        batched4(mc, [&](uint32_t c) { return ld_acq(&P.gnx[P.comp[c]]); },
                 [&](uint32_t c, uint32_t g) { G.cnx[c] = g >= kGTerm ? kCTerm : (uint16_t)rank(g); });
    }
    if (tid == 0) G.crt = rt == kNone ? kNone : rank(rt);
    __syncthreads();
    MP_MARK(12);
    const uint32_t crt = G.crt;

    // greatest fixpoint of K = {crt} U next(K), from K = all marked tails
    const uint32_t cw = (mc + 31u) / 32u;
    uint32_t *ka = G.kb[0], *kb = G.kb[1];
    for (uint32_t w = tid; w < cw; w += kMThreads) ka[w] = ~0u;
    __syncthreads();
    bool settled = mc == 0;
    for (uint32_t round = 0; round < kMaxPruneRounds && !settled; ++round) {
        for (uint32_t w = tid; w < cw; w += kMThreads) kb[w] = 0u;
        __syncthreads();
        if (tid == 0 && crt != kNone) atomicOr(&kb[crt >> 5], 1u << (crt & 31u));
        for (uint32_t c = tid; c < mc; c += kMThreads) {
            const uint16_t g = G.cnx[c];
            if (((ka[c >> 5] >> (c & 31u)) & 1u) && g != kCTerm) atomicOr(&kb[g >> 5], 1u << (g & 31u));
        }
        __syncthreads();
        int diff = 0;
        for (uint32_t w = tid; w < cw; w += kMThreads) {
            const uint32_t m = (w == cw - 1 && (mc & 31u)) ? (1u << (mc & 31u)) - 1u : ~0u;
            diff |= ((ka[w] ^ kb[w]) & m) != 0;
        }
        uint32_t *t = ka; ka = kb; kb = t;
        settled = !__syncthreads_or(diff);
    }
    MP_MARK(13);
    if (!settled) {
        // an input that keeps false tails alive for kMaxPruneRounds: the path
        // itself, walked from the root's tail (offsets increase along next, so
        // at most mc steps)
        for (uint32_t w = tid; w < cw; w += kMThreads) ka[w] = 0u;
        __syncthreads();
        if (tid == 0) {
            for (uint32_t c = crt; c != kNone && c < mc;) {
                ka[c >> 5] |= 1u << (c & 31u);
                const uint16_t g = G.cnx[c];
                c = g == kCTerm ? kNone : (uint32_t)g;
            }
        }
        __syncthreads();
    }

    // entries: the root, and every kept tail's landing survivor, with their chain counts
    if (tid == 0 && root != kNone) set_entry(0, G.root_ent, G.root_cnt);
    auto entry = [&](uint32_t c, uint64_t a, uint64_t b) {
        if (!((ka[c >> 5] >> (c & 31u)) & 1u)) return;
        const uint32_t ent = (uint32_t)a, hi = (uint32_t)(b >> 32);
        if (ent != kNone) set_entry(hi & 0x3FFFFFFFu, ent, (uint32_t)(a >> 32));
        if (G.cnx[c] == kCTerm) {                    // exactly one kept tail ends the path
            G.end_sid = (uint32_t)b;
            G.end_kind = hi >> 30;
            G.end_set = 1;
        }
    };
    if (reg) {
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t c = tid + j * kMThreads;
            if (c < mc) entry(c, pa[j], pb[j]);
        }
    } else {
        batched4(mc, [&](uint32_t c) {
                     const uint32_t x = P.comp[c];
                     return ulonglong2{ld_acq64(&P.tpk[2u * x]), ld_acq64(&P.tpk[2u * x + 1u])};
                 },
                 [&](uint32_t c, ulonglong2 v) { entry(c, v.x, v.y); });
    }
    __syncthreads();
    MP_MARK(14);

    // exclusive prefix of the per-ST frame counts, in ST order; every ST's entry
    // and base stored for k_emit
    uint32_t nf_path = 0, nsurv = 0;
    for (uint32_t s0 = 0; s0 < n_st; s0 += kSper * kMThreads) {
        const uint32_t lo = s0 + tid * kSper;
        uint32_t fc[kSper], sn[kSper], en[kSper];
        uint32_t fs = 0, ss = 0;
#pragma unroll
        for (uint32_t j = 0; j < kSper; ++j) {
            const bool in = lo + j < n_st;
            fc[j] = !in ? 0u : lds_st ? G.sfb[lo + j] : P.st_fbase[lo + j];
            en[j] = !in ? kNone : lds_st ? G.sent[lo + j] : 0u;
            sn[j] = s0 == 0 ? sn0[j] : in ? P.st_n[lo + j] : 0u;
        }
#pragma unroll
        for (uint32_t j = 0; j < kSper; ++j) {
            fs += fc[j];
            ss += sn[j];
        }
        uint32_t ft, st;
        (void)block_excl<uint32_t>(ss, G.red32, &st);
        nsurv += st;
        uint32_t fpre = nf_path + block_excl<uint32_t>(fs, G.red32, &ft);
#pragma unroll
        for (uint32_t j = 0; j < kSper; ++j) {
            if (lo + j < n_st) {
                P.st_fbase[lo + j] = fpre;
                if (lds_st) P.st_entry[lo + j] = en[j];
            }
            fpre += fc[j];
        }
        nf_path += ft;
    }
    MP_MARK(15);
    MP_ADD(16, mc);
    if (tid != 0) return;
    C[kCntSurv] = nsurv;
    if (root != kNone && !G.end_set) {               // no terminal on the path: cannot happen
        atomicOr(&C[kCntFallback], 1u);
        fws_decode_result r{};
        r.status = FWS_ERR_INTERNAL;
        C[kCntFrames] = 0;
        *P.res = r;
        return;
    }
    // terminal: the path's last header, then ParseFrameHdr from its exit on error
    fws_decode_result r{};
    r.status = FWS_OK;
    r.n_survivors = nsurv;
    uint64_t pos = 0;
    bool walk = N > 0 && root == kNone;              // no chain from offset 0 survived
    if (root != kNone) {
        const fws_frame_info fi = *P.rec(G.end_sid);
        pos = G.end_kind == kKindInc ? fi.hdr_off : exit_of(fi);
        walk = G.end_kind == kKindDead;
    }
    uint32_t nf = nf_path;
    const uint32_t cap = P.cap;
    if (walk) {
        for (;;) {
            if (pos >= N) break;
            Hdr h;
            const uint64_t q = pos;
            const int rc = parse_hdr([&](int i) -> uint32_t { return P.wire[q + i]; }, N - q, true, h);
            if (rc < 0) { r.status = rc; r.err_off = q; break; }
            if (rc == 0) break;                      // incomplete trailing header
            const uint64_t po = q + rc;
            if (nf < cap) {
                fws_frame_info fi;
                fi.hdr_off = q; fi.payload_len = h.plen; fi.key = h.key; fi.opcode = (uint8_t)h.opcode;
                fi.fin = (uint8_t)h.fin; fi.hdr_len = (uint8_t)rc;
                fi.flags = (po + h.plen > N) ? (uint8_t)FWS_FRAME_TRUNCATED : (uint8_t)0;
                P.put_frame(nf, fi);
            }
            ++nf;
            pos = po + h.plen;
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
    const uint32_t lim = nf < cap ? nf : cap;
    C[kCntFrames] = lim;
    if (lim > nf_path) {
        // walk frames (within one tile; k_emit spans the path frames): each
        // walk frame's span, the last one's to the end of the stream
        for (uint32_t f = nf_path; f < lim; ++f) {
            const uint64_t h = P.frames[f].hdr_off;
            P.plan_units(f, h, f + 1 < lim ? P.frames[f + 1].hdr_off : 0, f + 1 == lim);
        }
    }
    *P.res = r;
    MP_MARK(17);
}

// One thread per EXIT tail: the survivor its exit lands on, next(tail), the
// tail's tail_pack and the target bitmap. The last workgroup (atomic ticket)
// resolves the path.
// Hand-off inside the launch without release / acquire fences
// (cdna_hip_programming.md Guideline 16, MI355X_MICROARCH.md "Valid forms",
// first row): every handed-off word is stored sc1 (relaxed agent atomic
// store / atomicOr), each storing wave drains vmcnt before the workgroup
// barrier, one lane adds to the ticket, and the last adder reads them only
// with sc1 loads (ld_acq). Everything else it reads was written by earlier
// launches. One k_link workgroup per CU (its LDS).
__global__ __launch_bounds__(kMThreads) void k_link(MergeParams P) {
    __shared__ PathLds G;
    __shared__ uint32_t s_last;
    const uint32_t tid = threadIdx.x;
    uint32_t *const C = P.counters;
    MP_START(29);
    MP_T0();
    MP_INIT();
    // tail index space: the super tiles' runs [0, fixed), then the overflow area
    // (k_merge's reserve_tails); one thread per run slot, a grid-stride loop past it
    const uint32_t fixed = P.n_st * kTailRun, stride = gridDim.x * kMThreads;
    uint32_t x = blockIdx.x * kMThreads + tid;
    // the first tail's loads beside the counters (read past the valid ones: unused)
    fws_tail_rec tr = P.tails[x < P.tail_cap ? x : 0u];
    uint32_t nt = x < fixed ? P.st_nt[x / kTailRun] : 0u;
    const uint32_t total = fixed + C[kCntTails];
    if (!C[kCntFallback]) {
        while (x < total) {
            if (x >= fixed || x % kTailRun < nt) {
                const uint64_t tx = tr.exit;
                const uint32_t w = tr.w != kNone ? tr.w : P.find_node(tx);   // k_merge looked most up
                const uint32_t wst = (uint32_t)(tx >> P.st_shift);
                uint32_t g = kGTerm | kKindDead, ent = kNone, cnt = 0, esid = tr.id;
                if (w != kTermDead) {
                    const fws_node_res r = P.nres[w];
                    g = res_kind(r) == kKindExit ? r.tail : (kGTerm | res_kind(r));
                    ent = r.ent;
                    cnt = r.cnt;
                    if (g >= kGTerm) esid = P.tail_sid(wst, r);   // the path's last header if it ends here
                }
                gst64(&P.tpk[2u * x], (uint64_t)ent | ((uint64_t)cnt << 32));
                gst64(&P.tpk[2u * x + 1u], (uint64_t)esid | ((uint64_t)(wst | ((g >= kGTerm ? g & 3u : 0u) << 30)) << 32));
                gst(&P.gnx[x], g);
                if (g < kGTerm) atomicOr(&P.tmark[g >> 5], 1u << (g & 31u));
            }
            x += stride;
            if (x >= total) break;
            tr = P.tails[x];
            nt = x < fixed ? P.st_nt[x / kTailRun] : 0u;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
    __syncthreads();
    if (tid == 0)
        s_last = __hip_atomic_fetch_add(&C[kCntTicket], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                 gridDim.x - 1u;
    __syncthreads();
    MP_MARK(8);
    MP_ADD(9, 1);
    if (!s_last) return;
    resolve_path(P, G);
    __syncthreads();
    MP_SPAN(20, 21);
}

// ------------------------------------------------------------------ k_emit
struct EmitLds {
    union {
        struct {
            uint16_t ptr[2][kStCap];
            uint8_t mark[kStCap];
            uint16_t hist[kStCap + 2];               // marked survivors per chain depth (frames to the tail)
            uint16_t rs[kStCap + 2];                 // the entry chain's survivor at each depth
        };
        struct {                                     // emit_mid
            uint16_t mptr[kMidCap];
            uint8_t mmark[kMidCap];                  // bit 0: on the entry's chain; bit 1: a frame
        };
    };
    uint32_t mtb[kStTiles], mtsp[kStTiles];          // emit_mid: the ST's tile prefix
    uint32_t red32[kMWaves];
};
constexpr uint16_t kUnres = 0xFFFF;
constexpr uint32_t kDepthRounds = 16;                // then pointer doubling

// The big-ST path of k_emit (k_merge's merge_big): the same marking of the
// entry's chain by pointer doubling, over slot ids in global scratch; the
// frames in offset order are the ST's survivors in tile order.
__device__ void emit_big(const MergeParams &P, uint32_t s, uint32_t n, uint32_t e, uint32_t fbase, uint32_t lim) {
    __shared__ uint32_t s_tb[kStTiles], s_tsp[kStTiles], s_red[kMWaves];
    const uint32_t tid = threadIdx.x, t0 = s * P.st_tiles;
    uint32_t c = 0, sp = kNone;
    if (tid < P.st_tiles && t0 + tid < P.n_tiles) {
        c = P.tile_count[t0 + tid];
        sp = P.tile_spill[t0 + tid];
    }
    uint32_t tot;
    const uint32_t b = block_excl<uint32_t>(c, s_red, &tot);
    if (tid < kStTiles) {
        s_tb[tid] = b;
        s_tsp[tid] = sp;
    }
    __syncthreads();
    auto sid_of = [&](uint32_t i) -> uint32_t {
        uint32_t lo = 0, hi = kStTiles;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_tb[mid] <= i) lo = mid; else hi = mid;
        }
        return P.sid(t0 + lo, s_tsp[lo], i - s_tb[lo]);
    };
    uint32_t *const p0 = P.bg_ptr, *const p1 = P.bg_ptr + P.max_nodes;
    for (uint32_t i = tid; i < n; i += kMThreads) {
        const uint32_t id = sid_of(i);
        const uint32_t v = gld(P.bg_nx + id);
        gst(p0 + id, v >= kBgInc ? id : v);
        gst(P.bg_mark + id, id == e ? 1u : 0u);
    }
    __syncthreads();
    // marks double along the chain: after round k every node within 2^k steps of the entry
    uint32_t *pc = p0, *pn = p1;
    for (;;) {
        int changed = 0;
        for (uint32_t i = tid; i < n; i += kMThreads) {
            const uint32_t id = sid_of(i);
            const uint32_t p = gld(pc + id);
            if (gld(P.bg_mark + id) && !gld(P.bg_mark + p)) {
                gst(P.bg_mark + p, 1u);
                changed = 1;
            }
            gst(pn + id, gld(pc + p));
        }
        uint32_t *t = pc; pc = pn; pn = t;
        if (!__syncthreads_or(changed)) break;
    }
    // the chain's frames in offset order, in rounds of kMThreads survivors
    uint32_t f = fbase;
    for (uint32_t i0 = 0; i0 < n; i0 += kMThreads) {
        const uint32_t i = i0 + tid;
        uint32_t id = 0;
        bool fr = false;
        if (i < n) {
            id = sid_of(i);
            fr = gld(P.bg_mark + id) && gld(P.bg_wt + id);
        }
        uint32_t rt;
        const uint32_t o = f + block_excl<uint32_t>(fr ? 1u : 0u, s_red, &rt);
        if (fr && o < lim) {
            const fws_frame_info fi = *P.rec(id);
            P.put_frame(o, fi);
            P.plan_units(o, fi.hdr_off, exit_of(fi), o == lim - 1);
        }
        f += rt;
    }
}

// k_emit for a super tile merge_mid handled: the entry's chain marked by
// synchronous pointer doubling in LDS (each round reads every pointer and mark
// into registers, then writes), frames in offset order. Thread t owns
// survivors [kMidPer * t, kMidPer * (t + 1)).
constexpr uint32_t kMidPer = kMidCap / kMThreads;
constexpr uint32_t kMidBatch = 4;
static_assert(kMidPer * kMThreads == kMidCap && kMidPer % kMidBatch == 0, "mid survivors per thread");
__device__ void emit_mid(const MergeParams &P, EmitLds &L, uint32_t s, uint32_t n, uint32_t e, uint32_t fbase,
                         uint32_t lim) {
    const uint32_t tid = threadIdx.x, t0 = s * P.st_tiles;
    uint32_t c = 0, sp = kNone;
    if (tid < P.st_tiles && t0 + tid < P.n_tiles) {
        c = P.tile_count[t0 + tid];
        sp = P.tile_spill[t0 + tid];
    }
    uint32_t tot;
    const uint32_t b0 = block_excl<uint32_t>(c, L.red32, &tot);
    if (tid < kStTiles) {
        L.mtb[tid] = b0;
        L.mtsp[tid] = sp;
    }
    __syncthreads();
    const uint32_t i0 = kMidPer * tid;
    uint32_t tl0;
    {
        uint32_t lo = 0, hi = kStTiles;              // tile of survivor i0
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (L.mtb[mid] <= i0) lo = mid; else hi = mid;
        }
        tl0 = lo;
    }
    // slot ids of this thread's survivors kMidBatch at a time, walking the tiles forward
    auto ids = [&](uint32_t j0, uint32_t &tl, uint32_t (&id)[kMidBatch]) {
#pragma unroll
        for (uint32_t j = 0; j < kMidBatch; ++j) {
            const uint32_t i = i0 + j0 + j < n ? i0 + j0 + j : i0;
            while (tl + 1 < kStTiles && L.mtb[tl + 1] <= i) ++tl;
            id[j] = P.sid(t0 + tl, L.mtsp[tl], i - L.mtb[tl]);
        }
    };
    {
        uint32_t tl = tl0;
        for (uint32_t j0 = 0; j0 < kMidPer; j0 += kMidBatch) {
            uint32_t id[kMidBatch], nx[kMidBatch], wt[kMidBatch];
            ids(j0, tl, id);
#pragma unroll
            for (uint32_t j = 0; j < kMidBatch; ++j) {
                nx[j] = P.bg_ptr[id[j]];
                wt[j] = P.bg_wt[id[j]];
            }
#pragma unroll
            for (uint32_t j = 0; j < kMidBatch; ++j) {
                const uint32_t i = i0 + j0 + j;
                if (i < n) {
                    L.mptr[i] = (uint16_t)nx[j];
                    L.mmark[i] = (uint8_t)((id[j] == e ? 1u : 0u) | (wt[j] << 1));
                }
            }
        }
    }
    __syncthreads();
    for (;;) {
        uint32_t pr[kMidPer];                        // next pointer | target << 16
        uint32_t mk = 0;
#pragma unroll
        for (uint32_t j = 0; j < kMidPer; ++j) {
            const uint32_t i = i0 + j;
            pr[j] = 0;
            if (i < n) {
                const uint32_t p = L.mptr[i];
                pr[j] = L.mptr[p] | (p << 16);
                if ((L.mmark[i] & 1u) && !(L.mmark[p] & 1u)) mk |= 1u << j;
            }
        }
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < kMidPer; ++j) {
            if (i0 + j < n) L.mptr[i0 + j] = (uint16_t)pr[j];
            if (mk & (1u << j)) L.mmark[pr[j] >> 16] |= 1u;
        }
        if (!__syncthreads_or(mk != 0)) break;
    }
    // frames in offset order: this thread's run, then one block scan
    uint32_t fl = 0, fm = 0;
#pragma unroll
    for (uint32_t j = 0; j < kMidPer; ++j)
        if (i0 + j < n && L.mmark[i0 + j] == 3u) {
            fm |= 1u << j;
            ++fl;
        }
    uint32_t ft;
    uint32_t f = fbase + block_excl<uint32_t>(fl, L.red32, &ft);
    uint32_t tl = tl0;
    for (uint32_t j0 = 0; j0 < kMidPer; j0 += kMidBatch) {
        uint32_t id[kMidBatch];
        ids(j0, tl, id);
        fws_frame_info rc[kMidBatch];
#pragma unroll
        for (uint32_t j = 0; j < kMidBatch; ++j) rc[j] = *P.rec(id[j]);
#pragma unroll
        for (uint32_t j = 0; j < kMidBatch; ++j) {
            if (!((fm >> (j0 + j)) & 1u)) continue;
            if (f < lim) {
                P.put_frame(f, rc[j]);
                P.plan_units(f, rc[j].hdr_off, exit_of(rc[j]), f == lim - 1);
            }
            ++f;
        }
    }
}

// 6 waves per SIMD (80 VGPRs, no spill; the compiler's own choice, 91, held two
// workgroups per CU: C2 / C3's 513 super tiles then need a second round of one)
__global__ __launch_bounds__(kMThreads) __attribute__((amdgpu_waves_per_eu(6))) void k_emit(MergeParams P) {
    __shared__ EmitLds L;
    const uint32_t s = blockIdx.x, tid = threadIdx.x;
    uint32_t *const C = P.counters;
    MP_START(28);
    MP_T0();
    MP_INIT();
    if (s == 0)                                      // the next call's counter set
        for (uint32_t w = tid; w < kCntStride; w += kMThreads) P.zero_next[w] = 0u;
    if (s >= P.n_st) return;
    const uint32_t fb = C[kCntFallback], e = P.st_entry[s], fbase = P.st_fbase[s], n = P.st_n[s];
    const uint32_t lim = C[kCntFrames];
    if (fb || e == kNone || fbase >= lim) return;
    if (P.big(n)) {
        if (n <= kMidCap && !P.force_big) emit_mid(P, L, s, n, e, fbase, lim);
        else emit_big(P, s, n, e, fbase, lim);
        return;
    }
    // (loading all kStCap rows with the words above, before n is known, measured
    // 9.4 -> 13.6 us on C3: 16 MB of rows instead of ~1 MB; the first 512 rows
    // that way, with the entry's row from its thread through LDS, 9.1 -> ~15 us)
    const fws_st_node *const tab = P.st_nodes + (uint64_t)s * kStCap;
    const uint32_t i0 = kPer * tid;
    fws_st_node nd[kPer];
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) nd[j] = tab[i0 + j < n ? i0 + j : e];   // one batch, the entry's row too
    const fws_st_node ne = tab[e];
    // the entry's chain = the survivors at or after it with its tail, when their
    // frame count is the entry's: any other survivor joining the chain (a false
    // chain merging into it) makes the count larger, and the marks double along
    // the next pointers instead (exact either way)
    bool fr[kPer];
    uint32_t fl = 0;
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
        const uint32_t i = i0 + j;
        fr[j] = i < n && i >= e && nd[j].tail == ne.tail && nd[j].wt;
        fl += fr[j];
    }
    uint32_t ftot;
    uint32_t fpre = block_excl<uint32_t>(fl, L.red32, &ftot);
    MP_MARK(24);
    if (ftot != ne.cnt) {
        // other survivors joined the chain (false chains merging into it: common,
        // a few per super tile): exactly one survivor per depth is on the entry's
        // chain -- the only one at its depth, or next() of the one a depth above
        const uint32_t D = ne.cnt;                   // the entry's depth (frames to the tail)
        for (uint32_t c = tid; c <= D; c += kMThreads) {
            L.hist[c] = 0;
            L.rs[c] = kUnres;
        }
        __syncthreads();
        bool mk[kPer];
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) {
            const uint32_t i = i0 + j;
            mk[j] = i < n && i >= e && nd[j].tail == ne.tail && nd[j].cnt <= D;
            if (i < n) L.ptr[0][i] = nd[j].nx;
            if (mk[j]) {
                atomicAdd(reinterpret_cast<uint32_t *>(&L.hist[nd[j].cnt & ~1u]), 1u << (16u * (nd[j].cnt & 1u)));
                L.rs[nd[j].cnt] = (uint16_t)i;
            }
        }
        __syncthreads();
        for (uint32_t c = tid; c <= D; c += kMThreads)
            if (L.hist[c] != 1) L.rs[c] = c == D ? (uint16_t)e : kUnres;
        __syncthreads();
        bool open = true;
        for (uint32_t round = 0; round < kDepthRounds && open; ++round) {
            int pend = 0;
            for (uint32_t c = tid; c < D; c += kMThreads) {
                if (L.rs[c] != kUnres) continue;
                const uint16_t up = L.rs[c + 1];
                if (up != kUnres) L.rs[c] = L.ptr[0][up];
                else pend = 1;
            }
            open = __syncthreads_or(pend);
        }
        if (open) {
            if (tid == 0) atomicAdd(&C[kCntEmitDoubling], 1u);
#pragma unroll
            for (uint32_t j = 0; j < kPer; ++j) {
                const uint32_t i = i0 + j;
                if (i < n) {
                    const uint16_t v = nd[j].nx;
                    L.ptr[0][i] = v >= kNxInc ? (uint16_t)i : v;
                    L.mark[i] = i == e;
                }
            }
            __syncthreads();
            // marks double along the chain: after round k every node within 2^k steps of the entry
            int cur = 0;
            for (;;) {
                int changed = 0;
                for (uint32_t i = tid; i < n; i += kMThreads) {
                    const uint16_t p = L.ptr[cur][i];
                    if (L.mark[i] && !L.mark[p]) {
                        L.mark[p] = 1;
                        changed = 1;
                    }
                    L.ptr[cur ^ 1][i] = L.ptr[cur][p];
                }
                cur ^= 1;
                if (!__syncthreads_or(changed)) break;
            }
        }
        fl = 0;
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) {
            const uint32_t i = i0 + j;
            fr[j] = nd[j].wt && (open ? (i < n && L.mark[i]) : (mk[j] && L.rs[nd[j].cnt] == i));
            fl += fr[j];
        }
        fpre = block_excl<uint32_t>(fl, L.red32, &ftot);
    }
    MP_MARK(25);
    // the chain's frames in offset order (records loaded in one batch), and
    // their stream-space plan units
    fws_frame_info rc[kPer];                         // unconditional (slot 0 for the unused ones):
#pragma unroll                                        // conditional loads each waited for their data
    for (uint32_t j = 0; j < kPer; ++j) rc[j] = *P.rec(fr[j] ? nd[j].sid : s * P.st_tiles * kSlots + j);
    uint32_t f = fbase + fpre;
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
        if (!fr[j]) continue;
        if (f < lim) {
            P.put_frame(f, rc[j]);
            P.plan_units(f, rc[j].hdr_off, exit_of(rc[j]), f == lim - 1);
        }
        ++f;
    }
    __syncthreads();
    MP_MARK(26);
    MP_ADD(27, 1);
    MP_SPAN(28, 29);
}

}  // namespace fwsk

#ifdef FWS_SCAN_PROF
extern "C" int fws_internal_merge_trace(unsigned long long *out) {
    return fws_hip_status(hipMemcpyFromSymbol(out, HIP_SYMBOL(fwsk::g_merge_trace),
                                              sizeof(unsigned long long) * fwsk::kTraceWg * 32));
}
extern "C" int fws_internal_merge_prof(unsigned long long *out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(fwsk::g_merge_prof), sizeof(unsigned long long) * 32);
    if (e == hipSuccess && reset) {
        unsigned long long z[32] = {};
        z[6] = z[20] = z[28] = ~0ull;                // span minima
        e = hipMemcpyToSymbol(HIP_SYMBOL(fwsk::g_merge_prof), z, sizeof(z));
    }
    return fws_hip_status(e);
}
#endif

// ------------------------------------------------------------------ host side
using namespace fwsk;

// super tiles of kStTiles tiles, halved while that gives fewer than kStTarget
// (a short stream's resolve then spreads over more CUs), down to kStTilesMin
static uint64_t g_st_target = kStTarget;   // test hook: 1 = the largest super tiles on any stream
extern "C" __attribute__((visibility("default"))) int fws_internal_set_st_target(int t) {
    const int old = (int)g_st_target;
    g_st_target = t > 0 && (uint64_t)t <= kStTarget ? (uint64_t)t : kStTarget;   // fewer super tiles only:
    return old;                                                                    // the workspaces stay in bounds
}
static uint32_t st_tiles_for(uint64_t n_tiles) {
    uint32_t t = kStTiles;
    while (t > kStTilesMin && n_tiles < (uint64_t)t * g_st_target) t >>= 1;
    return t;
}
uint64_t fws_merge_super_tiles(uint64_t n_tiles) {
    const uint32_t t = st_tiles_for(n_tiles);
    return (n_tiles + t - 1) / t;
}
// a bound on fws_merge_super_tiles(n) for every n <= n_tiles (the count is not
// monotonic in n where the super tile halves): at most 2 kStTarget below
// kStTiles-sized super tiles, and never more than tiles / kStTilesMin
uint64_t fws_merge_super_tiles_cap(uint64_t n_tiles) {
    const uint64_t a = (n_tiles + kStTiles - 1) / kStTiles, lo = 2 * kStTarget;
    const uint64_t b = (n_tiles + kStTilesMin - 1) / kStTilesMin;
    const uint64_t c = a > lo ? a : lo;
    return c < b ? c : b;
}
uint64_t fws_merge_st_nodes(uint64_t n_tiles) { return fws_merge_super_tiles_cap(n_tiles) * kStCap; }

uint32_t fws_merge_comp_cap() { return kCompCap; }

uint32_t fws_merge_tail_cap(uint64_t n_tiles) {
    uint64_t c = fws_merge_super_tiles_cap(n_tiles) * 64u + 4096u;
    return (uint32_t)(c < kTailCapMax ? c : kTailCapMax);
}

int fws_launch_merge(fws_gpu_ctx *ctx, const uint8_t *wire, uint64_t N, uint32_t n_tiles, fws_frame_info *frames,
                     uint32_t cap, fws_decode_result *res, uint8_t *utf8_ok, bool force_big, uint32_t *zero_next,
                     hipStream_t s) {
    fws_decode_ws &d = ctx->dec;
    MergeParams P;
    P.wire = wire;
    P.N = N;
    P.n_tiles = n_tiles;
    P.st_tiles = st_tiles_for(n_tiles);
    P.st_shift = (uint32_t)__builtin_ctz(P.st_tiles) + (uint32_t)__builtin_ctz(kTile);
    P.n_st = (uint32_t)fws_merge_super_tiles(n_tiles);
    if (P.n_st > d.max_st) return FWS_ERR_INTERNAL;   // fws_decode_ensure sized the tables
    if ((uint64_t)P.n_st * kTailRun > d.tail_cap) return FWS_ERR_CAPACITY;   // > 8 GiB streams
    P.stage_info = d.stage_info;
    P.spill_info = d.spill_info;
    P.spill_w = d.spill_info;
    P.s_cap = (uint32_t)d.max_surv;
    P.tile_count = d.tile_count;
    P.tile_spill = d.tile_spill;
    P.spill_base = n_tiles * kSlots;
    P.tail_cap = d.tail_cap;
    P.counters = d.counters;
    P.nres = d.nres;
    P.tails = d.tails;
    P.gnx = d.gnx;
    P.tpk = d.tpk;
    P.tmark = d.tmark;
    P.comp = d.comp;
    P.st_nodes = d.st_nodes;
    P.st_n = d.st_n;
    P.st_nt = d.st_nt;
    P.st_entry = d.st_entry;
    P.st_fbase = d.st_fbase;
    P.frames = frames;
    P.cap = cap;
    P.res = res;
    P.utf8_ok = utf8_ok;
    P.unit_first = ctx->plan.unit_first;
    const uint64_t units = (N + kUnit - 1) / kUnit;
    P.n_units = units < ctx->plan.unit_cap ? units : ctx->plan.unit_cap;
    P.force_big = force_big ? 1u : 0u;
    P.zero_next = zero_next;
    P.bg_nx = d.bg_nx;
    P.bg_wt = d.bg_wt;
    P.bg_lref = d.bg_lref;
    P.bg_ptr = d.bg_ptr;
    P.bg_sc = d.bg_sc;
    P.bg_mark = d.bg_mark;
    P.max_nodes = d.max_nodes;
    const dim3 grid(P.n_st ? P.n_st : 1u), blk(kMThreads);
    hipLaunchKernelGGL(k_merge, grid, blk, 0, s, P);
    const uint32_t fixed = P.n_st * kTailRun;         // k_link: one thread per run slot (+ a loop past them)
    hipLaunchKernelGGL(k_link, dim3(fixed ? (fixed + kMThreads - 1) / kMThreads : 1u), blk, 0, s, P);
    hipLaunchKernelGGL(k_emit, grid, blk, 0, s, P);
    return fws_hip_status(hipGetLastError());
}
