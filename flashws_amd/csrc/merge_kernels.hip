// merge_kernels.hip -- second half of fws_gpu_decode_stream on the common
// path: from k_scan's per-tile survivors to the frame list, the payload
// descriptors and the unmask plan in two launches, with no grid barrier.
//
// OnRecvData's frame loop (net/w_socket.h:543-769) is a chain: the next
// header starts at this header's exit (hdr_off + hdr_len + payload_len,
// w_socket.h:750-764). k_scan (decode_kernels.hip) left, per 2 KiB tile, the
// offsets whose header chain reaches the tile end ("survivors"): every true
// header plus a few random offsets.
//
//  k_merge  one workgroup per super tile (ST = 128 tiles = 256 KiB). Loads
//           the ST's survivors into LDS in offset order, links each to the
//           survivor at its exit inside the ST (binary search), and pointer-
//           jumps (Wyllie) so every survivor knows the tail of its chain in
//           the ST, the frames and unmask chunks up to that tail, and how the
//           chain leaves the ST: EXIT (into a later ST), END (at or past the
//           stream end), DEAD (the exit is not a header: a protocol error or a
//           false chain) or INC (an incomplete header at the stream end).
//           EXIT tails go to a global list.
//  k_link   one thread per EXIT tail: the survivor its exit lands on (binary
//           search in that tile's survivors) and next(tail) = the tail of
//           that survivor's chain; marks every next() target in a bitmap.
//  last WG  the k_link workgroup that finishes last (atomic ticket) resolves
//           the path from the header at offset 0 over the marked tails
//           (compacted into LDS). The path's tails are the greatest fixpoint
//           of K = {root's tail} U next(K): offsets strictly increase along
//           next, so a false tail has a finite chain of predecessors and
//           drops out after a few rounds.
//           Each landing survivor on the path is its ST's entry; a scan over
//           the STs gives every ST's frame and chunk base. The terminal is
//           finished with ParseFrameHdr's rules (w_socket.h:435-524): the
//           error walk, carry-out and the fws_decode_result.
//  k_emit   one workgroup per ST with an entry: marks the entry's chain by
//           pointer doubling and writes fws_frame_info, fws_frame_desc and
//           the unmask plan (cbase, unit_first) in stream order.
//
// A super tile with more than kStCap survivors (dense small frames), a full
// tail list, a survivor overflow in k_scan or a pruning that does not settle
// sets kCntFallback: k_emit then returns at once and the cooperative k_resolve
// (resolve_kernels.hip) does the whole job.
#include "decode_common.h"

namespace fwsk {

constexpr uint32_t kStTiles = 128;                  // tiles per super tile
constexpr uint64_t kStBytes = uint64_t(kStTiles) * kTile;
constexpr uint32_t kStCap = 2048;                   // survivors of one ST in LDS
constexpr int kMThreads = 512;
constexpr int kMWaves = kMThreads / 64;
constexpr uint32_t kTailCapMax = 1u << 18;          // LDS bitmaps of the path pruning
constexpr uint32_t kMaxPruneRounds = 64;

// in-ST next of a survivor: an LDS index, or how the chain leaves the ST
constexpr uint16_t kNxInc = 0xFFFC, kNxDead = 0xFFFD, kNxEnd = 0xFFFE, kNxExit = 0xFFFF;
constexpr uint32_t kKindExit = 0, kKindEnd = 1, kKindDead = 2, kKindInc = 3;
constexpr uint32_t kGTerm = 0xFFFFFFF0u;            // next(tail) >= kGTerm: the path ends (kGTerm | kind)
constexpr uint32_t kCntMask = (1u << 30) - 1u;

__device__ __forceinline__ uint32_t kind_of(uint16_t code) {
    return code == kNxExit ? kKindExit : code == kNxEnd ? kKindEnd : code == kNxDead ? kKindDead : kKindInc;
}

struct MergeParams {
    const uint8_t *wire;
    uint64_t N;
    uint32_t n_tiles;
    uint32_t n_st;
    const fws_frame_info *stage_info;
    const fws_frame_info *spill_info;
    const uint32_t *tile_count;
    const uint32_t *tile_spill;
    uint32_t spill_base;                             // n_tiles * kSlots: first slot id of the spill area
    uint32_t tail_cap;
    uint32_t *counters;
    fws_node_res *nres;
    fws_tail_rec *tails;
    uint32_t *gnx;
    uint32_t *tmark;                                 // tail-target bitmap (tail_cap / 32 + 1 words)
    uint32_t *st_entry;
    uint32_t *st_fbase;
    uint64_t *st_cbase;
    fws_frame_info *frames;
    uint32_t cap;
    fws_frame_desc *descs;
    fws_decode_result *res;
    uint64_t *cbase;                                 // unmask plan (fws_plan_ws)
    uint32_t *unit_first;
    uint64_t *plan_total;
    uint64_t unit_cap;

    // slot id of survivor r of tile t (stage slots, or the tile's spill run)
    __device__ __forceinline__ uint32_t sid(uint32_t t, uint32_t sp, uint32_t r) const {
        return sp == kNone ? t * kSlots + r : spill_base + sp + r;
    }
    __device__ __forceinline__ fws_frame_info info(uint32_t id) const {
        return id < spill_base ? stage_info[id] : spill_info[id - spill_base];
    }
    // slot id of the survivor at offset x (x < N), or kTermDead
    __device__ uint32_t find_node(uint64_t x) const {
        const uint32_t t = (uint32_t)(x / kTile);
        const uint32_t n = tile_count[t], sp = tile_spill[t];
        uint32_t lo = 0, hi = n;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (info(sid(t, sp, mid)).hdr_off < x) lo = mid + 1; else hi = mid;
        }
        return (lo < n && info(sid(t, sp, lo)).hdr_off == x) ? sid(t, sp, lo) : kTermDead;
    }
    __device__ __forceinline__ uint64_t node_chunks(const fws_frame_info &fi) const {
        if (fi.hdr_len == 0) return 0;
        const uint64_t po = fi.hdr_off + fi.hdr_len;
        const uint64_t pl = (po + fi.payload_len > N) ? N - po : fi.payload_len;
        return chunks_of((uintptr_t)(wire + po), pl);
    }
};

__device__ __forceinline__ uint32_t ld_acq(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// One super tile's survivors in LDS, offset order.
struct StLds {
    uint32_t tcnt[kStTiles];
    uint32_t tsp[kStTiles];
    uint32_t tbase[kStTiles];
    uint32_t off[kStCap];                            // hdr_off - ST start
    uint32_t id[kStCap];                             // slot id
    uint32_t ch[kStCap];                             // unmask chunks of the payload (0: INC)
    uint16_t nx[kStCap];
    uint8_t wt[kStCap];                              // 1: a frame; 0: incomplete header
    union {
        uint64_t ext[kStCap];                        // exit offsets (until nx is built)
        uint32_t sh[2][kStCap];                      // k_merge: chunk sums to P
    };
    uint32_t red32[kMWaves];
    uint64_t red64[kMWaves];
    uint32_t n;
};

// Loads ST s (survivor count returned; nothing loaded past kStCap) and builds nx.
__device__ uint32_t st_load(const MergeParams &P, uint32_t s, StLds &L) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t t0 = s * kStTiles;
    const uint64_t st0 = uint64_t(s) * kStBytes, st_end = st0 + kStBytes;
    uint32_t c = 0, sp = kNone;
    if (tid < kStTiles && t0 + tid < P.n_tiles) {
        c = P.tile_count[t0 + tid];
        sp = P.tile_spill[t0 + tid];
    }
    uint32_t n;
    const uint32_t b = block_excl<uint32_t>(c, L.red32, &n);
    if (n > kStCap) return n;
    if (tid < kStTiles) {
        L.tcnt[tid] = c;
        L.tsp[tid] = sp;
        L.tbase[tid] = b;
    }
    __syncthreads();
    for (uint32_t tl = wv; tl < kStTiles; tl += kMWaves) {
        const uint32_t m = L.tcnt[tl];
        for (uint32_t r = lane; r < m; r += 64) {
            const uint32_t i = L.tbase[tl] + r;
            const uint32_t nid = P.sid(t0 + tl, L.tsp[tl], r);
            const fws_frame_info fi = P.info(nid);
            L.off[i] = (uint32_t)(fi.hdr_off - st0);
            L.id[i] = nid;
            L.wt[i] = fi.hdr_len ? 1 : 0;
            L.ch[i] = (uint32_t)P.node_chunks(fi);
            L.ext[i] = exit_of(fi);
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < n; i += kMThreads) {
        uint16_t v;
        const uint64_t x = L.ext[i];
        if (!L.wt[i]) v = kNxInc;
        else if (x >= P.N) v = kNxEnd;
        else if (x >= st_end) v = kNxExit;
        else {
            const uint32_t xr = (uint32_t)(x - st0);
            uint32_t lo = i + 1, hi = n;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (L.off[mid] < xr) lo = mid + 1; else hi = mid;
            }
            v = (lo < n && L.off[lo] == xr) ? (uint16_t)lo : kNxDead;
        }
        L.nx[i] = v;
    }
    __syncthreads();
    return n;
}

struct MergeWork {
    StLds st;
    uint16_t ptr[2][kStCap];                         // Wyllie pointer (tails point to themselves)
    uint16_t sc[2][kStCap];                          // frames from i up to ptr (exclusive)
    uint32_t lref[kStCap];                           // EXIT tail: index in its ST's tail run
    uint32_t n_tail, tail_base;
};

union MergeLds {
    MergeWork m;
};

// Chain tails, counts and the EXIT tail records of one super tile.
__device__ void merge_st(const MergeParams &P, uint32_t s, uint32_t n, MergeWork &W) {
    StLds &L = W.st;
    const uint32_t tid = threadIdx.x;
    uint32_t *const C = P.counters;
    for (uint32_t i = tid; i < n; i += kMThreads) {
        const uint16_t v = L.nx[i];
        const bool tail = v >= kNxInc;
        W.ptr[0][i] = tail ? (uint16_t)i : v;
        W.sc[0][i] = tail ? 0 : L.wt[i];
        L.sh[0][i] = tail ? 0u : L.ch[i];             // ext[] is dead after st_load
    }
    if (tid == 0) W.n_tail = 0;
    __syncthreads();
    int cur = 0;
    for (;;) {
        int changed = 0;
        for (uint32_t i = tid; i < n; i += kMThreads) {
            const uint16_t p = W.ptr[cur][i];
            const uint16_t q = W.ptr[cur][p];
            if (p != q) {
                W.ptr[cur ^ 1][i] = q;
                W.sc[cur ^ 1][i] = (uint16_t)(W.sc[cur][i] + W.sc[cur][p]);
                L.sh[cur ^ 1][i] = L.sh[cur][i] + L.sh[cur][p];
                changed = 1;
            } else {
                W.ptr[cur ^ 1][i] = p;
                W.sc[cur ^ 1][i] = W.sc[cur][i];
                L.sh[cur ^ 1][i] = L.sh[cur][i];
            }
        }
        cur ^= 1;
        if (!__syncthreads_or(changed)) break;
    }
    for (uint32_t i = tid; i < n; i += kMThreads)
        if (L.nx[i] == kNxExit) W.lref[i] = atomicAdd(&W.n_tail, 1u);
    __syncthreads();
    if (tid == 0) {
        const uint32_t k = W.n_tail;
        uint32_t base = k ? atomicAdd(&C[kCntTails], k) : 0u;
        if (k && (base > P.tail_cap || P.tail_cap - base < k)) {
            atomicOr(&C[kCntFallback], 1u);
            base = kNone;
        }
        W.tail_base = base;
    }
    __syncthreads();
    const uint32_t tb = W.tail_base;
    if (tb == kNone) return;
    for (uint32_t i = tid; i < n; i += kMThreads) {
        const uint32_t t = W.ptr[cur][i];
        const uint32_t kind = kind_of(L.nx[t]);
        const uint32_t cnt = W.sc[cur][i] + L.wt[t];
        const uint64_t cs = (uint64_t)L.sh[cur][i] + L.ch[t];
        const uint32_t ref = kind == kKindExit ? tb + W.lref[t] : L.id[t];
        P.nres[L.id[i]] = fws_node_res{ref, cnt | (kind << 30), cs};
        if (L.nx[i] == kNxExit) {
            const uint64_t x = exit_of(P.info(L.id[i]));
            P.tails[tb + W.lref[i]] = fws_tail_rec{x, L.id[i], kTermDead, (uint32_t)(x / kStBytes), 0u};
        }
    }
}

__global__ __launch_bounds__(kMThreads) void k_merge(MergeParams P) {
    __shared__ MergeLds L;
    const uint32_t s = blockIdx.x, tid = threadIdx.x;
    uint32_t *const C = P.counters;
    // the tail-target bitmap k_link sets
    for (uint64_t w = (uint64_t)s * kMThreads + tid; w < P.tail_cap / 32u + 1u; w += (uint64_t)gridDim.x * kMThreads)
        P.tmark[w] = 0u;
    if (s >= P.n_st) return;
    const uint32_t n = st_load(P, s, L.m.st);
    if (tid == 0) atomicAdd(&C[kCntSurv], n);
    if (n > kStCap) {
        if (tid == 0) atomicOr(&C[kCntFallback], 1u);
        return;
    }
    merge_st(P, s, n, L.m);
}

// ------------------------------------------------------------- k_link + path
constexpr uint32_t kCompCap = 8192;                 // tails that are some tail's next (+ the root's)
constexpr uint16_t kCTerm = 0xFFFF;

struct PathLds {
    uint32_t words[kTailCapMax / 32];                // tail-target bitmap (+ the root's tail)
    uint32_t wpre[kTailCapMax / 32];                 // marked tails before each word
    uint32_t comp[kCompCap];                         // compact index -> tail index
    uint16_t cnx[kCompCap];                          // compact next, or kCTerm
    uint32_t kb[2][kCompCap / 32];                   // kept bitmaps
    uint32_t red32[kMWaves];
    uint64_t red64[kMWaves];
    uint32_t root, rt, crt, end_tail, mc;
};

// The path from offset 0 over the target tails: ST entries and bases,
// terminal, result. Runs in the last k_link workgroup (after every other
// workgroup's release; acquire done by the caller).
__device__ void resolve_path(const MergeParams &P, PathLds &G) {
    uint32_t *const C = P.counters;
    const uint32_t tid = threadIdx.x;
    if (ld_acq(&C[kCntFallback]) || (ld_acq(&C[kCntOverflow]) & 1u)) {
        if (tid == 0) atomicOr(&C[kCntFallback], 1u);
        return;
    }
    const uint32_t M = ld_acq(&C[kCntTails]);
    const uint32_t n_st = P.n_st;
    const uint64_t N = P.N;
    if (tid == 0) {
        uint32_t root = kNone, rt = kNone;
        if (P.n_tiles && P.tile_count[0]) {
            const uint32_t id0 = P.sid(0, P.tile_spill[0], 0);
            if (P.info(id0).hdr_off == 0) root = id0;
        }
        if (root != kNone) {
            const fws_node_res r = P.nres[root];
            if ((r.cnt_kind >> 30) == kKindExit) rt = r.tail;
        }
        G.root = root;
        G.rt = rt;
        G.end_tail = kNone;
    }
    __syncthreads();
    const uint32_t root = G.root, rt = G.rt;

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
    if (mc > kCompCap) {
        if (tid == 0) atomicOr(&C[kCntFallback], 1u);
        return;
    }
    for (uint32_t w = w0; w < w1; ++w) {
        G.wpre[w] = pre;
        uint32_t v = G.words[w];
        while (v) {
            const uint32_t b = (uint32_t)__ffs(v) - 1u;
            v &= v - 1u;
            G.comp[pre++] = w * 32u + b;
        }
    }
    __syncthreads();
    auto rank = [&](uint32_t x) -> uint32_t {
        return G.wpre[x >> 5] + (uint32_t)__popc(G.words[x >> 5] & ((1u << (x & 31u)) - 1u));
    };
    for (uint32_t c = tid; c < mc; c += kMThreads) {
        const uint32_t g = P.gnx[G.comp[c]];
        G.cnx[c] = g >= kGTerm ? kCTerm : (uint16_t)rank(g);
    }
    if (tid == 0) G.crt = rt == kNone ? kNone : rank(rt);
    __syncthreads();
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
    if (!settled) {
        if (tid == 0) atomicOr(&C[kCntFallback], 1u);
        return;
    }

    // entries: the root, and every kept tail's landing survivor
    for (uint32_t s = tid; s < n_st; s += kMThreads) P.st_entry[s] = kNone;
    __syncthreads();
    if (tid == 0 && root != kNone) P.st_entry[0] = root;
    for (uint32_t c = tid; c < mc; c += kMThreads) {
        if ((ka[c >> 5] >> (c & 31u)) & 1u) {
            const uint32_t x = G.comp[c];
            const fws_tail_rec tr = P.tails[x];
            if (tr.w != kTermDead) P.st_entry[tr.wst] = tr.w;
            if (G.cnx[c] == kCTerm) G.end_tail = x;          // exactly one kept tail ends the path
        }
    }
    __syncthreads();

    // per-ST frame and chunk counts, then their exclusive prefix in ST order
    for (uint32_t s = tid; s < n_st; s += kMThreads) {
        const uint32_t e = P.st_entry[s];
        uint32_t c = 0;
        uint64_t k = 0;
        if (e != kNone) {
            const fws_node_res r = P.nres[e];
            c = r.cnt_kind & kCntMask;
            k = r.cs;
        }
        P.st_fbase[s] = c;
        P.st_cbase[s] = k;
    }
    __syncthreads();
    const uint32_t sper = (n_st + kMThreads - 1) / kMThreads;
    const uint32_t lo = tid * sper < n_st ? tid * sper : n_st;
    const uint32_t hi = lo + sper < n_st ? lo + sper : n_st;
    uint32_t fs = 0;
    uint64_t cs = 0;
    for (uint32_t s = lo; s < hi; ++s) {
        fs += P.st_fbase[s];
        cs += P.st_cbase[s];
    }
    uint32_t nf_path;
    uint64_t cs_path;
    uint32_t fpre = block_excl<uint32_t>(fs, G.red32, &nf_path);
    uint64_t cpre = block_excl<uint64_t>(cs, G.red64, &cs_path);
    for (uint32_t s = lo; s < hi; ++s) {
        const uint32_t c = P.st_fbase[s];
        const uint64_t k = P.st_cbase[s];
        P.st_fbase[s] = fpre;
        P.st_cbase[s] = cpre;
        fpre += c;
        cpre += k;
    }

    if (tid != 0) return;
    if (rt != kNone && G.end_tail == kNone) {        // no terminal on the path: cannot happen
        atomicOr(&C[kCntFallback], 1u);
        return;
    }
    // terminal: the path's last header, then ParseFrameHdr from its exit on error
    fws_decode_result r{};
    r.status = FWS_OK;
    r.n_survivors = ld_acq(&C[kCntSurv]);
    uint64_t pos = 0;
    bool walk = N > 0 && root == kNone;              // no chain from offset 0 survived
    if (root != kNone) {
        uint32_t end_id, kind;
        if (rt == kNone) {
            const fws_node_res rr = P.nres[root];
            end_id = rr.tail;
            kind = rr.cnt_kind >> 30;
        } else {
            const fws_tail_rec tr = P.tails[G.end_tail];
            if (tr.w == kTermDead) {
                end_id = tr.id;
                kind = kKindDead;
            } else {
                const fws_node_res rr = P.nres[tr.w];
                end_id = rr.tail;
                kind = rr.cnt_kind >> 30;
            }
        }
        const fws_frame_info fi = P.info(end_id);
        pos = kind == kKindInc ? fi.hdr_off : exit_of(fi);
        walk = kind == kKindDead;
    }
    uint32_t nf = nf_path;
    uint64_t run = cs_path;
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
            const uint64_t pl = (po + h.plen > N) ? N - po : h.plen;
            if (nf < cap) {
                fws_frame_info fi;
                fi.hdr_off = q; fi.payload_len = h.plen; fi.key = h.key; fi.opcode = (uint8_t)h.opcode;
                fi.fin = (uint8_t)h.fin; fi.hdr_len = (uint8_t)rc;
                fi.flags = (po + h.plen > N) ? (uint8_t)FWS_FRAME_TRUNCATED : (uint8_t)0;
                P.frames[nf] = fi;
                P.descs[nf] = fws_frame_desc{po, pl, h.key, 0u};
                const uint64_t c = chunks_of((uintptr_t)(P.wire + po), pl);
                P.cbase[nf] = run;
                if (c) {
                    uint64_t u = (run + kUnitChunks - 1) / kUnitChunks;
                    uint64_t ue = (run + c + kUnitChunks - 1) / kUnitChunks;
                    if (ue > P.unit_cap) ue = P.unit_cap;
                    for (; u < ue; ++u) P.unit_first[u] = nf;
                }
                run += c;
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
    if (lim == 0 || lim > nf_path) {                 // else k_emit's writer of frame lim - 1 closes the plan
        P.cbase[lim] = lim ? run : 0;
        *P.plan_total = lim ? run : 0;
    }
    *P.res = r;
}

// One thread per EXIT tail: the survivor its exit lands on, next(tail), and
// the target bitmap. The last workgroup (atomic ticket) resolves the path.
__global__ __launch_bounds__(kMThreads) void k_link(MergeParams P) {
    __shared__ PathLds G;
    __shared__ uint32_t s_last;
    const uint32_t tid = threadIdx.x;
    uint32_t *const C = P.counters;
    const uint32_t M = C[kCntTails];
    const uint32_t x = blockIdx.x * kMThreads + tid;
    if (x < M && !C[kCntFallback]) {
        fws_tail_rec &tr = P.tails[x];
        const uint32_t w = P.find_node(tr.exit);
        uint32_t g = kGTerm | kKindDead;
        if (w != kTermDead) {
            tr.w = w;
            const fws_node_res r = P.nres[w];
            const uint32_t kind = r.cnt_kind >> 30;
            g = kind == kKindExit ? r.tail : (kGTerm | kind);
        }
        P.gnx[x] = g;
        if (g < kGTerm) atomicOr(&P.tmark[g >> 5], 1u << (g & 31u));
    }
    __threadfence();                                 // release this workgroup's records
    __syncthreads();
    if (tid == 0) s_last = atomicAdd(&C[kCntTicket], 1u) == gridDim.x - 1u;
    __syncthreads();
    if (!s_last) return;
    __threadfence();                                 // acquire every other workgroup's
    resolve_path(P, G);
}

struct EmitLds {
    StLds st;
    uint16_t ptr[2][kStCap];
    uint8_t mark[kStCap];
    uint32_t le;
};

__global__ __launch_bounds__(kMThreads) void k_emit(MergeParams P) {
    __shared__ EmitLds L;
    const uint32_t s = blockIdx.x, tid = threadIdx.x;
    uint32_t *const C = P.counters;
    if (s >= P.n_st || C[kCntFallback]) return;
    const uint32_t e = P.st_entry[s];
    if (e == kNone) return;
    const uint32_t lim = C[kCntFrames], fbase = P.st_fbase[s];
    if (fbase >= lim) return;
    StLds &S = L.st;
    const uint32_t n = st_load(P, s, S);
    if (n > kStCap) return;                          // (k_merge fell back; not reached)
    for (uint32_t i = tid; i < n; i += kMThreads) {
        const uint16_t v = S.nx[i];
        L.ptr[0][i] = v >= kNxInc ? (uint16_t)i : v;
        L.mark[i] = 0;
        if (S.id[i] == e) L.le = i;
    }
    __syncthreads();
    if (tid == 0) L.mark[L.le] = 1;
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
    // frames of the chain in offset order: 4 consecutive nodes per thread
    constexpr uint32_t kPer = kStCap / kMThreads;
    uint32_t fl = 0;
    uint64_t cl = 0;
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
        const uint32_t i = tid * kPer + j;
        if (i < n && L.mark[i] && S.wt[i]) {
            ++fl;
            cl += S.ch[i];
        }
    }
    uint32_t ftot;
    uint64_t ctot;
    uint32_t f = fbase + block_excl<uint32_t>(fl, S.red32, &ftot);
    uint64_t cb = P.st_cbase[s] + block_excl<uint64_t>(cl, S.red64, &ctot);
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
        const uint32_t i = tid * kPer + j;
        if (!(i < n && L.mark[i] && S.wt[i])) continue;
        if (f < lim) {
            const fws_frame_info fi = P.info(S.id[i]);
            const uint64_t po = fi.hdr_off + fi.hdr_len;
            const uint64_t pl = (po + fi.payload_len > P.N) ? P.N - po : fi.payload_len;
            const uint64_t c = S.ch[i];
            if (f < P.cap) P.frames[f] = fi;
            P.descs[f] = fws_frame_desc{po, pl, fi.key, 0u};
            P.cbase[f] = cb;
            if (c) {
                uint64_t u = (cb + kUnitChunks - 1) / kUnitChunks;
                uint64_t ue = (cb + c + kUnitChunks - 1) / kUnitChunks;
                if (ue > P.unit_cap) ue = P.unit_cap;
                for (; u < ue; ++u) P.unit_first[u] = f;
            }
            if (f == lim - 1) {
                P.cbase[lim] = cb + c;
                *P.plan_total = cb + c;
            }
        }
        ++f;
        cb += S.ch[i];
    }
}

}  // namespace fwsk

// ------------------------------------------------------------------ host side
using namespace fwsk;

uint64_t fws_merge_super_tiles(uint64_t n_tiles) { return (n_tiles + kStTiles - 1) / kStTiles; }

uint32_t fws_merge_tail_cap(uint64_t n_tiles) {
    uint64_t c = fws_merge_super_tiles(n_tiles) * 64u + 4096u;
    return (uint32_t)(c < kTailCapMax ? c : kTailCapMax);
}

int fws_launch_merge(fws_gpu_ctx *ctx, const uint8_t *wire, uint64_t N, uint32_t n_tiles, fws_frame_info *frames,
                     uint32_t cap, fws_decode_result *res, hipStream_t s) {
    fws_decode_ws &d = ctx->dec;
    MergeParams P;
    P.wire = wire;
    P.N = N;
    P.n_tiles = n_tiles;
    P.n_st = (uint32_t)fws_merge_super_tiles(n_tiles);
    P.stage_info = d.stage_info;
    P.spill_info = d.spill_info;
    P.tile_count = d.tile_count;
    P.tile_spill = d.tile_spill;
    P.spill_base = n_tiles * kSlots;
    P.tail_cap = d.tail_cap;
    P.counters = d.counters;
    P.nres = d.nres;
    P.tails = d.tails;
    P.gnx = d.gnx;
    P.tmark = d.tmark;
    P.st_entry = d.st_entry;
    P.st_fbase = d.st_fbase;
    P.st_cbase = d.st_cbase;
    P.frames = frames;
    P.cap = cap;
    P.descs = d.descs;
    P.res = res;
    P.cbase = ctx->plan.cbase;
    P.unit_first = ctx->plan.unit_first;
    P.plan_total = ctx->plan.total;
    P.unit_cap = ctx->plan.unit_cap;
    const dim3 grid(P.n_st ? P.n_st : 1u), blk(kMThreads);
    hipLaunchKernelGGL(k_merge, grid, blk, 0, s, P);
    hipLaunchKernelGGL(k_link, dim3((P.tail_cap + kMThreads - 1) / kMThreads), blk, 0, s, P);
    hipLaunchKernelGGL(k_emit, grid, blk, 0, s, P);
    return fws_hip_status(hipGetLastError());
}
