// unmask_kernels.hip -- descriptor-mode XOR unmask for gfx950.
//
// The hot loop of flashws's RX path is WSMaskBytesFast (crypto/ws_mask.h:175)
// called once per frame part from OnRecvData (net/w_socket.h:586,614). Here a
// whole batch of frame payloads is one launch: the payload bytes are cut into
// 16-byte aligned chunks, the chunk space of all frames is concatenated
// (exclusive prefix `cbase`, built by the two plan kernels), and every wave
// owns a 4 KiB unit of that space (64 lanes x 4 chunks), so any mix of frame
// sizes is load-balanced and every full chunk is one global_load_dwordx4 +
// v_xor + global_store_dwordx4 with the key broadcast in registers.
// HBM-bound: bytes = payload read + payload write (+ header bytes of partially
// covered chunks). No LDS, no MFMA.
#include "fws_device.h"
#include "fws_internal.h"
#include "plan_common.h"

namespace fwsk {

// The unmask kernels' streaming stores: write-through nontemporal (`sc1 nt`,
// fws_device.h gstore16_wt) unless kWT is false or the build sets
// FWS_UNMASK_WT=0 (the r05 nontemporal stores, A/B). Measured in one process
// per build, alternating (profiles/r06/ab_wt_stores.jsonl): C2 84.6-84.7 ->
// 83.25-83.4 us, C3 decode 0.181 -> 0.1805 ms, C5 stream 2.659 -> 2.636 ms;
// the sorted UTF-8 kernel (C5 descriptor) 1.430 -> 1.532 ms, so it keeps the
// nontemporal stores (kWT false).
#ifndef FWS_UNMASK_WT
#define FWS_UNMASK_WT 1
#endif
template <bool kNT, bool kWT = true>
__device__ __forceinline__ void ustore16(uintptr_t a, u32x4 v) {
    if constexpr (kNT && kWT && FWS_UNMASK_WT != 0) gstore16_wt(a, v);
    else gstore16<kNT>(a, v);
}

// ---------------------------------------------------------------- plan
constexpr int kPlanItems = 1;                        // frames per thread (k_plan)
constexpr int kPlanTile = kBlock * kPlanItems;       // frames per block

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v, int lane) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        uint64_t t = __shfl_up(v, o, kWave);
        if (lane >= o) v += t;
    }
    return v;
}

// Block exclusive scan of one u64 per thread; returns the block total in *total.
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t *total) {
    __shared__ uint64_t wsum[kBlock / kWave];
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    uint64_t inc = wave_incl_scan(v, lane);
    if (lane == kWave - 1) wsum[w] = inc;
    __syncthreads();
    uint64_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kBlock / kWave; ++i) {
        uint64_t s = wsum[i];
        off += (i < w) ? s : 0;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

__device__ __forceinline__ uint64_t desc_chunks(const uint8_t *base, const fws_frame_desc &d) {
    return chunks_of((uintptr_t)(base + d.payload_off), d.payload_len);
}

// k_plan: the whole descriptor plan in one launch (single-pass scan with a
// decoupled look-back over ticket-ordered blocks, so it never waits on a block
// that has not started). Per frame: the chunk prefix cbase and the chunk-space
// unit map (any descriptor order); the byte-space unit map (frame f owns the
// 4 KiB unit starts in [po_f, po_{f+1})); and whether the payloads are sorted
// and non-overlapping, carried through the look-back with the chunk sums. The
// block holding the last frame writes fws_plan_mode.
//
struct PlanArgs {
    uint64_t *cbase;
    uint32_t *unit_first;
    u32x4 *unit_rec;
    uint64_t *total;
    uint64_t *status;
    uint32_t *ticket;
    fws_plan_mode *mode;
    uint64_t unit_cap;
    uint32_t epoch;
};

// Byte-space unit record (16 B, written by k_plan, one scalar load in the
// run). Fast kind: the unit meets at most two frames A = the owner of its
// first byte and B = the next one, and no outer edge of the batch: x, y =
// their keys rotated for 4-aligned dwords, z = A's payload clipped to the
// unit as [a0, a1) (13 bits each), w = B's [b0, b1). Slow kind (z bit 30):
// x = the owner frame; the run walks the frames from there.
constexpr uint32_t kRecSlow = 1u << 30;

__device__ __forceinline__ uint32_t rec_clip(uint64_t x, uint64_t U0) {
    return x <= U0 ? 0u : (x >= U0 + 4096u ? 4096u : (uint32_t)(x - U0));
}

// U0, E0, E1, po*, pe* base-relative; rk* = aligned_key of the frame.
__device__ __forceinline__ u32x4 unit_record(uint64_t U0, uint64_t E0, uint64_t E1, uint32_t f, uint64_t poA,
                                             uint64_t peA, uint32_t rkA, bool hasB, uint64_t poB, uint64_t peB,
                                             uint32_t rkB, bool hasC, uint64_t poC) {
    if (U0 < E0 || U0 + 4096u > E1 || (hasC && poC < U0 + 4096u)) return u32x4{f, 0u, kRecSlow, 0u};
    const uint32_t a0 = rec_clip(poA, U0), a1 = rec_clip(peA, U0);
    const uint32_t b0 = hasB ? rec_clip(poB, U0) : 0u, b1 = hasB ? rec_clip(peB, U0) : 0u;
    return u32x4{rkA, hasB ? rkB : 0u, a0 | (a1 << 13), b0 | (b1 << 13)};
}


__global__ __launch_bounds__(kBlock) void k_plan(const uint8_t *base, const fws_frame_desc *__restrict__ d,
                                                 uint32_t n, const uint32_t *__restrict__ n_dev, PlanArgs a) {
    __shared__ uint64_t s_wsum[kBlock / kWave];
    __shared__ uint32_t s_wbad[kBlock / kWave];
    if (n_dev && *n_dev < n) n = *n_dev;
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const uint32_t blk = plan_block_order(a.ticket);
    if (n == 0) {
        if (blk == 0 && threadIdx.x == 0) {
            a.cbase[0] = 0;
            *a.total = 0;
            *a.mode = fws_plan_mode{0, 0, 0, 0, 0, {0, 0, 0}};
        }
        return;
    }
    const uintptr_t b0 = (uintptr_t)base;
    // one round of loads: this thread's frame, the next one and the payload
    // start of the one after (unit records), the batch's first and last frame
    static_assert(kPlanItems == 1, "k_plan: one frame per thread");
    const uint64_t f = uint64_t(blk) * kPlanTile + threadIdx.x;
    const bool has = f < n, hasB = f + 1 < n, hasC = f + 2 < n;
    fws_frame_desc fa{0, 0, 0, 0}, fb{0, 0, 0, 0};
    if (has) fa = d[f];
    if (hasB) fb = d[f + 1];
    const uint64_t poC = hasC ? d[f + 2].payload_off : 0;
    const uint64_t po0 = d[0].payload_off;            // byte-space units start at S = (b0 + po_0) & ~15
    const uint64_t last_pe = d[n - 1].payload_off + d[n - 1].payload_len;
    const uint64_t poA = fa.payload_off, peA = fa.payload_off + fa.payload_len;
    const uint64_t poB = fb.payload_off, peB = fb.payload_off + fb.payload_len;
    const uint64_t s = has ? chunks_of(b0 + poA, fa.payload_len) : 0;
    const bool srt = !hasB || (peA >= poA && peA <= poB);
    // block scan of the chunk counts and AND of the sorted bits, one barrier
    const uint64_t inc = wave_incl_scan64(s, lane);
    const uint64_t bad = __ballot(!srt);
    if (lane == kWave - 1) {
        s_wsum[w] = inc;
        s_wbad[w] = bad != 0;
    }
    __syncthreads();
    uint64_t run0 = inc - s, agg = 0;
    bool blk_sorted = true;
#pragma unroll
    for (int i = 0; i < kBlock / kWave; ++i) {
        run0 += i < w ? s_wsum[i] : 0;
        agg += s_wsum[i];
        blk_sorted = blk_sorted && !s_wbad[i];
    }
    bool all_sorted;
    const uint64_t prefix = block_lookback(a.status, blk, agg, blk_sorted, a.epoch, &all_sorted);
    // unit origin S (base-relative, modulo 2^64: below the base when dev_base is
    // not 16-B aligned and the first payload starts within 15 B of it); every
    // comparison below is made on absolute addresses, which never wrap
    const uint64_t Sa = (b0 + po0) & ~uint64_t(15);
    const uint64_t S = Sa - b0;
    const uint64_t cap = a.unit_cap;
    const uint64_t nus = b0 + last_pe > Sa ? (b0 + last_pe - Sa + 4095u) / 4096u : 0;
    uint64_t run = prefix + run0;
    // this frame's unit-map runs: chunk space [cu, cue), byte space [bu, bue)
    uint64_t cu = 0, cue = 0, bu = 0, bue = 0;
    if (has) {
        a.cbase[f] = run;
        if (s) {                                      // chunk space: units starting in this frame
            cu = (run + kUnitChunks - 1) / kUnitChunks;
            cue = (run + s + kUnitChunks - 1) / kUnitChunks;
        }
        run += s;
        // byte space: the unit starts in [po_f, po_{f+1})
        bu = f == 0 ? 0 : (b0 + poA >= Sa ? (b0 + poA - Sa + 4095u) / 4096u : cap);
        bue = !hasB ? nus : (b0 + poB >= Sa ? (b0 + poB - Sa + 4095u) / 4096u : 0);
        if (f == n - 1) {                             // the thread holding the last frame
            a.cbase[n] = run;
            *a.total = run;
            const bool dense = all_sorted && nus + 1 <= cap && (last_pe - S) <= 2u * (run * 16u) + 65536u;
            fws_plan_mode m{dense ? 1ull : 0ull, S, po0, last_pe, nus, {0, 0, 0}};
            *a.mode = m;
        }
    }
    if (cue > cap) cue = cap;                         // contract violation guard, never OOB
    if (bue > cap) bue = cap;
    // byte space is used only for a sorted batch: once a block (or one before
    // it) is out of order its records would be dead writes -- and a permuted
    // batch's runs [po_f, po_{f+1}) span a third of the batch each (C2
    // permuted: 1.43 ms of record writes before this, one 4096-frame block
    // unsorted is enough to know)
    if (!all_sorted) bue = bu;
    if (cue < cu) cue = cu;
    if (bue < bu) bue = bu;
    wave_fill_runs(a.unit_first, cu, (uint32_t)(cue - cu), (uint32_t)f, lane);
    // byte-space records, wave-cooperatively like wave_fill_runs
    struct RecCtx {
        uint64_t poA, peA, poB, peB, poC;
        uint32_t f, rkA, rkB;
        bool hasB, hasC;
    };
    const RecCtx mine{poA, peA, poB, peB, poC, (uint32_t)f, aligned_key(fa.key, fa.phase, b0 + poA),
                      aligned_key(fb.key, fb.phase, b0 + poB), hasB, hasC};
    wave_for_runs(
        bu, (uint32_t)(bue - bu),
        [&](int L) -> RecCtx {
            if (L < 0) return mine;
            return RecCtx{readlane64(mine.poA, L), readlane64(mine.peA, L), readlane64(mine.poB, L),
                          readlane64(mine.peB, L), readlane64(mine.poC, L),
                          (uint32_t)__builtin_amdgcn_readlane(mine.f, L), (uint32_t)__builtin_amdgcn_readlane(mine.rkA, L),
                          (uint32_t)__builtin_amdgcn_readlane(mine.rkB, L),
                          __builtin_amdgcn_readlane((int)mine.hasB, L) != 0,
                          __builtin_amdgcn_readlane((int)mine.hasC, L) != 0};
        },
        [&](const RecCtx &c, uint64_t u) {
            a.unit_rec[u] = unit_record(Sa + 4096u * u, b0 + po0, b0 + last_pe, c.f, b0 + c.poA, b0 + c.peA, c.rkA,
                                        c.hasB, b0 + c.poB, b0 + c.peB, c.rkB, c.hasC, b0 + c.poC);
        });
}

// ---------------------------------------------------------------- unmask
// fws_gpu_mask: one region (WSMaskBytesFast's device twin). One wave = one
// unit of kUnitChunks chunks; a lane's loads are all issued before any
// XOR/store so each lane keeps 64 B in flight.
__global__ __launch_bounds__(kBlock) void k_mask_single(uint8_t *base, fws_frame_desc single) {
    const uintptr_t a0 = (uintptr_t)(base + single.payload_off);
    const uintptr_t lo = a0, hi = a0 + single.payload_len;
    const uint64_t total = chunks_of(a0, single.payload_len);
    const uint64_t n_units = (total + kUnitChunks - 1) / kUnitChunks;
    const uint32_t rk = aligned_key(single.key, single.phase, a0);
    const uintptr_t safe = a0 & ~uintptr_t(15);
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = uint64_t(gridDim.x) * (kBlock / kWave);
    for (uint64_t u = uint64_t(blockIdx.x) * (kBlock / kWave) + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave); u < n_units;
         u += nwaves) {
        uintptr_t ca[kUnmaskU];
        bool live[kUnmaskU], full[kUnmaskU];
        u32x4 v[kUnmaskU];
#pragma unroll
        for (int j = 0; j < kUnmaskU; ++j) {
            const uint64_t g = u * kUnitChunks + uint64_t(j) * kWave + lane;
            live[j] = g < total;
            ca[j] = safe + (uintptr_t)(g << 4);
            full[j] = live[j] && ca[j] >= lo && ca[j] + 16u <= hi;
            // unconditional load so every lane's loads issue back to back
            // before any wait; non-full lanes read the region's first chunk
            v[j] = gload16(full[j] ? ca[j] : safe);
        }
#pragma unroll
        for (int j = 0; j < kUnmaskU; ++j) {
            if (full[j]) gstore16(ca[j], v[j] ^ rk);
            else if (live[j]) xor_partial_chunk(ca[j], lo, hi, rk);
        }
    }
}

// One chunk by the generic path: per-lane search of its frame, then a full
// 16-B XOR or a byte-exact partial one (region heads/tails).
__device__ __forceinline__ void unmask_one_chunk(uint8_t *base, const fws_frame_desc *__restrict__ d,
                                              const uint64_t *__restrict__ cbase, uint32_t flo, uint32_t fhi,
                                              uint64_t g) {
    const uint32_t f = find_frame(cbase, flo, fhi, g);
    const fws_frame_desc fd = d[f];
    const uintptr_t a0 = (uintptr_t)(base + fd.payload_off);
    const uintptr_t ca = (a0 & ~uintptr_t(15)) + (uintptr_t)((g - cbase[f]) << 4);
    const uint32_t rk = aligned_key(fd.key, fd.phase, a0);
    if (ca >= a0 && ca + 16u <= a0 + fd.payload_len) {
        gstore16(ca, gload16(ca) ^ rk);
    } else {
        xor_partial_chunk(ca, a0, a0 + fd.payload_len, rk);
    }
}

// XOR the in-region bytes [lo, hi) of the loaded chunk v at ca and store only
// those (dword stores where a whole dword is inside, byte stores at the edges).
__device__ __forceinline__ void store_partial(uintptr_t ca, u32x4 v, uint32_t rk, uintptr_t lo, uintptr_t hi) {
    const uint32_t w4[4] = {v.x ^ rk, v.y ^ rk, v.z ^ rk, v.w ^ rk};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uintptr_t w = ca + 4u * i;
        if (w >= lo && w + 4u <= hi) {
            *(__attribute__((address_space(1))) uint32_t *)w = w4[i];
        } else if (w + 4u > lo && w < hi) {
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (w + b >= lo && w + b < hi)
                    *(__attribute__((address_space(1))) uint8_t *)(w + b) = (uint8_t)(w4[i] >> (8 * b));
        }
    }
}

// ----------------------------------------------------------- stream space
// Unmask of a decoded wire stream (fws_gpu_decode_stream) in stream-byte
// space: unit u = stream bytes [4 KiB u, 4 KiB (u + 1)), unit_first[u] = the
// frame whose span [hdr_off, next hdr_off) holds the unit's first byte (the
// decode writes it). Every 16-B chunk of the stream belongs to exactly one
// lane, so a chunk is one 16-B load, an XOR with a per-byte key mask (zero on
// header bytes and outside the decoded payloads) and one 16-B store -- no
// partial stores. When the unit meets at most 2 frames (frames >= 4 KiB) the
// metadata is wave-uniform; otherwise each chunk finds its frames.

// Bytes of the dword at w that lie in [lo, hi), as a byte-select mask.
__device__ __forceinline__ uint32_t byte_sel(uint64_t w, uint64_t lo, uint64_t hi) {
    if (w + 4u <= lo || w >= hi) return 0u;
    const uint32_t s = lo > w ? (uint32_t)(lo - w) : 0u;          // 0..3
    const uint32_t e = hi < w + 4u ? (uint32_t)(w + 4u - hi) : 0u; // 0..3
    return (0xFFFFFFFFu << (8u * s)) & (0xFFFFFFFFu >> (8u * e));
}

// Key mask of the chunk at stream offset c (16-aligned) for one payload region
// [po, pe) with key k (phase 0 at po: w_socket.h:504,758).
__device__ __forceinline__ u32x4 region_mask(uint64_t c, uint64_t po, uint64_t pe, uint32_t k) {
    const uint32_t rk = rotr32(k, 8u * ((uint32_t)(c - po) & 3u));
    return u32x4{rk & byte_sel(c, po, pe), rk & byte_sel(c + 4u, po, pe), rk & byte_sel(c + 8u, po, pe),
                 rk & byte_sel(c + 12u, po, pe)};
}

struct StreamFrame {
    uint64_t po, pe;                                 // payload [po, pe), clipped to the stream
    uint32_t key;
    bool text;                                       // UTF-8 checked: TEXT, FIN, complete
};

// A frame record by whole dwords: at a wave-uniform address these are scalar
// loads (a byte field read on its own is a vector load, and its wait would also
// wait for the unit's data loads issued before it)
__device__ __forceinline__ fws_frame_info ld_frame(const fws_frame_info *p) {
    const uint32_t *w = (const uint32_t *)p;
    const uint32_t a0 = w[0], a1 = w[1], a2 = w[2], a3 = w[3], a4 = w[4], a5 = w[5];
    fws_frame_info f;
    f.hdr_off = a0 | (uint64_t(a1) << 32);
    f.payload_len = a2 | (uint64_t(a3) << 32);
    f.key = a4;
    f.opcode = (uint8_t)a5;
    f.fin = (uint8_t)(a5 >> 8);
    f.hdr_len = (uint8_t)(a5 >> 16);
    f.flags = (uint8_t)(a5 >> 24);
    return f;
}

__device__ __forceinline__ StreamFrame stream_frame(const fws_frame_info &fi, uint64_t N) {
    const uint64_t po = fi.hdr_off + fi.hdr_len;
    const uint64_t pe = po + fi.payload_len < N ? po + fi.payload_len : N;
    const bool text = fi.opcode == 1u && fi.fin && !(fi.flags & FWS_FRAME_TRUNCATED) && po + fi.payload_len <= N;
    return StreamFrame{po, pe, fi.key, text};
}

// UTF-8 errors of region R in the unmasked chunk u at stream offset c, given
// the unmasked dword before the chunk; bytes outside R count as zero. The
// first `skip` bytes are not judged (their context is in another unit).
__device__ __forceinline__ bool utf8_chunk_bad(const u32x4 &u, uint32_t prev, uint64_t c, uint64_t lo, uint64_t hi,
                                               uint32_t skip) {
    u32x4 x = u;
    uint32_t p = prev;
    if (!(c >= lo && c + 16u <= hi)) {               // not wholly inside R: zero the outside bytes
        x.x &= sel_bytes(c, lo, hi);
        x.y &= sel_bytes(c + 4u, lo, hi);
        x.z &= sel_bytes(c + 8u, lo, hi);
        x.w &= sel_bytes(c + 12u, lo, hi);
    }
    if (!(c >= lo + 4u && c <= hi)) p &= sel_bytes(c - 4u, lo, hi);
    if (!((x.x | x.y | x.z | x.w | p) & 0x80808080u)) return false;   // ASCII, no open sequence
    uint32_t e0 = utf8_err(x.x, p);
    if (skip) e0 &= 0xFF000000u;                     // bytes 0..2 are judged by k_utf8_seam
    return (e0 | utf8_err(x.y, x.x) | utf8_err(x.z, x.y) | utf8_err(x.w, x.z)) != 0u;
}

// utf8_chunk_bad on unit-relative 32-bit offsets (a fast unit's record: the
// payloads clipped to the unit): chunk at r, region [lo, hi); returns the
// error flags.
__device__ __forceinline__ uint32_t sel_bytes32(int32_t w, int32_t lo, int32_t hi) {
    if (w + 4 <= lo || w >= hi) return 0u;
    const uint32_t s = lo > w ? (uint32_t)(lo - w) : 0u;
    const uint32_t e = hi < w + 4 ? (uint32_t)(w + 4 - hi) : 0u;
    return (0xFFFFFFFFu << (8u * s)) & (0xFFFFFFFFu >> (8u * e));
}
__device__ __forceinline__ uint32_t utf8_chunk_err32(const u32x4 &u, uint32_t prev, int32_t r, int32_t lo, int32_t hi,
                                                     uint32_t skip) {
    u32x4 x = u;
    uint32_t p = prev;
    if (!(r >= lo && r + 16 <= hi)) {
        x.x &= sel_bytes32(r, lo, hi);
        x.y &= sel_bytes32(r + 4, lo, hi);
        x.z &= sel_bytes32(r + 8, lo, hi);
        x.w &= sel_bytes32(r + 12, lo, hi);
    }
    if (!(r >= lo + 4 && r <= hi)) p &= sel_bytes32(r - 4, lo, hi);
    uint32_t e0 = utf8_err(x.x, p);
    if (skip) e0 &= 0xFF000000u;
    return e0 | utf8_err(x.y, x.x) | utf8_err(x.z, x.y) | utf8_err(x.w, x.z);
}

#ifndef FWS_UNMASK_PRE
#define FWS_UNMASK_PRE 1
#endif
#ifndef FWS_ABL_U8
#define FWS_ABL_U8 0
#endif
constexpr bool kUnmaskPre = FWS_UNMASK_PRE != 0;   // A/B: every unit's loads before its frame lookup

// kPf (UTF-8 only, r05): the next unit's loads go out at the top of each unit,
// so they are in flight during this unit's lookup and UTF-8 work (the check
// is ~28 VALU per dword; without the prefetch a wave has no load in flight
// while it runs, and the pass ran 10-15 % above the plain unmask's time)
template <bool kNT, bool kUtf8, bool kRev, bool kPf = false>
__global__ __launch_bounds__(kBlock) void k_unmask_stream(uint8_t *base, uint64_t N,
                                                          const fws_frame_info *__restrict__ fr, uint32_t cap,
                                                          const uint32_t *__restrict__ n_dev,
                                                          const uint32_t *__restrict__ unit_first, uint64_t n_units,
                                                          uint8_t *__restrict__ ok,
                                                          uint32_t *__restrict__ seam) {
    uint32_t n = *n_dev;
    if (n > cap) n = cap;
    if (n == 0) return;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t nwaves = uint64_t(gridDim.x) * (kBlock / kWave);
    const uintptr_t b0 = (uintptr_t)base;
    const uint64_t last = (N - 1u) & ~uint64_t(15);
    auto unit_of = [&](uint64_t ui) -> uint64_t { return kRev ? n_units - 1u - ui : ui; };
    auto load_unit = [&](uint64_t u, u32x4 (&dst)[kUnmaskU]) {
        const uint64_t c0 = u * 4096u + uint64_t(lane) * 16u;
#pragma unroll
        for (int j = 0; j < kUnmaskU; ++j) {
            const uint64_t c = c0 + uint64_t(j) * 1024u;
            dst[j] = gload16<kNT>(b0 + (c < N ? c : last));
        }
    };
    u32x4 nxt[kUnmaskU];
    const uint64_t ui0 = uint64_t(blockIdx.x) * (kBlock / kWave) + wave;
    if constexpr (kPf) {
        if (ui0 < n_units) load_unit(unit_of(ui0), nxt);
    }
    for (uint64_t ui = ui0; ui < n_units; ui += nwaves) {
        // kRev: the first-dispatched waves take the END of the stream, which the
        // decode's scan read last -- those lines are still in the 256 MB
        // Infinity Cache (MALL) when this pass re-reads them
        const uint64_t u = unit_of(ui);
        const uint64_t c0 = u * 4096u + uint64_t(lane) * 16u;
        // kUtf8 (VALU-heavier per unit): the unit's loads are issued before the frame
        // lookup, whose dependent round trips then overlap them
        u32x4 pre[kUnmaskU];
        if constexpr (kPf) {
#pragma unroll
            for (int j = 0; j < kUnmaskU; ++j) pre[j] = nxt[j];
            if (ui + nwaves < n_units) load_unit(unit_of(ui + nwaves), nxt);
            asm volatile("" ::: "memory");
        } else if constexpr (kUtf8 || kUnmaskPre) {
            load_unit(u, pre);
            asm volatile("" ::: "memory");           // issued here, not sunk into the branches
        }
        const uint32_t flo = unit_first[u];
        const uint32_t fhi = (u + 1 < n_units) ? unit_first[u + 1] : n - 1;
        if (!kUtf8 && fhi - flo >= 2u && fhi - flo < 64u) {
            // 3..64 frames meet the unit (frames under ~2 KiB): lane i holds frame
            // flo + i in registers, as unit-relative offsets, and each chunk finds its
            // frames by a binary search over the lanes (ds_bpermute), so the unit costs
            // two dependent global round trips (unit_first, the records) instead of a
            // search through global records per chunk
            const uint32_t nf = fhi - flo + 1u;
            const uint64_t U = u * 4096u;
            u32x4 v[kUnmaskU];
#pragma unroll
            for (int j = 0; j < kUnmaskU; ++j) {      // the unit's data, overlapping the record loads
                const uint64_t c = c0 + uint64_t(j) * 1024u;
                if constexpr (kUnmaskPre) v[j] = pre[j];
                else v[j] = gload16<kNT>(b0 + (c < N ? c : U));
            }
            const fws_frame_info fi = fr[flo + (lane < (int)nf ? (uint32_t)lane : nf - 1u)];
            const StreamFrame sf = stream_frame(fi, N);
            auto rel = [&](uint64_t x) -> int32_t {   // unit-relative, clamped to [-16, 4096 + 16]
                return x + 16u <= U ? -16 : (x >= U + 4112u ? 4112 : (int32_t)(x - U));
            };
            const int32_t fh = rel(fi.hdr_off), fp = rel(sf.po), fe = rel(sf.pe);
            const uint32_t fk = rotr32(sf.key, 8u * ((uint32_t)(U - sf.po) & 3u));   // key phase at 4-aligned bytes
            u32x4 m[kUnmaskU];
#pragma unroll
            for (int j = 0; j < kUnmaskU; ++j) {
                const int32_t rc = j * 1024 + lane * 16;
                uint32_t lo = 0;                      // last frame with hdr_off <= chunk start
#pragma unroll
                for (uint32_t s = 32; s; s >>= 1) {
                    const int32_t h = (int32_t)__shfl((int)fh, (int)(lo + s), 64);
                    if (lo + s < nf && h <= rc) lo += s;
                }
                m[j] = u32x4{0u, 0u, 0u, 0u};
                bool go = true;
                for (uint32_t k = lo;; ++k) {         // the frames from there that start before the chunk end
                    const uint32_t kk = k < 64u ? k : 63u;
                    const int32_t h = (int32_t)__shfl((int)fh, (int)(kk), 64);
                    const int32_t p = (int32_t)__shfl((int)fp, (int)(kk), 64), e = (int32_t)__shfl((int)fe, (int)(kk), 64);
                    const uint32_t key = (uint32_t)__shfl((int)fk, (int)kk, 64);
                    go = go && k < nf && h < rc + 16;
                    if (go) {
                        m[j].x |= key & sel_bytes32(rc, p, e);
                        m[j].y |= key & sel_bytes32(rc + 4, p, e);
                        m[j].z |= key & sel_bytes32(rc + 8, p, e);
                        m[j].w |= key & sel_bytes32(rc + 12, p, e);
                    }
                    if (!__any(go)) break;
                }
            }
#pragma unroll
            for (int j = 0; j < kUnmaskU; ++j) {
                const uint64_t c = c0 + uint64_t(j) * 1024u;
                if (c < N && (m[j].x | m[j].y | m[j].z | m[j].w)) ustore16<kNT>(b0 + c, v[j] ^ m[j]);
            }
            continue;
        }
        if (fhi - flo >= 2u) {                       // small frames: per-chunk search
            uint32_t carry = 0;                      // lane 63's last unmasked dword of step j - 1
#pragma unroll 1
            for (int j = 0; j < kUnmaskU; ++j) {
                const uint64_t c = c0 + uint64_t(j) * 1024u;
                uint32_t lo = flo, hi = fhi;         // last frame with hdr_off <= c
                while (lo < hi) {
                    const uint32_t mid = lo + ((hi - lo + 1u) >> 1);
                    if (fr[mid].hdr_off <= c) lo = mid; else hi = mid - 1u;
                }
                u32x4 m{0u, 0u, 0u, 0u};
                for (uint32_t f = lo; f < n; ++f) {
                    const fws_frame_info fi = fr[f];
                    if (fi.hdr_off >= c + 16u) break;
                    const StreamFrame sf = stream_frame(fi, N);
                    m |= region_mask(c, sf.po, sf.pe, sf.key);
                }
                u32x4 v{0u, 0u, 0u, 0u};
                const bool touched = c < N && (m.x | m.y | m.z | m.w);
                if (kUtf8 ? c < N : touched) v = gload16<kNT>(b0 + c);
                if (touched) ustore16<kNT>(b0 + c, v ^ m);
                if constexpr (kUtf8) {
                    const u32x4 x = v ^ m;
                    uint32_t prev = __shfl_up(x.w, 1, 64);
                    if (lane == 0) prev = carry;
                    carry = __shfl(x.w, 63, 64);
                    // the unit's first and last unmasked dwords for k_utf8_seam
                    if (j == 0 && lane == 0) seam[2u * u] = x.x;
                    if (j == kUnmaskU - 1 && lane == 63) seam[2u * u + 1u] = x.w;
                    // frames whose payload or 3-byte tail meets the chunk (lo - 1: the tail of the one before)
                    for (uint32_t f = lo > flo ? lo - 1u : lo; f < n; ++f) {
                        const fws_frame_info fi = fr[f];
                        if (fi.hdr_off >= c + 16u) break;
                        const StreamFrame sf = stream_frame(fi, N);
                        if (sf.text && c + 16u > sf.po && c < sf.pe + 3u &&
                            utf8_chunk_bad(x, prev, c, sf.po, sf.pe, j == 0 && lane == 0))
                            ok[f] = 0;
                    }
                }
            }
            continue;
        }
        const StreamFrame A = stream_frame(ld_frame(fr + flo), N), B = stream_frame(ld_frame(fr + fhi), N);
        const bool two = fhi != flo;
        if constexpr (kUtf8) {
            const uint64_t U = u * 4096u;
            if (!two && A.text && A.po <= U && A.pe >= U + 4096u) {
                // the unit lies wholly inside one TEXT payload (the common unit of large
                // frames): one key, no per-chunk region tests; a chunk's left context by
                // a DPP wave shift (lane 0: lane 63 of the chunk before, carried)
                const uint32_t rk = rotr32(A.key, 8u * ((uint32_t)(U - A.po) & 3u));
                u32x4 x[kUnmaskU];
#pragma unroll
                for (int j = 0; j < kUnmaskU; ++j) {
                    x[j] = pre[j] ^ u32x4{rk, rk, rk, rk};
                    ustore16<kNT>(b0 + c0 + uint64_t(j) * 1024u, x[j]);
                }
                if (lane == 0) seam[2u * u] = x[0].x;
                if (lane == 63) seam[2u * u + 1u] = x[kUnmaskU - 1].w;
                uint32_t err = 0, carry = 0;
#pragma unroll
                for (int j = 0; j < kUnmaskU; ++j) {
                    const uint32_t prev = __builtin_amdgcn_update_dpp(carry, x[j].w, 0x138, 0xF, 0xF, false);
                    carry = __builtin_amdgcn_readlane(x[j].w, 63);
                    uint32_t e0 = utf8_err(x[j].x, prev);
                    if (j == 0 && lane == 0) e0 &= 0xFF000000u;   // bytes 0..2: k_utf8_seam's
                    err |= e0 | utf8_err(x[j].y, x[j].x) | utf8_err(x[j].z, x[j].y) | utf8_err(x[j].w, x[j].z);
                }
                if (__any(err != 0u) && lane == 0) ok[flo] = 0;
                continue;
            }
        }
        uintptr_t ca[kUnmaskU];
        u32x4 mk[kUnmaskU];
        bool live[kUnmaskU];
#pragma unroll
        for (int j = 0; j < kUnmaskU; ++j) {
            const uint64_t c = c0 + uint64_t(j) * 1024u;
            ca[j] = b0 + c;
            const bool inA = c >= A.po && c + 16u <= A.pe, inB = two && c >= B.po && c + 16u <= B.pe;
            if (inA || inB) {
                const uint32_t rk = inA ? rotr32(A.key, 8u * ((uint32_t)(c - A.po) & 3u))
                                        : rotr32(B.key, 8u * ((uint32_t)(c - B.po) & 3u));
                mk[j] = u32x4{rk, rk, rk, rk};
            } else {
                mk[j] = region_mask(c, A.po, A.pe, A.key);
                if (two) mk[j] |= region_mask(c, B.po, B.pe, B.key);
            }
            live[j] = c < N && (mk[j].x | mk[j].y | mk[j].z | mk[j].w);
        }
        const uintptr_t safe = b0 + (A.po & ~uint64_t(15));
        u32x4 v[kUnmaskU];
#pragma unroll
        for (int j = 0; j < kUnmaskU; ++j) {
            if constexpr (kUtf8 || kUnmaskPre) v[j] = pre[j];    // (a dead chunk's bytes are never stored)
            else v[j] = gload16<kNT>(live[j] ? ca[j] : safe);
        }
#pragma unroll
        for (int j = 0; j < kUnmaskU; ++j)
            if (live[j]) ustore16<kNT>(ca[j], v[j] ^ mk[j]);
        if constexpr (kUtf8) {
            if (A.text || (two && B.text)) {
                bool badA = false, badB = false;
                uint32_t carry = 0;
#pragma unroll
                for (int j = 0; j < kUnmaskU; ++j) {
                    const uint64_t c = c0 + uint64_t(j) * 1024u;
                    const u32x4 x = v[j] ^ mk[j];    // bytes outside A, B are zeroed below
                    uint32_t prev = __shfl_up(x.w, 1, 64);
                    if (lane == 0) prev = carry;
                    carry = __shfl(x.w, 63, 64);
                    // (a unit with no TEXT frame writes no seam words: k_utf8_seam judges
                    // only TEXT payload bytes, and none of this unit's are)
                    if (j == 0 && lane == 0) seam[2u * u] = x.x;
                    if (j == kUnmaskU - 1 && lane == 63) seam[2u * u + 1u] = x.w;
                    const uint32_t skip = j == 0 && lane == 0;
                    if (A.text && c + 16u > A.po && c < A.pe + 3u)
                        badA |= utf8_chunk_bad(x, prev, c, A.po, A.pe, skip);
                    if (two && B.text && c + 16u > B.po && c < B.pe + 3u)
                        badB |= utf8_chunk_bad(x, prev, c, B.po, B.pe, skip);
                }
                if (__any(badA) && lane == 0) ok[flo] = 0;
                if (__any(badB) && lane == 0) ok[fhi] = 0;
            }
        }
    }
}

// The first 3 bytes of every stream unit u in [1, n_units], whose left context
// lies in unit u - 1 (k_unmask_stream skipped them), for the frame holding
// byte 4 KiB * u and the one before it (the 3-byte tail past its payload).
// Reads the already unmasked stream.
__global__ __launch_bounds__(kBlock) void k_utf8_seam(const uint8_t *base, uint64_t N,
                                                      const fws_frame_info *__restrict__ fr, uint32_t cap,
                                                      const uint32_t *__restrict__ n_dev,
                                                      const uint32_t *__restrict__ unit_first, uint64_t n_units,
                                                      uint8_t *__restrict__ ok, const uint32_t *__restrict__ seam) {
    uint32_t n = *n_dev;
    if (n > cap) n = cap;
    const uint64_t u = uint64_t(blockIdx.x) * kBlock + threadIdx.x + 1u;
    if (n == 0 || u > n_units) return;
    const uint64_t P = u * 4096u;
    const uint32_t f = u < n_units ? unit_first[u] : n - 1;
    // the unmask's per-unit record (adjacent words) rather than two stream lines 4 KiB apart
    const uint32_t cur = P < N ? seam[2u * u] : 0u;                      // bytes past N: zeroed below
    const uint32_t prev = seam[2u * u - 1u];
    for (uint32_t g = f > 0 ? f - 1u : 0u; g <= f; ++g) {
        const StreamFrame sf = stream_frame(fr[g], N);
        if (!sf.text || P + 3u <= sf.po || P >= sf.pe + 3u) continue;
        const uint32_t x = cur & sel_bytes(P, sf.po, sf.pe), p = prev & sel_bytes(P - 4u, sf.po, sf.pe);
        if (utf8_err(x, p) & 0x00FFFFFFu) ok[g] = 0;
    }
}


// ------------------------------------------------- descriptor batch, byte space
// k_unmask_desc: the run of a k_plan. When the payloads are sorted and do not
// overlap (fws_plan_mode.byte_space) the batch is unmasked in byte space like a
// decoded stream: unit u = bytes [S + 4 KiB u, S + 4 KiB (u + 1)), every 16-B
// chunk belongs to one lane, and a chunk is one load, an XOR with a per-byte
// key mask (zero outside the payloads) and one full 16-B store. Non-payload
// bytes that share a chunk with payload bytes between the batch's first and
// last payload byte are stored back unchanged; only the batch's two outer edge
// chunks use byte-exact stores. No partial-line writes reach HBM inside the
// batch. Otherwise the chunk-space path (chunk_space_unit).

// Store the bytes of x that lie in [lo, hi) (dword stores where whole).
__device__ __forceinline__ void store_bytes(uintptr_t ca, const u32x4 &x, uintptr_t lo, uintptr_t hi) {
    const uint32_t w4[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uintptr_t w = ca + 4u * i;
        if (w >= lo && w + 4u <= hi) {
            *(__attribute__((address_space(1))) uint32_t *)w = w4[i];
        } else if (w + 4u > lo && w < hi) {
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (w + b >= lo && w + b < hi)
                    *(__attribute__((address_space(1))) uint8_t *)(w + b) = (uint8_t)(w4[i] >> (8 * b));
        }
    }
}

struct DescRegion {
    uint64_t po, pe;                                 // absolute payload [po, pe)
    uint32_t rk;                                     // key for 4-aligned dwords (phase applied)
};

__device__ __forceinline__ DescRegion desc_region(const fws_frame_desc &fd, uintptr_t b0) {
    const uint64_t po = b0 + fd.payload_off;
    return DescRegion{po, po + fd.payload_len, aligned_key(fd.key, fd.phase, po)};
}

__device__ __forceinline__ u32x4 desc_mask(uint64_t c, const DescRegion &r) {
    return u32x4{r.rk & byte_sel(c, r.po, r.pe), r.rk & byte_sel(c + 4u, r.po, r.pe),
                 r.rk & byte_sel(c + 8u, r.po, r.pe), r.rk & byte_sel(c + 12u, r.po, r.pe)};
}


// Bytes of the dword at unit offset o that lie in [lo, hi) (all < 2^13).
__device__ __forceinline__ uint32_t byte_sel32(uint32_t o, uint32_t lo, uint32_t hi) {
    if (o + 4u <= lo || o >= hi) return 0u;
    const uint32_t s = lo > o ? lo - o : 0u, e = hi < o + 4u ? o + 4u - hi : 0u;
    return (0xFFFFFFFFu << (8u * s)) & (0xFFFFFFFFu >> (8u * e));
}

// Slow-kind unit (3+ frames, or an outer edge of the batch): the wave loads
// the frames from the owner on, 64 at a time (lane i: frame flo + i), clips
// each payload to the unit ([0, 4096] offsets, 32-bit) and every lane ORs the
// key masks of the frames starting before the unit's end into its 4 chunks
// (frame k broadcast by readlane); then the 4 loads, XOR and stores. Chunks
// reaching outside [E0, E1) are stored byte-exact.
__device__ __forceinline__ void slow_unit_masks(const fws_frame_desc *__restrict__ d, uint32_t n, uint32_t flo,
                                                uintptr_t b0, uint64_t U0, int lane, u32x4 (&m)[kUnmaskU]) {
#pragma unroll
    for (int j = 0; j < kUnmaskU; ++j) m[j] = u32x4{0u, 0u, 0u, 0u};
    uint32_t o0 = (uint32_t)lane * 16u;
    asm volatile("" : "+v"(o0));                     // opaque: keeps the 16 dword offsets out of registers
    for (uint32_t fb = flo; fb < n; fb += kWave) {
        const uint32_t f = fb + (uint32_t)lane;
        uint32_t lo = 0, hi = 0, rk = 0;
        bool starts = false;
        if (f < n) {
            const fws_frame_desc fd = d[f];
            const uint64_t po = b0 + fd.payload_off;
            starts = po < U0 + 4096u;
            lo = rec_clip(po, U0);
            hi = rec_clip(po + fd.payload_len, U0);
            rk = aligned_key(fd.key, fd.phase, po);
        }
        const int cnt = __popcll(__ballot(starts));  // sorted: a prefix of the lanes
#pragma unroll
        for (int j = 0; j < kUnmaskU; ++j) {         // chunk by chunk: few live registers
            const uint32_t o = o0 + (uint32_t)j * 1024u;
            u32x4 mj = m[j];
#pragma unroll 1
            for (int k = 0; k < cnt; ++k) {
                const uint32_t l = __builtin_amdgcn_readlane(lo, k), h = __builtin_amdgcn_readlane(hi, k);
                if (o + 16u <= l || o >= h) continue;
                const uint32_t r = __builtin_amdgcn_readlane(rk, k);
                mj |= u32x4{r & byte_sel32(o, l, h), r & byte_sel32(o + 4u, l, h), r & byte_sel32(o + 8u, l, h),
                            r & byte_sel32(o + 12u, l, h)};
            }
            m[j] = mj;
        }
        if (cnt < kWave) break;
    }
}

// XOR and store of a slow-kind unit's chunks (loaded from c0 + 1024 j, clamped
// into the span): chunks reaching outside [E0, E1) are stored byte-exact.
template <bool kNT, bool kWT = true>
__device__ __forceinline__ void slow_unit_store(uint64_t c0, uint64_t E0, uint64_t E1, const u32x4 (&v)[kUnmaskU],
                                                const u32x4 (&m)[kUnmaskU]) {
#pragma unroll
    for (int j = 0; j < kUnmaskU; ++j) {
        const uint64_t c = c0 + uint64_t(j) * 1024u;
        if (c >= E1 || !(m[j].x | m[j].y | m[j].z | m[j].w)) continue;
        const u32x4 x = v[j] ^ m[j];
        if (c >= E0 && c + 16u <= E1) ustore16<kNT, kWT>(c, x);
        else store_bytes(c, x, E0, E1);
    }
}

template <bool kNT>
__device__ __forceinline__ void byte_space_unit_slow(uint8_t *base, const fws_frame_desc *__restrict__ d,
                                                     uint32_t n, uint32_t flo, uint64_t E0, uint64_t E1, uint64_t U0,
                                                     int lane) {
    const uint64_t c0 = U0 + uint64_t(lane) * 16u;
    const uint64_t safe = (E1 - 1u) & ~uint64_t(15);   // chunks in [S, E1) hold a byte of the span
    u32x4 m[kUnmaskU];
    slow_unit_masks(d, n, flo, (uintptr_t)base, U0, lane, m);
    u32x4 v[kUnmaskU];
#pragma unroll
    for (int j = 0; j < kUnmaskU; ++j) {
        const uint64_t c = c0 + uint64_t(j) * 1024u;
        v[j] = gload16<kNT>(c < E1 ? c : safe);
    }
    slow_unit_store<kNT>(c0, E0, E1, v, m);
}

// Key masks of a fast-kind unit's four chunks of this lane from its record.
__device__ __forceinline__ void fast_unit_masks(const u32x4 &rec, int lane, u32x4 (&mk)[kUnmaskU]) {
    const uint32_t a0 = rec.z & 0x1FFFu, a1 = (rec.z >> 13) & 0x1FFFu;
    const uint32_t e0 = rec.w & 0x1FFFu, e1 = (rec.w >> 13) & 0x1FFFu;
    uint32_t o0 = (uint32_t)lane * 16u;
    asm volatile("" : "+v"(o0));                     // opaque per unit: no hoisted per-dword offsets
#pragma unroll
    for (int j = 0; j < kUnmaskU; ++j) {
        const uint32_t o = o0 + (uint32_t)j * 1024u;
        const bool inA = o >= a0 && o + 16u <= a1, inB = o >= e0 && o + 16u <= e1;
        if (inA || inB) {
            const uint32_t rk = inA ? rec.x : rec.y;
            mk[j] = u32x4{rk, rk, rk, rk};
        } else {
            mk[j] = u32x4{(rec.x & byte_sel32(o, a0, a1)) | (rec.y & byte_sel32(o, e0, e1)),
                          (rec.x & byte_sel32(o + 4u, a0, a1)) | (rec.y & byte_sel32(o + 4u, e0, e1)),
                          (rec.x & byte_sel32(o + 8u, a0, a1)) | (rec.y & byte_sel32(o + 8u, e0, e1)),
                          (rec.x & byte_sel32(o + 12u, a0, a1)) | (rec.y & byte_sel32(o + 12u, e0, e1))};
        }
    }
}

// One byte-space unit from its k_plan record (fast kind: <= 2 frames, no
// outer edge, so every chunk of the unit lies inside the batch's span).
template <bool kNT>
__device__ __forceinline__ void byte_space_unit(uint8_t *base, const fws_frame_desc *__restrict__ d, uint32_t n,
                                                const u32x4 &rec, const fws_plan_mode &pm, uint64_t u, int lane) {
    const uintptr_t b0 = (uintptr_t)base;
    const uint64_t U0 = b0 + pm.s0 + u * 4096u;
    if (rec.z & kRecSlow) {
        if (pm.last_pe > pm.first_po)
            byte_space_unit_slow<kNT>(base, d, n, rec.x, b0 + pm.first_po, b0 + pm.last_pe, U0, lane);
        return;
    }
    u32x4 mk[kUnmaskU];
    fast_unit_masks(rec, lane, mk);
    const uint64_t c0 = U0 + uint64_t(lane) * 16u;
    u32x4 v[kUnmaskU];
#pragma unroll
    for (int j = 0; j < kUnmaskU; ++j) v[j] = gload16<kNT>(c0 + uint64_t(j) * 1024u);
#pragma unroll
    for (int j = 0; j < kUnmaskU; ++j)
        if (mk[j].x | mk[j].y | mk[j].z | mk[j].w) ustore16<kNT>(c0 + uint64_t(j) * 1024u, v[j] ^ mk[j]);
}


// One chunk-space plan unit (any descriptor order).
template <bool kNT>
__device__ __forceinline__ void chunk_space_unit(uint8_t *base, const fws_frame_desc *__restrict__ d, uint32_t n,
                                                 const uint64_t *__restrict__ cbase,
                                                 const uint32_t *__restrict__ unit_first, uint64_t unit_cap,
                                                 uint64_t total, uint64_t n_units, uint64_t u, int lane) {
    constexpr int J = kUnmaskU;
    const uint32_t flo = unit_owner(unit_first, unit_cap, cbase, n, u, u * kUnitChunks);
    const uint32_t fhi = (u + 1 < n_units) ? unit_owner(unit_first, unit_cap, cbase, n, u + 1, (u + 1) * kUnitChunks)
                                           : n - 1;
    const uint64_t g0 = u * kUnitChunks + lane;
    if (fhi - flo >= 2u) {
#pragma unroll 1
        for (int j = 0; j < J; ++j) {
            const uint64_t g = g0 + uint64_t(j) * kWave;
            if (g < total) unmask_one_chunk(base, d, cbase, flo, fhi, g);
        }
        return;
    }
    const fws_frame_desc d0 = d[flo], d1 = d[fhi];
    const uint64_t CB1 = cbase[flo + 1];
    const uintptr_t a0 = (uintptr_t)(base + d0.payload_off), a1 = (uintptr_t)(base + d1.payload_off);
    const uint64_t A0 = (uint64_t)(a0 & ~uintptr_t(15)) - (cbase[flo] << 4);
    const uint64_t A1 = (uint64_t)(a1 & ~uintptr_t(15)) - (CB1 << 4);
    const uint32_t R0 = aligned_key(d0.key, d0.phase, a0), R1 = aligned_key(d1.key, d1.phase, a1);
    const uint64_t S1 = (fhi > flo) ? CB1 : ~0ull;
    uintptr_t ca[J];
    bool live[J], s1[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const uint64_t g = g0 + uint64_t(j) * kWave;
        s1[j] = g >= S1;
        ca[j] = (uintptr_t)((s1[j] ? A1 : A0) + (g << 4));
        live[j] = g < total;
    }
    const uintptr_t safe = a0 & ~uintptr_t(15);
    u32x4 v[J];
#pragma unroll
    for (int j = 0; j < J; ++j) v[j] = gload16<kNT>(live[j] ? ca[j] : safe);
#pragma unroll
    for (int j = 0; j < J; ++j) {
        if (!live[j]) continue;
        const uintptr_t lo = s1[j] ? a1 : a0, hi = s1[j] ? a1 + d1.payload_len : a0 + d0.payload_len;
        const uint32_t rk = s1[j] ? R1 : R0;
        if (ca[j] >= lo && ca[j] + 16u <= hi) ustore16<kNT>(ca[j], v[j] ^ rk);
        else store_partial(ca[j], v[j], rk, lo, hi);
    }
}

template <bool kNT>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8))) void k_unmask_desc(uint8_t *base, const fws_frame_desc *__restrict__ d,
                                                        uint32_t n, const uint64_t *__restrict__ cbase,
                                                        const uint32_t *__restrict__ unit_first,
                                                        const u32x4 *__restrict__ unit_rec,
                                                        const uint64_t *__restrict__ total_ptr,
                                                        const fws_plan_mode *__restrict__ mode, uint64_t unit_cap) {
    if (n == 0) return;
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = uint64_t(gridDim.x) * (kBlock / kWave);
    const uint64_t u0 = uint64_t(blockIdx.x) * (kBlock / kWave) + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    // first round of scalar loads: the plan words and this wave's first unit
    // record together (index clamped in-bounds; used only if the unit exists)
    const u32x4 rec0 = unit_rec[u0 < unit_cap ? u0 : unit_cap - 1];
    const fws_plan_mode pm = *mode;
    const uint64_t total = *total_ptr;
    if (pm.byte_space) {
        u32x4 rec = rec0;
        for (uint64_t u = u0; u < pm.n_units; u += nwaves) {
            const u32x4 next = (u + nwaves < pm.n_units) ? unit_rec[u + nwaves] : rec;   // prefetch
            byte_space_unit<kNT>(base, d, n, rec, pm, u, lane);
            rec = next;
        }
        return;
    }
    // every unit of the batch: past the unit map's capacity (a batch larger than
    // the reservation) the owners come from a search of cbase
    const uint64_t n_units = (total + kUnitChunks - 1) / kUnitChunks;
    for (uint64_t u = u0; u < n_units; u += nwaves)
        chunk_space_unit<kNT>(base, d, n, cbase, unit_first, unit_cap, total, n_units, u, lane);
}

#ifndef FWS_SORTED_WPE
#define FWS_SORTED_WPE 6
#endif
// ---------------------------------------------------------------- sorted, one launch
// fws_gpu_unmask_sorted: k_unmask_desc's byte-space unmask without k_plan, for
// batches whose descriptors are sorted by payload_off and non-overlapping (a
// packed read batch, the decoder's frame list). Each wave finds the owner of
// its unit's first byte (the last frame with payload_off <= U0, else frame 0,
// as k_plan assigns it) by itself: an interpolation guess from the batch span,
// one scalar round of four payload offsets around it, and a binary search only
// when the guess misses (uneven frame sizes). It then builds the record k_plan
// would have written (unit_record) and runs the same unit body. Units that
// meet no payload (gaps of a sparse batch) are skipped without loads.
// Absolute addresses throughout (U0, po: base + offset), so a dev_base that is
// not 16-B aligned never wraps the unit origin below the base.
// rate = frames per 4 KiB unit of the span (the guess of unit u is u * rate).
__device__ __forceinline__ uint32_t sorted_owner(const fws_frame_desc *__restrict__ d, uint32_t n, uintptr_t b0,
                                                 uint64_t U0, uint64_t po0, uint64_t u, float rate) {
    if (U0 < po0 || n == 1) return 0u;
    const float gf = (float)(uint32_t)u * rate;
    uint64_t g = (uint32_t)__builtin_amdgcn_readfirstlane((int)(gf < 4.0e9f ? (uint32_t)gf : 0xFFFFFFFFu));
    g = g >= 1u ? g - 1u : 0u;
    if (g > n - 1u) g = n - 1u;
    uint64_t p[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) p[k] = b0 + d[g + k < n ? g + k : n - 1u].payload_off;   // one scalar round
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint64_t i = g + k;
        if (i < n && p[k] <= U0 && (i + 1u >= n || p[k + 1] > U0)) return (uint32_t)i;
    }
    uint32_t lo = 0, hi = n;                         // count of frames starting at or before U0 (>= 1)
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2u;
        if (b0 + d[mid].payload_off <= U0) lo = mid + 1u;
        else hi = mid;
    }
    return lo - 1u;
}

// kEarly: the unit's data loads are issued before the owner lookup (their
// addresses depend only on the span), so the lookup's scalar rounds overlap
// the HBM latency; gap units then cost their loads. Without it, the lookup
// comes first and units that meet no payload are skipped without loads.
// UTF-8 of one chunk of a slow-kind unit (kUtf8): every non-empty region that
// meets the chunk as payload or 3-byte tail, found per lane (the last region
// starting before the chunk end by binary search from the unit's owner, then
// walking down while the region's tail still reaches the chunk; pe is
// non-decreasing over sorted disjoint regions).
__device__ __forceinline__ void utf8_slow_chunk(const fws_frame_desc *__restrict__ d, uint32_t n, uint32_t A,
                                                uintptr_t b0, uint64_t c, const u32x4 &x, uint32_t prev,
                                                uint32_t skip, uint8_t *__restrict__ ok) {
    if (b0 + d[A].payload_off >= c + 16u) return;
    uint32_t lo = A, hi = n - 1u;                    // last f with po_f < c + 16
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo + 1u) >> 1);
        if (b0 + d[mid].payload_off < c + 16u) lo = mid;
        else hi = mid - 1u;
    }
    for (uint32_t f = lo + 1u; f-- > A;) {
        const fws_frame_desc fd = d[f];
        const uint64_t po = b0 + fd.payload_off, pe = po + fd.payload_len;
        if (pe + 3u <= c) break;
        if (fd.payload_len && utf8_chunk_bad(x, prev, c, po, pe, skip)) ok[f] = 0;
    }
}

// Workgroup -> unit order with each XCD on runs of 8 consecutive workgroups
// (32 units): workgroups are dealt round robin over the 8 XCDs, so in the
// plain order every 16 KiB of units changes XCD and the descriptor lines at
// the seams are fetched by two XCDs' L2s. Within each group of 64 workgroups,
// dispatch slot r = 8 k + x becomes workgroup 8 x + k. A speed choice only
// (dispatch order and placement are not promised); the last partial group
// keeps the plain order, so the map is a bijection on any grid.
__device__ __forceinline__ uint32_t xcd_run_block(uint32_t b, uint32_t nb) {
    const uint32_t g = b >> 6;
    if ((g << 6) + 64u > nb) return b;
    const uint32_t r = b & 63u;
    return (g << 6) | ((r & 7u) << 3) | (r >> 3);
}

template <bool kNT, bool kEarly, bool kUtf8 = false, bool kXcdRun = false>
__device__ __forceinline__ void unmask_sorted_body(uint8_t *base, const fws_frame_desc *__restrict__ d, uint32_t n,
                                                   uint8_t *__restrict__ ok = nullptr,
                                                   uint32_t *__restrict__ seam = nullptr,
                                                   uint64_t seam_units = 0) {
    if (n == 0) return;
    const int lane = threadIdx.x & (kWave - 1);
    const uintptr_t b0 = (uintptr_t)base;
    const uint64_t nwaves = uint64_t(gridDim.x) * (kBlock / kWave);
    const uint32_t blk = kXcdRun ? xcd_run_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint64_t u0 = uint64_t(blk) * (kBlock / kWave) + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t po0 = d[0].payload_off;
    const fws_frame_desc dl = d[n - 1];
    const uint64_t last_pe = dl.payload_off + dl.payload_len;
    const uint64_t E0 = b0 + po0, E1 = b0 + last_pe;   // absolute span of the batch's payloads
    const uint64_t Sa = E0 & ~uint64_t(15);
    const uint64_t nus = E1 > Sa ? (E1 - Sa + 4095u) / 4096u : 0;
    const uint64_t safe = (E1 - 1u) & ~uint64_t(15);   // chunk holding the span's last byte
    const float rate = (float)n * 4096.0f / (float)(E1 > E0 ? E1 - E0 : 1u);
    for (uint64_t u = u0; u < nus; u += nwaves) {
        const uint64_t U0 = Sa + 4096u * u;
        const uint64_t c0 = U0 + uint64_t(lane) * 16u;
        u32x4 v[kUnmaskU];
        if (kEarly) {
#pragma unroll
            for (int j = 0; j < kUnmaskU; ++j) {
                const uint64_t c = c0 + uint64_t(j) * 1024u;
                v[j] = gload16<kNT>(c < E1 ? c : safe);
            }
        }
        const uint32_t A = sorted_owner(d, n, b0, U0, E0, u, rate);
        const bool hasB = A + 1u < n, hasC = A + 2u < n;
        const fws_frame_desc fa = d[A];
        fws_frame_desc fb{0, 0, 0, 0};
        if (hasB) fb = d[A + 1u];
        const uint64_t poC = hasC ? b0 + d[A + 2u].payload_off : 0;
        const uint64_t poA = b0 + fa.payload_off, peA = poA + fa.payload_len;
        const uint64_t poB = b0 + fb.payload_off, peB = poB + fb.payload_len;
        const u32x4 rec = unit_record(U0, E0, E1, A, poA, peA, aligned_key(fa.key, fa.phase, poA), hasB, poB, peB,
                                      aligned_key(fb.key, fb.phase, poB), hasC, poC);
        const bool slow = (rec.z & kRecSlow) != 0;
        // seam words exist for units below seam_units (the context's seam buffer); a
        // unit past it (a batch wider than the reservation) leaves its two dwords to
        // k_utf8_seam_sorted's stream reads
        const bool sw = u < seam_units;
        if constexpr (kUtf8) {
            if (rec.z == (4096u << 13) && ((rec.w >> 13) & 0x1FFFu) <= (rec.w & 0x1FFFu)) {
                // the unit lies wholly inside A's payload and B has no byte in it (the
                // common unit of large frames): one key, no per-chunk region tests;
                // a chunk's left context by a DPP wave shift (lane 0: lane 63 of the
                // chunk before, bound_ctrl off keeps the carried value)
                u32x4 x[kUnmaskU];
#pragma unroll
                for (int j = 0; j < kUnmaskU; ++j) x[j] = kEarly ? v[j] : gload16<kNT>(c0 + uint64_t(j) * 1024u);
                const uint32_t rk = rec.x;
#pragma unroll
                for (int j = 0; j < kUnmaskU; ++j) {
                    x[j] = x[j] ^ u32x4{rk, rk, rk, rk};
                    ustore16<kNT, !kUtf8>(c0 + uint64_t(j) * 1024u, x[j]);
                }
                // the unit's first and last unmasked dwords for k_utf8_seam_sorted
#if (FWS_ABL_U8 & 2) == 0          // (ablation builds only: make exp EXP_DEFS=-DFWS_ABL_U8=1|2|3)
                if (sw && lane == 0) seam[2u * u] = x[0].x;
                if (sw && lane == 63) seam[2u * u + 1u] = x[kUnmaskU - 1].w;
#endif
#if (FWS_ABL_U8 & 1) == 0
                uint32_t err = 0, carry = 0;
#pragma unroll
                for (int j = 0; j < kUnmaskU; ++j) {
                    const uint32_t prev = __builtin_amdgcn_update_dpp(carry, x[j].w, 0x138, 0xF, 0xF, false);
                    carry = __builtin_amdgcn_readlane(x[j].w, 63);
                    uint32_t e0 = utf8_err(x[j].x, prev);
                    if (j == 0 && lane == 0) e0 &= 0xFF000000u;   // bytes 0..2: k_utf8_seam_sorted's
                    err |= e0 | utf8_err(x[j].y, x[j].x) | utf8_err(x[j].z, x[j].y) | utf8_err(x[j].w, x[j].z);
                }
                if (__any(err != 0u) && lane == 0) ok[A] = 0;
#endif
                continue;
            }
        }
        if ((!kEarly || kUtf8) && !slow) {
            const uint32_t a0 = rec.z & 0x1FFFu, a1 = (rec.z >> 13) & 0x1FFFu;
            const uint32_t e0 = rec.w & 0x1FFFu, e1 = (rec.w >> 13) & 0x1FFFu;
            // a gap between payloads (a tail of A reaches at most bytes 0..2: the seam kernel's)
            if (a1 <= a0 && e1 <= e0) continue;
        }
        u32x4 m[kUnmaskU];
        if (slow) slow_unit_masks(d, n, A, b0, U0, lane, m);
        else fast_unit_masks(rec, lane, m);
        if (!kEarly) {
#pragma unroll
            for (int j = 0; j < kUnmaskU; ++j) {
                const uint64_t c = c0 + uint64_t(j) * 1024u;
                v[j] = gload16<kNT>(c < E1 ? c : safe);
            }
        }
        if constexpr (kUtf8) {
            // unmask in place (the masks die here: fewer live registers in the UTF-8 pass)
#pragma unroll
            for (int j = 0; j < kUnmaskU; ++j) {
                const bool t = (m[j].x | m[j].y | m[j].z | m[j].w) != 0u;
                v[j] = v[j] ^ m[j];
                const uint64_t c = c0 + uint64_t(j) * 1024u;
                if (!t || (slow && c >= E1)) continue;
                if (!slow || (c >= E0 && c + 16u <= E1)) ustore16<kNT, !kUtf8>(c, v[j]);
                else store_bytes(c, v[j], E0, E1);
            }
        } else if (slow) {
            slow_unit_store<kNT>(c0, E0, E1, v, m);
        } else {
#pragma unroll
            for (int j = 0; j < kUnmaskU; ++j)      // fast kind: every chunk lies inside [E0, E1)
                if (m[j].x | m[j].y | m[j].z | m[j].w) ustore16<kNT, !kUtf8>(c0 + uint64_t(j) * 1024u, v[j] ^ m[j]);
        }
        if constexpr (kUtf8) {
            // the unmasked chunks, still in registers; a chunk's left context is the previous
            // lane's last dword (lane 0: lane 63's of chunk j - 1). Bytes 0..2 of the unit are
            // judged by k_utf8_seam_sorted (their context is another wave's unit).
            if (slow) {
                uint32_t carry = 0;
#pragma unroll
                for (int j = 0; j < kUnmaskU; ++j) {
                    const u32x4 x = v[j];
                    uint32_t prev = __shfl_up(x.w, 1, 64);
                    if (lane == 0) prev = carry;
                    carry = __shfl(x.w, 63, 64);
                    if (sw && j == 0 && lane == 0) seam[2u * u] = x.x;
                    if (sw && j == kUnmaskU - 1 && lane == 63) seam[2u * u + 1u] = x.w;
                    utf8_slow_chunk(d, n, A, b0, c0 + uint64_t(j) * 1024u, x, prev, j == 0 && lane == 0, ok);
                }
                continue;
            }
            // fast kind: the unit-clipped payloads of A and B from the unit record, as
            // 32-bit unit offsets (a region ending inside the unit's last 3 bytes leaves
            // its truncation flag to bytes 0..2 of the next unit: k_utf8_seam_sorted's)
            const int32_t loA = rec.z & 0x1FFFu, hiA = (rec.z >> 13) & 0x1FFFu;
            const int32_t loB = rec.w & 0x1FFFu, hiB = (rec.w >> 13) & 0x1FFFu;
            uint32_t errA = 0, errB = 0;
            uint32_t carry = 0;
            int32_t r0 = lane * 16;
            asm volatile("" : "+v"(r0));             // opaque per unit: no hoisted per-dword offsets
#pragma unroll
            for (int j = 0; j < kUnmaskU; ++j) {
                const u32x4 x = v[j];
                uint32_t prev = __shfl_up(x.w, 1, 64);
                if (lane == 0) prev = carry;
                carry = __shfl(x.w, 63, 64);
                if (sw && j == 0 && lane == 0) seam[2u * u] = x.x;
                if (sw && j == kUnmaskU - 1 && lane == 63) seam[2u * u + 1u] = x.w;
                const uint32_t skip = j == 0 && lane == 0;
                const int32_t r = r0 + j * 1024;
                if (r + 16 > loA && r < hiA + 3) errA |= utf8_chunk_err32(x, prev, r, loA, hiA, skip);
                if (r + 16 > loB && r < hiB + 3) errB |= utf8_chunk_err32(x, prev, r, loB, hiB, skip);
            }
            if (__any(errA != 0u) && lane == 0) ok[A] = 0;
            if (__any(errB != 0u) && lane == 0) ok[A + 1u] = 0;
        }
    }
}

// The first 3 bytes of every unit u in [0, n_units) of a sorted batch, whose
// left context lies in unit u - 1 (k_unmask_sorted_utf8 skipped them), for
// every non-empty region meeting them as payload or 3-byte tail. One thread
// per unit seam; reads the already unmasked bytes. The owner of the seam is
// found like sorted_owner, per thread.
__global__ __launch_bounds__(kBlock) void k_utf8_seam_sorted(const uint8_t *base, const fws_frame_desc *__restrict__ d,
                                                             uint32_t n, uint8_t *__restrict__ ok,
                                                             const uint32_t *__restrict__ seam, uint64_t seam_units) {
    if (n == 0) return;
    const uintptr_t b0 = (uintptr_t)base;
    const uint64_t E0 = b0 + d[0].payload_off;
    const fws_frame_desc dl = d[n - 1];
    const uint64_t E1 = b0 + dl.payload_off + dl.payload_len;
    const uint64_t Sa = E0 & ~uint64_t(15);
    const uint64_t nus = E1 > Sa ? (E1 - Sa + 4095u) / 4096u : 0;
    const float rate = (float)n / (float)(E1 > E0 ? E1 - E0 : 1u);
    // unit 0 too (r06): its bytes 0..2 are payload when the first region starts
    // within 2 bytes past a 16-B boundary, and the unmask skips them in every unit
#ifndef FWS_SEAM_U0
#define FWS_SEAM_U0 1                                // 0: the r05 loop from unit 1 (A/B of the test only)
#endif
    for (uint64_t u = uint64_t(blockIdx.x) * kBlock + threadIdx.x + (FWS_SEAM_U0 ? 0u : 1u); u < nus;
         u += uint64_t(gridDim.x) * kBlock) {
    const uint64_t P = Sa + 4096u * u;               // P < E1: the dwords at P - 4 and P are in the span's chunks
    if (u == 0 && E0 >= P + 3u) continue;            // no region byte among unit 0's first 3
    // last region with po < P + 3: guess from the span, bracket check, else binary search
    uint64_t g = P > E0 ? (uint64_t)((float)(P - E0) * rate) : 0u;
    g = g >= 1u ? g - 1u : 0u;
    if (g > n - 1u) g = n - 1u;
    uint32_t L;
    const bool lo_ok = b0 + d[g].payload_off < P + 3u;
    const bool hi_ok = g + 1u >= n || b0 + d[g + 1u].payload_off >= P + 3u;
    if (lo_ok && hi_ok) {
        L = (uint32_t)g;
    } else {
        uint32_t lo = 0, hi = n - 1u;
        while (lo < hi) {
            const uint32_t mid = lo + ((hi - lo + 1u) >> 1);
            if (b0 + d[mid].payload_off < P + 3u) lo = mid;
            else hi = mid - 1u;
        }
        L = lo;
    }
    // the unmask's per-unit record (two adjacent words per thread) rather than two
    // stream lines 4 KiB apart; the software-pipelined unmask writes none (seam null)
    const bool sw = seam && u < seam_units;          // else the unmask wrote no words for u
    uint32_t cur = 0, prev = 0;                      // unit 0: no region byte lies before it
    if (u == 0) {
        if (sw) {
            cur = seam[0];
        } else {                                     // the bytes at or past E0 (>= base) only
            for (uint32_t k = 0; k < 4u; ++k)
                if (P + k >= E0) cur |= (uint32_t)gget(base + (P + k - b0)) << (8u * k);
        }
    } else {
        cur = sw ? seam[2u * u] : *(const uint32_t *)(base + (P - b0));
        prev = sw ? seam[2u * u - 1u] : *(const uint32_t *)(base + (P - 4u - b0));
    }
    for (uint32_t f = L + 1u; f-- > 0;) {
        const fws_frame_desc fd = d[f];
        const uint64_t po = b0 + fd.payload_off, pe = po + fd.payload_len;
        if (pe + 3u <= P) break;
        if (!fd.payload_len || po >= P + 3u) continue;
        const uint32_t x = cur & sel_bytes(P, po, pe), p = prev & sel_bytes(P - 4u, po, pe);
        if (utf8_err(x, p) & 0x00FFFFFFu) ok[f] = 0;
    }
    }
}

// k_unmask_sorted (lookup first, 8 waves per SIMD, no spills) is the default;
// k_unmask_sorted_early needs 80 VGPRs (the unit's 16 data registers live
// across the lookup and the slow-kind mask walk) and measured slower at 6
// waves per SIMD (84.9 vs 82.7 us on C2), kept behind the tuning hook
template <bool kNT>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(FWS_SORTED_WPE))) void k_unmask_sorted_early(
    uint8_t *base, const fws_frame_desc *__restrict__ d, uint32_t n) {
    unmask_sorted_body<kNT, true>(base, d, n);
}

template <bool kNT, bool kXcdRun = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8))) void k_unmask_sorted(
    uint8_t *base, const fws_frame_desc *__restrict__ d, uint32_t n) {
    unmask_sorted_body<kNT, false, false, kXcdRun>(base, d, n);
}

// Software-pipelined form of unmask_sorted_body<.., kUtf8 = true>: a wave's
// grid-stride units (16 per wave on C5) are processed so that the next unit's
// owner lookup and data loads are issued before the current unit's UTF-8
// check, whose VALU work then overlaps the next unit's HBM latency.
struct SortedUnit {
    uint64_t U0, poA, peA, poB, peB;
    u32x4 rec;
    uint32_t A, lenA, lenB;
    bool hasB, slow, gap;
};

template <bool kNT>
__device__ __forceinline__ void unmask_sorted_utf8_pipe(uint8_t *base, const fws_frame_desc *__restrict__ d,
                                                        uint32_t n, uint8_t *__restrict__ ok,
                                                        uint32_t *__restrict__ seam, uint64_t seam_units) {
    if (n == 0) return;
    const int lane = threadIdx.x & (kWave - 1);
    const uintptr_t b0 = (uintptr_t)base;
    const uint64_t nwaves = uint64_t(gridDim.x) * (kBlock / kWave);
    const uint64_t u0 = uint64_t(blockIdx.x) * (kBlock / kWave) + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t po0 = d[0].payload_off;
    const fws_frame_desc dl = d[n - 1];
    const uint64_t E0 = b0 + po0, E1 = b0 + dl.payload_off + dl.payload_len;
    const uint64_t Sa = E0 & ~uint64_t(15);
    const uint64_t nus = E1 > Sa ? (E1 - Sa + 4095u) / 4096u : 0;
    const uint64_t safe = (E1 - 1u) & ~uint64_t(15);
    const float rate = (float)n * 4096.0f / (float)(E1 > E0 ? E1 - E0 : 1u);
    auto lookup = [&](uint64_t u) -> SortedUnit {
        SortedUnit I;
        I.U0 = Sa + 4096u * u;
        I.A = sorted_owner(d, n, b0, I.U0, E0, u, rate);
        I.hasB = I.A + 1u < n;
        const bool hasC = I.A + 2u < n;
        const fws_frame_desc fa = d[I.A];
        fws_frame_desc fb{0, 0, 0, 0};
        if (I.hasB) fb = d[I.A + 1u];
        const uint64_t poC = hasC ? b0 + d[I.A + 2u].payload_off : 0;
        I.poA = b0 + fa.payload_off;
        I.peA = I.poA + fa.payload_len;
        I.poB = b0 + fb.payload_off;
        I.peB = I.poB + fb.payload_len;
        I.lenA = fa.payload_len != 0;
        I.lenB = fb.payload_len != 0;
        I.rec = unit_record(I.U0, E0, E1, I.A, I.poA, I.peA, aligned_key(fa.key, fa.phase, I.poA), I.hasB, I.poB,
                            I.peB, aligned_key(fb.key, fb.phase, I.poB), hasC, poC);
        I.slow = (I.rec.z & kRecSlow) != 0;
        const uint32_t a0 = I.rec.z & 0x1FFFu, a1 = (I.rec.z >> 13) & 0x1FFFu;
        const uint32_t e0 = I.rec.w & 0x1FFFu, e1 = (I.rec.w >> 13) & 0x1FFFu;
        I.gap = !I.slow && a1 <= a0 && e1 <= e0;     // no payload (a tail of A: bytes 0..2, the seam's)
        return I;
    };
    auto load = [&](const SortedUnit &I, u32x4 (&v)[kUnmaskU]) {
        if (I.gap) return;
        const uint64_t c0 = I.U0 + uint64_t(lane) * 16u;
#pragma unroll
        for (int j = 0; j < kUnmaskU; ++j) {
            const uint64_t c = c0 + uint64_t(j) * 1024u;
            v[j] = gload16<kNT>(c < E1 ? c : safe);
        }
    };
    uint64_t u = u0;
    if (u >= nus) return;
    SortedUnit cur = lookup(u);
    u32x4 v[kUnmaskU];
    load(cur, v);
    for (;;) {
        const uint64_t c0 = cur.U0 + uint64_t(lane) * 16u;
        u32x4 x[kUnmaskU];
        // one key: the unit lies wholly inside A's payload and B has no byte in it (the
        // common unit of large frames, as in unmask_sorted_body)
        const bool onekey = !cur.slow && cur.rec.z == (4096u << 13) &&
                            ((cur.rec.w >> 13) & 0x1FFFu) <= (cur.rec.w & 0x1FFFu);
        if (onekey) {
            const uint32_t rk = cur.rec.x;
#pragma unroll
            for (int j = 0; j < kUnmaskU; ++j) {
                x[j] = v[j] ^ u32x4{rk, rk, rk, rk};
                ustore16<kNT, false>(c0 + uint64_t(j) * 1024u, x[j]);
            }
        } else if (!cur.gap) {
            u32x4 m[kUnmaskU];
            if (cur.slow) slow_unit_masks(d, n, cur.A, b0, cur.U0, lane, m);
            else fast_unit_masks(cur.rec, lane, m);
            if (cur.slow) {
                slow_unit_store<kNT, false>(c0, E0, E1, v, m);
            } else {
#pragma unroll
                for (int j = 0; j < kUnmaskU; ++j)
                    if (m[j].x | m[j].y | m[j].z | m[j].w) ustore16<kNT, false>(c0 + uint64_t(j) * 1024u, v[j] ^ m[j]);
            }
#pragma unroll
            for (int j = 0; j < kUnmaskU; ++j) x[j] = v[j] ^ m[j];
        }
        // the next unit's lookup and loads go out before this unit's UTF-8 work
        const uint64_t un = u + nwaves;
        const bool more = un < nus;
        SortedUnit nx;
        if (more) {
            nx = lookup(un);
            load(nx, v);
        }
        // the unit's first and last unmasked dwords for k_utf8_seam_sorted
        if (!cur.gap && u < seam_units) {
            if (lane == 0) seam[2u * u] = x[0].x;
            if (lane == 63) seam[2u * u + 1u] = x[kUnmaskU - 1].w;
        }
        if (onekey) {
            uint32_t err = 0, carry = 0;
#pragma unroll
            for (int j = 0; j < kUnmaskU; ++j) {
                const uint32_t prev = __builtin_amdgcn_update_dpp(carry, x[j].w, 0x138, 0xF, 0xF, false);
                carry = __builtin_amdgcn_readlane(x[j].w, 63);
                uint32_t e0 = utf8_err(x[j].x, prev);
                if (j == 0 && lane == 0) e0 &= 0xFF000000u;   // bytes 0..2: k_utf8_seam_sorted's
                err |= e0 | utf8_err(x[j].y, x[j].x) | utf8_err(x[j].z, x[j].y) | utf8_err(x[j].w, x[j].z);
            }
            if (__any(err != 0u) && lane == 0) ok[cur.A] = 0;
        } else if (!cur.gap) {
            bool badA = false, badB = false;
            uint32_t carry = 0;
#pragma unroll
            for (int j = 0; j < kUnmaskU; ++j) {
                const uint64_t c = c0 + uint64_t(j) * 1024u;
                uint32_t prev = __shfl_up(x[j].w, 1, 64);
                if (lane == 0) prev = carry;
                carry = __shfl(x[j].w, 63, 64);
                const uint32_t skip = j == 0 && lane == 0;
                if (cur.slow) {
                    utf8_slow_chunk(d, n, cur.A, b0, c, x[j], prev, skip, ok);
                    continue;
                }
                if (cur.lenA && c + 16u > cur.poA && c < cur.peA + 3u)
                    badA |= utf8_chunk_bad(x[j], prev, c, cur.poA, cur.peA, skip);
                if (cur.hasB && cur.lenB && c + 16u > cur.poB && c < cur.peB + 3u)
                    badB |= utf8_chunk_bad(x[j], prev, c, cur.poB, cur.peB, skip);
            }
            if (!cur.slow) {
                if (__any(badA) && lane == 0) ok[cur.A] = 0;
                if (__any(badB) && lane == 0) ok[cur.A + 1u] = 0;
            }
        }
        if (!more) break;
        cur = nx;
        u = un;
    }
}

// unmask + per-region UTF-8 flags (C5 in descriptor mode); ok preset to 1
#ifndef FWS_UTF8_WPE
#define FWS_UTF8_WPE 1
#endif
// kForm 0: lookup, then the unit's loads; 1: software-pipelined over a wave's
// units; 2: the unit's loads before its lookup (kEarly: one unit per wave on
// C5, so the owner lookup's scalar rounds overlap the HBM latency, as
// k_unmask_stream's kPf does for the stream form; the default: 1.439-1.447
// against 1.447-1.457 ms on C5, 86 VGPRs, 5 waves per SIMD). Measured slower
// and removed: 2 with write-through stores (1.53 ms) and 2 held to 6 waves per
// SIMD (1.466 ms, 80 VGPRs and scratch), profiles/r06/ab_c5d_early.jsonl.
template <bool kNT, int kForm>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(FWS_UTF8_WPE))) void k_unmask_sorted_utf8(uint8_t *base, const fws_frame_desc *__restrict__ d,
                                                               uint32_t n, uint8_t *__restrict__ ok,
                                                               uint32_t *__restrict__ seam, uint64_t seam_units) {
    if (kForm == 1) unmask_sorted_utf8_pipe<kNT>(base, d, n, ok, seam, seam_units);
    else unmask_sorted_body<kNT, kForm == 2, true>(base, d, n, ok, seam, seam_units);
}

// ------------------------------------------------------------ one launch, any order
// fws_gpu_unmask_batch without its plan launch: descriptor-major. One wavefront
// per region (grid-stride); the region's aligned 16-B chunks inside it are
// XORed whole (loads of 4 steps of 64 lanes issued before their stores), the
// partial chunks at its ends byte by byte (a chunk shared with a neighbouring
// region or piece is written only at this region's bytes, so regions in any
// order never race). A region longer than kAnyPiece is cut: the wave unmasks
// the first piece and queues the others (region index | piece << 32) for
// k_unmask_pieces, which the host launches after it; the queue count runs on
// two words by call parity (this call's, zeroed by the previous call's
// k_unmask_any; the next call's, zeroed here). When the queue is full the wave
// does the pieces itself.
constexpr uint64_t kAnyPiece = 64u * 1024u;
constexpr uint64_t kAnyEmpty = ~0ull;                // a queue slot no piece took

// Bytes [lo, hi) of region (po, key, phase), lo < hi, hi - lo <= kAnyPiece:
// every 16-B chunk meeting them is loaded in one batch (a partial chunk's other
// bytes are only read), XORed with the key at its phase, and stored whole or,
// for a partial chunk, byte by byte at this range's bytes only.
template <bool kNT>
__device__ __forceinline__ void unmask_range(uintptr_t po, uint32_t key, uint32_t phase, uintptr_t lo, uintptr_t hi,
                                             int lane) {
    // 5 steps of 64 chunks per round: a 4 KiB region off the 16-B grid (257
    // chunks, the C2 shape) takes one round, so no load waits for a store
    constexpr int kSteps = 5;
    const uintptr_t c0 = lo & ~uintptr_t(15);
    for (uintptr_t cs = c0; cs < hi; cs += (uintptr_t)kSteps * 1024u) {
        u32x4 v[kSteps];
#pragma unroll
        for (int j = 0; j < kSteps; ++j) {
            const uintptr_t c = cs + (uintptr_t)j * 1024u + (uintptr_t)lane * 16u;
            if (c < hi) v[j] = gload16<kNT>(c);
        }
        // the whole chunks first, with no variable-count branch between their
        // stores (the compiler then waits for no store before the next one)
        uint32_t part = 0;
#pragma unroll
        for (int j = 0; j < kSteps; ++j) {
            const uintptr_t c = cs + (uintptr_t)j * 1024u + (uintptr_t)lane * 16u;
            const uint32_t rk = rotr32(key, 8u * ((uint32_t)(c - po + phase) & 3u));
            v[j] = v[j] ^ u32x4{rk, rk, rk, rk};
            if (c >= lo && c + 16u <= hi) ustore16<kNT>(c, v[j]);
            else if (c < hi) part |= 1u << j;
        }
        // the range's partial chunks (at most its first and last), byte stores
        if (__builtin_expect(part != 0, 0)) {
#pragma unroll
            for (int j = 0; j < kSteps; ++j) {
                if (!((part >> j) & 1u)) continue;
                const uintptr_t c = cs + (uintptr_t)j * 1024u + (uintptr_t)lane * 16u;
                const uint32_t w[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
                for (int t = 0; t < 16; ++t)
                    if (c + (uintptr_t)t >= lo && c + (uintptr_t)t < hi)
                        *(uint8_t *)(c + (uintptr_t)t) = (uint8_t)(w[t >> 2] >> (8 * (t & 3)));
            }
        }
    }
}

template <bool kNT>
__global__ __launch_bounds__(kBlock) void k_unmask_any(uint8_t *base, const fws_frame_desc *__restrict__ d, uint32_t n,
                                                       uint64_t *__restrict__ queue, uint32_t qcap,
                                                       uint32_t *__restrict__ qcnt, uint32_t *__restrict__ qnext) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *qnext = 0u;   // the next call's count (its pieces kernel is done)
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t nw = gridDim.x * (kBlock / kWave);
    const uintptr_t b0 = (uintptr_t)base;
    for (uint32_t i = blockIdx.x * (kBlock / kWave) + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave); i < n; i += nw) {
        const fws_frame_desc fd = d[i];
        if (fd.payload_len == 0) continue;
        const uintptr_t po = b0 + fd.payload_off, pe = po + fd.payload_len;
        const uint32_t ph = fd.phase & 3u;
        if (fd.payload_len <= kAnyPiece) {
            unmask_range<kNT>(po, fd.key, ph, po, pe, lane);
            continue;
        }
        const uint64_t np = (fd.payload_len + kAnyPiece - 1u) / kAnyPiece;   // pieces 1 .. np - 1 queued
        uint32_t at = 0;
        if (lane == 0) at = atomicAdd(qcnt, (uint32_t)(np - 1u));
        at = __shfl(at, 0, 64);
        const bool queued = (uint64_t)at + (np - 1u) <= qcap;
        // (a refused reservation blanks the slots of it that lie below qcap: the
        // pieces kernel reads up to qcap entries of a count that includes them)
        for (uint64_t k = 1u + (uint64_t)lane; k < np; k += kWave)
            if ((uint64_t)at + k - 1u < qcap) queue[at + k - 1u] = queued ? (uint64_t)i | (k << 32) : kAnyEmpty;
        const uint64_t kend = queued ? 1u : np;       // queue full: every piece here
        for (uint64_t k = 0; k < kend; ++k) {
            const uintptr_t lo = po + k * kAnyPiece, hi = lo + kAnyPiece < pe ? lo + kAnyPiece : pe;
            unmask_range<kNT>(po, fd.key, ph, lo, hi, lane);
        }
    }
}

// The queued pieces of this call (count: *qcnt, at most qcap of them listed).
template <bool kNT>
__global__ __launch_bounds__(kBlock) void k_unmask_pieces(uint8_t *base, const fws_frame_desc *__restrict__ d,
                                                          const uint64_t *__restrict__ queue, uint32_t qcap,
                                                          const uint32_t *__restrict__ qcnt) {
    uint32_t cnt = *qcnt;
    if (cnt > qcap) cnt = qcap;                      // (an overflowing wave did its own pieces)
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t nw = gridDim.x * (kBlock / kWave);
    const uintptr_t b0 = (uintptr_t)base;
    for (uint32_t e = blockIdx.x * (kBlock / kWave) + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave); e < cnt; e += nw) {
        const uint64_t q = queue[e];
        if (q == kAnyEmpty) continue;
        const fws_frame_desc fd = d[(uint32_t)q];
        const uint64_t k = q >> 32;
        const uintptr_t po = b0 + fd.payload_off, pe = po + fd.payload_len;
        const uintptr_t lo = po + k * kAnyPiece, hi = lo + kAnyPiece < pe ? lo + kAnyPiece : pe;
        unmask_range<kNT>(po, fd.key, fd.phase & 3u, lo, hi, lane);
    }
}

}  // namespace fwsk

// ---------------------------------------------------------------- launchers
using namespace fwsk;

// Workgroups of the streaming kernels: a grid-stride loop over 4 KiB units per
// wavefront, capped per kernel family (measured on MI355X, tools/tune_c5.py):
// the sorted unmask runs one unit per wavefront (1.39 vs 1.54 ms on C5's 4 GiB
// at 16384 workgroups: its owner lookup and loads are not pipelined across a
// wave's units), and so does the UTF-8 form since its per-prefix lookup check
// (r05, tools/ab_c5d.py: 1.436 ms at 1<<20 vs 1.568 / 1.493 / 1.437 at 65536 /
// 131072 / 262144 workgroups); the stream unmask too since its UTF-8 form's
// cross-unit prefetch (r05, tools/ab_c5s.py on the 4 GiB C5 stream decode:
// 2.807-2.837 ms at 1<<20 against 2.860-2.889 at 131072 and 2.91 / 3.01 at
// 65536 / 32768; C2 / C3 batches have <= 65536 units, one per wavefront either way).
constexpr int kCapStream = 16384, kCapSorted = 1 << 20, kCapSortedUtf8 = 1 << 20, kCapStreamUnmask = 1 << 20;
static int g_grid_cap = 0;  // tuning hook: max workgroups of every streaming kernel (0: the defaults above)
extern "C" __attribute__((visibility("default"))) int fws_internal_set_grid_cap(int blocks) {
    const int old = g_grid_cap;
    if (blocks >= 0) g_grid_cap = blocks;
    return old;
}

// tuning hook: 0 = k_unmask_sorted, 1 = k_unmask_sorted_early, 3 = k_unmask_sorted
// with XCD runs (xcd_run_block). (2 was r06's loads-first k_unmask_sorted_ld with
// the slow units deferred past the unit loop: 83.27 against 83.02 us, removed;
// DESIGN.md §4.1b, profiles/r06/ab_sorted_ld.jsonl.)
static int g_sorted_early = 0;
extern "C" __attribute__((visibility("default"))) int fws_internal_set_sorted_early(int on) {
    const int old = g_sorted_early;
    g_sorted_early = on == 1 || on == 3 ? on : 0;
    return old;
}

// tuning hook: k_unmask_sorted_utf8 form -- 0 lookup first (r02-r06 default),
// 1 software-pipelined (measured slower, 2.12 vs 1.89 ms on C5: 90 VGPRs),
// 2 loads before the lookup (default)
static int g_sorted_utf8_pipe = 2;
extern "C" __attribute__((visibility("default"))) int fws_internal_set_sorted_utf8_pipe(int on) {
    const int old = g_sorted_utf8_pipe;
    g_sorted_utf8_pipe = on >= 0 && on <= 2 ? on : 2;
    return old;
}

// tuning hook: k_unmask_stream variant -- 0 forward nontemporal, 1 reverse
// nontemporal, 2 forward default policy, 3 reverse default policy
static int g_stream_variant = 0;
static int g_stream_utf8_pf = 1;   // tuning hook: k_unmask_stream<utf8> with the cross-unit prefetch (kPf)
extern "C" __attribute__((visibility("default"))) int fws_internal_set_stream_utf8_pf(int on) {
    const int old = g_stream_utf8_pf;
    g_stream_utf8_pf = on != 0;
    return old;
}
extern "C" __attribute__((visibility("default"))) int fws_internal_set_stream_variant(int v) {
    const int old = g_stream_variant;
    if (v >= 0 && v <= 3) g_stream_variant = v;
    return old;
}

static int grid_for_units(uint64_t units, int cap = kCapStream) {
    // memory-bound: one wavefront per unit up to the cap, grid-stride past it
    if (g_grid_cap > 0) cap = g_grid_cap;
    uint64_t blocks = (units + (kBlock / kWave) - 1) / (kBlock / kWave);
    if (blocks > (uint64_t)cap) blocks = (uint64_t)cap;
    if (blocks < 1) blocks = 1;
    return (int)blocks;
}

int fws_launch_mask_single(void *dev_ptr, uint64_t n, uint32_t key, uint32_t phase, hipStream_t s) {
    if (n == 0) return 0;
    fws_frame_desc one{0, n, key, phase};
    const uint64_t chunks = ((((uintptr_t)dev_ptr) + n + 15u) >> 4) - (((uintptr_t)dev_ptr) >> 4);
    const uint64_t units = (chunks + kUnitChunks - 1) / kUnitChunks;
    hipLaunchKernelGGL(k_mask_single, dim3(grid_for_units(units)), dim3(kBlock), 0, s, (uint8_t *)dev_ptr, one);
    return fws_hip_status(hipGetLastError());
}

int fws_launch_plan(const uint8_t *base, const fws_frame_desc *d, uint32_t n, const uint32_t *n_dev,
                    fws_plan_ws &ws, hipStream_t s) {
    const uint32_t nb = (n + kPlanTile - 1) / kPlanTile;
    if (nb == 0) return 0;
    if (nb > ws.status_cap) return FWS_ERR_CAPACITY;
    int r = fws_plan_next_epoch(ws, s);
    if (r) return r;
    PlanArgs a{ws.cbase, ws.unit_first, (u32x4 *)ws.unit_rec, ws.total, ws.status, ws.ticket,
               (fws_plan_mode *)ws.mode, ws.unit_cap, ws.epoch};
    hipLaunchKernelGGL(k_plan, dim3(nb), dim3(kBlock), 0, s, base, d, n, n_dev, a);
    return fws_hip_status(hipGetLastError());
}

namespace fwsk {
// fws_gpu_check_sorted: the first i whose region does not end at or before
// region i + 1's start (or whose end overflows), by an atomic minimum; the
// word is preset to ~0 (no violation) by the caller's memset
__global__ __launch_bounds__(kBlock) void k_check_sorted(const fws_frame_desc *__restrict__ d, uint32_t n,
                                                         uint32_t *__restrict__ bad) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    bool v = false;
    if (i < n) {
        const uint64_t e = d[i].payload_off + d[i].payload_len;
        v = e < d[i].payload_off || (i + 1 < n && e > d[i + 1].payload_off);
    }
    const uint64_t m = __ballot(v);
    if (m && (threadIdx.x & 63) == (uint32_t)__ffsll((unsigned long long)m) - 1u) atomicMin(bad, i);
}
}  // namespace fwsk

int fws_launch_check_sorted(const fws_frame_desc *d, uint32_t n, uint32_t *bad, hipStream_t s) {
    hipError_t e = hipMemsetAsync(bad, 0xFF, sizeof(uint32_t), s);
    if (e != hipSuccess) return fws_hip_status(e);
    if (n) hipLaunchKernelGGL(fwsk::k_check_sorted, dim3((n + fwsk::kBlock - 1) / fwsk::kBlock), dim3(fwsk::kBlock), 0,
                              s, d, n, bad);
    return fws_hip_status(hipGetLastError());
}

int fws_launch_unmask_sorted(uint8_t *base, const fws_frame_desc *d, uint32_t n, uint64_t max_span,
                             hipStream_t s) {
    if (n == 0) return 0;
    const uint64_t units = max_span / 4096u + 2u;
    if (g_sorted_early == 3)
        hipLaunchKernelGGL((k_unmask_sorted<true, true>), dim3(grid_for_units(units, kCapSorted)), dim3(kBlock), 0, s, base, d, n);
    else if (g_sorted_early)
        hipLaunchKernelGGL(k_unmask_sorted_early<true>, dim3(grid_for_units(units, kCapSorted)), dim3(kBlock), 0, s, base, d, n);
    else
        hipLaunchKernelGGL(k_unmask_sorted<true>, dim3(grid_for_units(units, kCapSorted)), dim3(kBlock), 0, s, base, d, n);
    return fws_hip_status(hipGetLastError());
}

int fws_launch_unmask_sorted_utf8(uint8_t *base, const fws_frame_desc *d, uint32_t n, uint64_t max_span,
                                  uint8_t *ok, uint32_t *seam, uint64_t seam_words, hipStream_t s) {
    const uint64_t seam_units = seam ? seam_words / 2u : 0u;
    if (n == 0) return 0;
    int r = fws_hip_status(hipMemsetAsync(ok, 1, n, s));
    if (r) return r;
    const uint64_t units = max_span / 4096u + 2u;
    const dim3 grid(grid_for_units(units, kCapSortedUtf8));
    if (g_sorted_utf8_pipe == 1)
        hipLaunchKernelGGL((k_unmask_sorted_utf8<true, 1>), grid, dim3(kBlock), 0, s, base, d, n, ok, seam, seam_units);
    else if (g_sorted_utf8_pipe == 2)
        hipLaunchKernelGGL((k_unmask_sorted_utf8<true, 2>), grid, dim3(kBlock), 0, s, base, d, n, ok, seam, seam_units);

    else
        hipLaunchKernelGGL((k_unmask_sorted_utf8<true, 0>), grid, dim3(kBlock), 0, s, base, d, n, ok, seam, seam_units);
    const uint64_t seam_blocks = (units + kBlock - 1) / kBlock;   // grid-stride: any span is covered
    hipLaunchKernelGGL(k_utf8_seam_sorted, dim3((unsigned)(seam_blocks < 4096u ? seam_blocks : 4096u)), dim3(kBlock), 0, s,
                       (const uint8_t *)base, d, n, ok, seam, seam_units);
    return fws_hip_status(hipGetLastError());
}

int fws_launch_unmask_stream(uint8_t *base, uint64_t N, const fws_frame_info *frames, uint32_t cap,
                             const uint32_t *n_dev, const uint32_t *unit_first, uint8_t *utf8_ok,
                             uint32_t *seam, hipStream_t s) {
    const uint64_t units = (N + 4095) / 4096;
    if (units == 0 || cap == 0) return 0;
    const dim3 grid(grid_for_units(units, kCapStreamUnmask)), blk(kBlock);
    const int v = g_stream_variant;
    if (utf8_ok == nullptr) {
        if (v == 0)
            hipLaunchKernelGGL((k_unmask_stream<true, false, false>), grid, blk, 0, s, (uint8_t *)base, N, frames, cap,
                               n_dev, unit_first, units, nullptr, nullptr);
        else if (v == 1)
            hipLaunchKernelGGL((k_unmask_stream<true, false, true>), grid, blk, 0, s, (uint8_t *)base, N, frames, cap,
                               n_dev, unit_first, units, nullptr, nullptr);
        else if (v == 2)
            hipLaunchKernelGGL((k_unmask_stream<false, false, false>), grid, blk, 0, s, (uint8_t *)base, N, frames,
                               cap, n_dev, unit_first, units, nullptr, nullptr);
        else
            hipLaunchKernelGGL((k_unmask_stream<false, false, true>), grid, blk, 0, s, (uint8_t *)base, N, frames,
                               cap, n_dev, unit_first, units, nullptr, nullptr);
    } else {
        if (g_stream_utf8_pf && (v == 1 || v == 3))
            hipLaunchKernelGGL((k_unmask_stream<true, true, true, true>), grid, blk, 0, s, (uint8_t *)base, N, frames,
                               cap, n_dev, unit_first, units, utf8_ok, seam);
        else if (g_stream_utf8_pf)
            hipLaunchKernelGGL((k_unmask_stream<true, true, false, true>), grid, blk, 0, s, (uint8_t *)base, N, frames,
                               cap, n_dev, unit_first, units, utf8_ok, seam);
        else if (v == 1 || v == 3)
            hipLaunchKernelGGL((k_unmask_stream<true, true, true>), grid, blk, 0, s, (uint8_t *)base, N, frames, cap,
                               n_dev, unit_first, units, utf8_ok, seam);
        else
            hipLaunchKernelGGL((k_unmask_stream<true, true, false>), grid, blk, 0, s, (uint8_t *)base, N, frames, cap,
                               n_dev, unit_first, units, utf8_ok, seam);
        hipLaunchKernelGGL(k_utf8_seam, dim3((unsigned)((units + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                           (const uint8_t *)base, N, frames, cap, n_dev, unit_first, units, utf8_ok, seam);
    }
    return fws_hip_status(hipGetLastError());
}

int fws_launch_unmask(uint8_t *base, const fws_frame_desc *d, uint32_t n, const uint32_t *n_dev,
                      const fws_plan_ws &ws, uint64_t max_chunks, hipStream_t s) {
    const uint64_t units = (max_chunks + kUnitChunks - 1) / kUnitChunks;
    hipLaunchKernelGGL(k_unmask_desc<true>, dim3(grid_for_units(units)), dim3(kBlock), 0, s, base, d, n, ws.cbase,
                       ws.unit_first, (const u32x4 *)ws.unit_rec, ws.total, (const fws_plan_mode *)ws.mode, ws.unit_cap);
    return fws_hip_status(hipGetLastError());
}

// tuning hook: fws_gpu_unmask_batch as k_unmask_any + k_unmask_pieces (1) or
// k_plan + k_unmask_desc (0, the default: sorted C2 0.0906 ms against 0.1058,
// permuted C2 0.142 against 0.123 -- DESIGN.md §4.3b)
static int g_unmask_any = 0;
extern "C" __attribute__((visibility("default"))) int fws_internal_set_unmask_any(int on) {
    const int old = g_unmask_any;
    g_unmask_any = on != 0;
    return old;
}
bool fws_unmask_any_on() { return g_unmask_any != 0; }

int fws_launch_unmask_any(uint8_t *base, const fws_frame_desc *d, uint32_t n, uint64_t *queue, uint32_t qcap,
                          uint32_t *qcnt, uint32_t *qnext, uint32_t piece_grid, hipStream_t s) {
    if (n == 0) return 0;
    uint64_t blocks = (n + (kBlock / kWave) - 1) / (kBlock / kWave);
    if (blocks > (1u << 20)) blocks = 1u << 20;      // grid-stride past it
    hipLaunchKernelGGL(k_unmask_any<true>, dim3((unsigned)blocks), dim3(kBlock), 0, s, base, d, n, queue, qcap, qcnt,
                       qnext);
    hipLaunchKernelGGL(k_unmask_pieces<true>, dim3(piece_grid ? piece_grid : 1u), dim3(kBlock), 0, s, base, d, queue,
                       qcap, qcnt);
    return fws_hip_status(hipGetLastError());
}
