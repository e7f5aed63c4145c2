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

namespace fwsk {

// ---------------------------------------------------------------- plan
constexpr int kPlanItems = 4;                        // frames per thread
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

__global__ __launch_bounds__(kBlock) void k_plan_count(const uint8_t *base,
                                                       const fws_frame_desc *__restrict__ d,
                                                       uint32_t n, const uint32_t *__restrict__ n_dev,
                                                       uint64_t *__restrict__ block_sums) {
    if (n_dev && *n_dev < n) n = *n_dev;
    const uint64_t f0 = uint64_t(blockIdx.x) * kPlanTile + uint64_t(threadIdx.x) * kPlanItems;
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < kPlanItems; ++i)
        if (f0 + i < n) s += desc_chunks(base, d[f0 + i]);
    uint64_t tot;
    block_excl_scan(s, &tot);
    if (threadIdx.x == 0) block_sums[blockIdx.x] = tot;
}

// cbase[f] = chunks of frames [0, f); cbase[n] = total; unit_first[u] = frame
// holding chunk u * kUnitChunks; *total_out = total chunks.
__global__ __launch_bounds__(kBlock) void k_plan_scan(const uint8_t *base,
                                                      const fws_frame_desc *__restrict__ d, uint32_t n,
                                                      const uint32_t *__restrict__ n_dev,
                                                      const uint64_t *__restrict__ block_sums,
                                                      uint64_t *__restrict__ cbase,
                                                      uint32_t *__restrict__ unit_first,
                                                      uint64_t *__restrict__ total_out,
                                                      uint64_t unit_cap) {
    if (n_dev && *n_dev < n) n = *n_dev;
    __shared__ uint64_t s_prefix;
    // prefix of earlier blocks (n_blocks is small: n / 1024)
    uint64_t p = 0;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += kBlock) p += block_sums[b];
    uint64_t dummy;
    uint64_t pe = block_excl_scan(p, &dummy);
    if (threadIdx.x == kBlock - 1) s_prefix = pe + p;
    __syncthreads();
    const uint64_t prefix = s_prefix;

    const uint64_t f0 = uint64_t(blockIdx.x) * kPlanTile + uint64_t(threadIdx.x) * kPlanItems;
    uint64_t c[kPlanItems];
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < kPlanItems; ++i) {
        c[i] = (f0 + i < n) ? desc_chunks(base, d[f0 + i]) : 0;
        s += c[i];
    }
    uint64_t tot;
    uint64_t run = prefix + block_excl_scan(s, &tot);
#pragma unroll
    for (int i = 0; i < kPlanItems; ++i) {
        const uint64_t f = f0 + i;
        if (f < n) {
            cbase[f] = run;
            if (c[i]) {
                uint64_t u = (run + kUnitChunks - 1) / kUnitChunks;
                uint64_t ue = (run + c[i] + kUnitChunks - 1) / kUnitChunks;
                if (ue > unit_cap) ue = unit_cap;   // contract violation guard, never OOB
                for (; u < ue; ++u) unit_first[u] = (uint32_t)f;
            }
            run += c[i];
            if (f == n - 1) {   // the thread holding the last frame has the grand total
                cbase[n] = run;
                *total_out = run;
            }
        }
    }
    if (n == 0 && blockIdx.x == 0 && threadIdx.x == 0) {
        cbase[0] = 0;
        *total_out = 0;
    }
}

// ---------------------------------------------------------------- unmask
// One wave = one unit of kUnitChunks chunks. Loads for all U chunks of a lane
// are issued before any XOR/store so each lane keeps 64 B in flight.
template <bool kSingle>
__global__ __launch_bounds__(kBlock) void k_unmask(uint8_t *base, const fws_frame_desc *__restrict__ d,
                                                   uint32_t n, const uint32_t *__restrict__ n_dev,
                                                   const uint64_t *__restrict__ cbase,
                                                   const uint32_t *__restrict__ unit_first,
                                                   const uint64_t *__restrict__ total_ptr,
                                                   uint64_t unit_cap, fws_frame_desc single) {
    if (!kSingle && n_dev && *n_dev < n) n = *n_dev;
    if (n == 0) return;
    const uint64_t total = kSingle ? chunks_of((uintptr_t)(base + single.payload_off), single.payload_len)
                                   : *total_ptr;
    uint64_t n_units = (total + kUnitChunks - 1) / kUnitChunks;
    if (!kSingle && n_units > unit_cap) n_units = unit_cap;
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = uint64_t(gridDim.x) * (kBlock / kWave);
    for (uint64_t u = uint64_t(blockIdx.x) * (kBlock / kWave) + threadIdx.x / kWave; u < n_units;
         u += nwaves) {
        uint32_t flo = 0, fhi = 0;
        if (!kSingle) {
            flo = unit_first[u];
            fhi = (u + 1 < n_units) ? unit_first[u + 1] : n - 1;
        }
        const uintptr_t safe =
            (uintptr_t)(base + (kSingle ? single.payload_off : d[flo].payload_off)) & ~uintptr_t(15);
        uintptr_t ca[kUnmaskU], lo[kUnmaskU], hi[kUnmaskU];
        uint32_t rk[kUnmaskU];
        bool live[kUnmaskU];
#pragma unroll
        for (int j = 0; j < kUnmaskU; ++j) {
            const uint64_t g = u * kUnitChunks + uint64_t(j) * kWave + lane;
            live[j] = g < total;
            fws_frame_desc fd = single;
            uint64_t cb = 0;
            if (!kSingle) {
                const uint32_t f = find_frame(cbase, flo, fhi, live[j] ? g : cbase[flo]);
                fd = d[f];
                cb = cbase[f];
            }
            const uintptr_t a0 = (uintptr_t)(base + fd.payload_off);
            lo[j] = a0;
            hi[j] = a0 + fd.payload_len;
            ca[j] = (a0 & ~uintptr_t(15)) + (uintptr_t)((g - cb) << 4);
            rk[j] = aligned_key(fd.key, fd.phase, a0);
        }
        u32x4 v[kUnmaskU];
        bool full[kUnmaskU];
#pragma unroll
        for (int j = 0; j < kUnmaskU; ++j) {
            full[j] = live[j] && ca[j] >= lo[j] && ca[j] + 16u <= hi[j];
            // unconditional load so every lane's loads issue back to back before
            // any wait; non-full lanes read the chunk holding the first byte of
            // the unit's first frame (non-empty, inside the caller's buffer)
            v[j] = gload16(full[j] ? ca[j] : safe);
        }
#pragma unroll
        for (int j = 0; j < kUnmaskU; ++j) {
            if (full[j]) {
                gstore16(ca[j], v[j] ^ rk[j]);
            } else if (live[j]) {
                xor_partial_chunk(ca[j], lo[j], hi[j], rk[j]);
            }
        }
    }
}

// Fast variant. A wave owns G consecutive plan units (G x 4 KiB). When those
// units touch at most 4 frames (every frame >= ~4 KiB, e.g. BASELINE C2) the
// frame metadata is wave-uniform: it is fetched with scalar loads (lgkmcnt, so
// it never queues behind the payload loads on vmcnt), the lane's frame is
// picked by three compares, and all G*4 16-B loads of a lane are in flight
// before the first XOR. Units with more frames take the per-lane search path.
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

// Scalar (wave-uniform) metadata of one plan unit: its first frame and
// whether the unit touches at most 2 frames.
struct UnitMeta {
    uint32_t flo, fhi;
};

__device__ __forceinline__ UnitMeta unit_meta(const uint32_t *__restrict__ unit_first, uint64_t u, uint64_t n_units,
                                              uint32_t n) {
    UnitMeta m{0u, 0u};
    if (u < n_units) {
        m.flo = unit_first[u];
        m.fhi = (u + 1 < n_units) ? unit_first[u + 1] : n - 1;
    }
    return m;
}

// Fast variant, one 4 KiB plan unit per wave step. When the unit touches at
// most 2 frames (every frame >= 4 KiB, e.g. BASELINE C2) the frame metadata is
// wave-uniform: fetched with scalar loads (lgkmcnt, never queued behind the
// payload loads on vmcnt), the lane's frame is one 64-bit compare, all 4
// loads of a lane issue back to back, region heads/tails are stored byte-exact
// from the same loaded chunk, and the next unit's metadata is fetched while
// this unit's payload is in flight. Units with more frames take the per-lane
// search path.
template <bool kNT>
__global__ __launch_bounds__(kBlock) void k_unmask_fast(uint8_t *base, const fws_frame_desc *__restrict__ d,
                                                        uint32_t n, const uint32_t *__restrict__ n_dev,
                                                        const uint64_t *__restrict__ cbase,
                                                        const uint32_t *__restrict__ unit_first,
                                                        const uint64_t *__restrict__ total_ptr, uint64_t unit_cap) {
    constexpr int J = kUnmaskU;
    if (n_dev && *n_dev < n) n = *n_dev;
    if (n == 0) return;
    const uint64_t total = *total_ptr;
    uint64_t n_units = (total + kUnitChunks - 1) / kUnitChunks;
    if (n_units > unit_cap) n_units = unit_cap;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t nwaves = uint64_t(gridDim.x) * (kBlock / kWave);
    uint64_t u = uint64_t(blockIdx.x) * (kBlock / kWave) + wave;
    UnitMeta m = unit_meta(unit_first, u, n_units, n);
    for (; u < n_units; u += nwaves) {
        const uint32_t flo = m.flo, fhi = m.fhi;
        const uint64_t g0 = u * kUnitChunks + lane;
        if (fhi - flo >= 2u) {                          // many small frames: generic path
            m = unit_meta(unit_first, u + nwaves, n_units, n);
#pragma unroll 1
            for (int j = 0; j < J; ++j) {
                const uint64_t g = g0 + uint64_t(j) * kWave;
                if (g < total) unmask_one_chunk(base, d, cbase, flo, fhi, g);
            }
            continue;
        }
        uint64_t A[2], L[2], H[2];
        uint32_t R[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t f = (flo + (uint32_t)k <= fhi) ? flo + (uint32_t)k : fhi;
            const fws_frame_desc fd = d[f];
            const uint64_t c = cbase[f];
            const uintptr_t a0 = (uintptr_t)(base + fd.payload_off);
            A[k] = (uint64_t)(a0 & ~uintptr_t(15)) - (c << 4);          // chunk g lives at A + 16 g
            L[k] = a0;
            H[k] = a0 + fd.payload_len;
            R[k] = aligned_key(fd.key, fd.phase, a0);
        }
        const uint64_t CB1 = (fhi > flo) ? cbase[flo + 1] : ~0ull;
        uintptr_t ca[J];
        uint32_t rk[J];
        bool live[J], s1[J];
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const uint64_t g = g0 + uint64_t(j) * kWave;
            s1[j] = g >= CB1;
            rk[j] = s1[j] ? R[1] : R[0];
            ca[j] = (uintptr_t)((s1[j] ? A[1] : A[0]) + (g << 4));
            live[j] = g < total;
        }
        const uintptr_t safe = (uintptr_t)L[0] & ~uintptr_t(15);   // holds a byte of frame flo
        u32x4 v[J];
#pragma unroll
        for (int j = 0; j < J; ++j) v[j] = gload16<kNT>(live[j] ? ca[j] : safe);
        m = unit_meta(unit_first, u + nwaves, n_units, n);        // next unit, overlapped
#pragma unroll
        for (int j = 0; j < J; ++j) {
            if (!live[j]) continue;
            const uintptr_t lo = s1[j] ? L[1] : L[0], hi = s1[j] ? H[1] : H[0];
            if (ca[j] >= lo && ca[j] + 16u <= hi) gstore16<kNT>(ca[j], v[j] ^ rk[j]);
            else store_partial(ca[j], v[j], rk[j], lo, hi);
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
    if (skip) e0 &= 0x80000000u;                     // bytes 0..2 are judged by k_utf8_seam
    return (e0 | utf8_err(x.y, x.x) | utf8_err(x.z, x.y) | utf8_err(x.w, x.z)) != 0u;
}

template <bool kNT, bool kUtf8>
__global__ __launch_bounds__(kBlock) void k_unmask_stream(uint8_t *base, uint64_t N,
                                                          const fws_frame_info *__restrict__ fr, uint32_t cap,
                                                          const uint32_t *__restrict__ n_dev,
                                                          const uint32_t *__restrict__ unit_first, uint64_t n_units,
                                                          uint8_t *__restrict__ ok) {
    uint32_t n = *n_dev;
    if (n > cap) n = cap;
    if (n == 0) return;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t nwaves = uint64_t(gridDim.x) * (kBlock / kWave);
    const uintptr_t b0 = (uintptr_t)base;
    for (uint64_t u = uint64_t(blockIdx.x) * (kBlock / kWave) + wave; u < n_units; u += nwaves) {
        const uint32_t flo = unit_first[u];
        const uint32_t fhi = (u + 1 < n_units) ? unit_first[u + 1] : n - 1;
        const uint64_t c0 = u * 4096u + uint64_t(lane) * 16u;
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
                if (touched) gstore16<kNT>(b0 + c, v ^ m);
                if constexpr (kUtf8) {
                    const u32x4 x = v ^ m;
                    uint32_t prev = __shfl_up(x.w, 1, 64);
                    if (lane == 0) prev = carry;
                    carry = __shfl(x.w, 63, 64);
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
        const StreamFrame A = stream_frame(fr[flo], N), B = stream_frame(fr[fhi], N);
        const bool two = fhi != flo;
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
        for (int j = 0; j < kUnmaskU; ++j) v[j] = gload16<kNT>(live[j] ? ca[j] : safe);
#pragma unroll
        for (int j = 0; j < kUnmaskU; ++j)
            if (live[j]) gstore16<kNT>(ca[j], v[j] ^ mk[j]);
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
                                                      uint8_t *__restrict__ ok) {
    uint32_t n = *n_dev;
    if (n > cap) n = cap;
    const uint64_t u = uint64_t(blockIdx.x) * kBlock + threadIdx.x + 1u;
    if (n == 0 || u > n_units) return;
    const uint64_t P = u * 4096u;
    const uint32_t f = u < n_units ? unit_first[u] : n - 1;
    const uint32_t cur = P < N ? *(const uint32_t *)(base + P) : 0u;      // bytes past N: zeroed below
    const uint32_t prev = *(const uint32_t *)(base + P - 4u);
    for (uint32_t g = f > 0 ? f - 1u : 0u; g <= f; ++g) {
        const StreamFrame sf = stream_frame(fr[g], N);
        if (!sf.text || P + 3u <= sf.po || P >= sf.pe + 3u) continue;
        const uint32_t x = cur & sel_bytes(P, sf.po, sf.pe), p = prev & sel_bytes(P - 4u, sf.po, sf.pe);
        if (utf8_err(x, p) & 0x00808080u) ok[g] = 0;
    }
}

}  // namespace fwsk

// ---------------------------------------------------------------- launchers
using namespace fwsk;

// Kernel variant used by fws_launch_unmask (tuning hook, not part of the ABI):
// 0 = k_unmask (per-lane search), 1 = k_unmask_fast, 5 = k_unmask_fast nontemporal.
static int g_unmask_variant = 5;
extern "C" __attribute__((visibility("default"))) int fws_internal_set_unmask_variant(int v) {
    const int old = g_unmask_variant;
    if (v >= 0 && v <= 7) g_unmask_variant = v;
    return old;
}

static int g_grid_cap = 16384;  // tuning hook: max workgroups of the streaming kernels
extern "C" __attribute__((visibility("default"))) int fws_internal_set_grid_cap(int blocks) {
    const int old = g_grid_cap;
    if (blocks > 0) g_grid_cap = blocks;
    return old;
}

static int grid_for_units(uint64_t units) {
    // memory-bound: cap near 256 CUs x 8 blocks and grid-stride the rest
    uint64_t blocks = (units + (kBlock / kWave) - 1) / (kBlock / kWave);
    if (blocks > (uint64_t)g_grid_cap) blocks = (uint64_t)g_grid_cap;
    if (blocks < 1) blocks = 1;
    return (int)blocks;
}

int fws_launch_mask_single(void *dev_ptr, uint64_t n, uint32_t key, uint32_t phase, hipStream_t s) {
    if (n == 0) return 0;
    fws_frame_desc one{0, n, key, phase};
    const uint64_t chunks = ((((uintptr_t)dev_ptr) + n + 15u) >> 4) - (((uintptr_t)dev_ptr) >> 4);
    const uint64_t units = (chunks + kUnitChunks - 1) / kUnitChunks;
    hipLaunchKernelGGL(k_unmask<true>, dim3(grid_for_units(units)), dim3(kBlock), 0, s,
                       (uint8_t *)dev_ptr, nullptr, 1u, nullptr, nullptr, nullptr, nullptr, 0ull, one);
    return fws_hip_status(hipGetLastError());
}

int fws_launch_plan(const uint8_t *base, const fws_frame_desc *d, uint32_t n, const uint32_t *n_dev,
                    fws_plan_ws &ws, hipStream_t s) {
    const uint32_t nb = (n + kPlanTile - 1) / kPlanTile;
    hipLaunchKernelGGL(k_plan_count, dim3(nb), dim3(kBlock), 0, s, base, d, n, n_dev, ws.block_sums);
    hipLaunchKernelGGL(k_plan_scan, dim3(nb), dim3(kBlock), 0, s, base, d, n, n_dev, ws.block_sums, ws.cbase,
                       ws.unit_first, ws.total, ws.unit_cap);
    return fws_hip_status(hipGetLastError());
}

int fws_launch_unmask_stream(uint8_t *base, uint64_t N, const fws_frame_info *frames, uint32_t cap,
                             const uint32_t *n_dev, const uint32_t *unit_first, uint8_t *utf8_ok, hipStream_t s) {
    const uint64_t units = (N + 4095) / 4096;
    if (units == 0 || cap == 0) return 0;
    if (utf8_ok == nullptr) {
        hipLaunchKernelGGL((k_unmask_stream<true, false>), dim3(grid_for_units(units)), dim3(kBlock), 0, s,
                           (uint8_t *)base, N, frames, cap, n_dev, unit_first, units, nullptr);
    } else {
        hipLaunchKernelGGL((k_unmask_stream<true, true>), dim3(grid_for_units(units)), dim3(kBlock), 0, s,
                           (uint8_t *)base, N, frames, cap, n_dev, unit_first, units, utf8_ok);
        hipLaunchKernelGGL(k_utf8_seam, dim3((unsigned)((units + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                           (const uint8_t *)base, N, frames, cap, n_dev, unit_first, units, utf8_ok);
    }
    return fws_hip_status(hipGetLastError());
}

int fws_launch_unmask(uint8_t *base, const fws_frame_desc *d, uint32_t n, const uint32_t *n_dev,
                      const fws_plan_ws &ws, uint64_t max_chunks, hipStream_t s) {
    const uint64_t units = (max_chunks + kUnitChunks - 1) / kUnitChunks;
    fws_frame_desc none{0, 0, 0, 0};
    const int v = g_unmask_variant;
    const dim3 grid(grid_for_units(units)), blk(kBlock);
    if (v == 0 || v == 4)
        hipLaunchKernelGGL(k_unmask<false>, grid, blk, 0, s, base, d, n, n_dev, ws.cbase, ws.unit_first, ws.total,
                           ws.unit_cap, none);
    else if (v < 4)
        hipLaunchKernelGGL(k_unmask_fast<false>, grid, blk, 0, s, base, d, n, n_dev, ws.cbase, ws.unit_first,
                           ws.total, ws.unit_cap);
    else
        hipLaunchKernelGGL(k_unmask_fast<true>, grid, blk, 0, s, base, d, n, n_dev, ws.cbase, ws.unit_first,
                           ws.total, ws.unit_cap);
    return fws_hip_status(hipGetLastError());
}
