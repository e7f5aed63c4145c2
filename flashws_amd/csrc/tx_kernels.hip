// tx_kernels.hip -- batch frame builder for the send path:
// the bytes WSocket::SendFrame (net/w_socket.h:832-944) writes for each frame,
// for a whole batch in one pass over the output.
//
// A frame is header + payload: b0 = FIN << 7 | opcode (:914), b1 = MASK << 7 |
// len7 with the 16- or 64-bit big-endian length after it (:867-881), then for
// a client frame the 4 key bytes (native LE u32, :862-866) and the payload
// XORed with them from phase 0 (WSMaskBytesFast, :861). The opcode / FIN
// sequencing of a connection (last_msg_not_fin_, :903-913) is host logic
// (fws_tx_next); the device builds bytes.
//
// Plan: k_out_plan (outplan_kernels.hip, one launch): obase = exclusive prefix
// of the frame sizes, total, unit_first[u] = the frame spanning output byte
// 4 KiB * u. k_tx_encode: one wave per 4 KiB output unit; each lane owns 16-B
// output chunks, so every chunk is one full 16-B store (the last chunk of the
// output stops at the total). A chunk inside one payload is two aligned source
// loads shifted by the payload's source misalignment, XORed with the key at the
// frame-relative phase -- the k_gather_fast data path; header bytes and chunks
// on a frame seam are built bytewise. HBM bytes = payload read + frames written.
#include "fws_device.h"
#include "fws_internal.h"
#include "outplan_common.h"    // out_size; plan_common.h: the look-back

namespace fwsk {

constexpr uint64_t kTxUnit = 4096;

__device__ __forceinline__ uint32_t tx_hdr_len(const fws_tx_desc &d) {   // w_socket.h:49-65
    const uint32_t ext = d.len < 126u ? 0u : (d.len <= 65535u ? 2u : 8u);
    return 2u + (d.masked ? 4u : 0u) + ext;
}

// Byte i (< tx_hdr_len) of the frame header.
__device__ __forceinline__ uint32_t tx_hdr_byte(const fws_tx_desc &d, uint32_t i) {
    const uint32_t m = d.masked ? 0x80u : 0u;
    const uint32_t ext = d.len < 126u ? 0u : (d.len <= 65535u ? 2u : 8u);
    if (i == 0) return ((uint32_t)(d.fin != 0) << 7) | (d.opcode & 15u);
    if (i == 1) return m | (ext == 0 ? (uint32_t)d.len : (ext == 2 ? 126u : 127u));
    if (i < 2u + ext) return (uint32_t)(d.len >> (8u * (ext - 1u - (i - 2u)))) & 0xFFu;   // big endian
    return (d.key >> (8u * (i - 2u - ext))) & 0xFFu;                                     // key bytes, LE
}

// 16 bytes starting sh (0..15) bytes into the 32-byte window v0:v1
__device__ __forceinline__ u32x4 tx_shr_bytes(const u32x4 &v0, const u32x4 &v1, uint32_t sh) {
    const bool s8 = (sh & 8u) != 0, s4 = (sh & 4u) != 0;
    const uint32_t a0 = s8 ? v0.z : v0.x, a1 = s8 ? v0.w : v0.y, a2 = s8 ? v1.x : v0.z;
    const uint32_t a3 = s8 ? v1.y : v0.w, a4 = s8 ? v1.z : v1.x;
    const uint32_t c0 = s4 ? a1 : a0, c1 = s4 ? a2 : a1, c2 = s4 ? a3 : a2, c3 = s4 ? a4 : a3;
    const uint32_t c4 = s4 ? (s8 ? v1.w : v1.y) : a4;
    const uint32_t b = sh & 3u;
    return u32x4{__builtin_amdgcn_alignbyte(c1, c0, b), __builtin_amdgcn_alignbyte(c2, c1, b),
                 __builtin_amdgcn_alignbyte(c3, c2, b), __builtin_amdgcn_alignbyte(c4, c3, b)};
}

// Output bytes [a, min(a + 16, total)) built one by one from frame f on
// (units meeting 3+ frames).
__device__ void tx_bytes(uint8_t *out, const uint8_t *src, const fws_tx_desc *__restrict__ d,
                         const uint64_t *__restrict__ obase, uint32_t f, uint64_t a, uint64_t total) {
    for (uint64_t b = a; b < a + 16 && b < total; ++b) {
        while (b >= obase[f + 1]) ++f;
        const fws_tx_desc fd = d[f];
        const uint32_t h = tx_hdr_len(fd);
        const uint64_t k = b - obase[f];
        uint32_t v;
        if (k < h) {
            v = tx_hdr_byte(fd, (uint32_t)k);
        } else {
            const uint64_t j = k - h;
            v = src[fd.src_off + j] ^ (fd.masked ? (fd.key >> (8u * (uint32_t)(j & 3u))) & 0xFFu : 0u);
        }
        out[b] = (uint8_t)v;
    }
}

// A 16-B output chunk at a that meets a frame seam, in a unit of at most two
// frames A (output [OA, EA)) and B (from OB = EA): header bytes come from the
// descriptors in registers, payload bytes from each frame's shifted, keyed
// 16-B source window (two aligned block loads each, issued with the unit's
// other loads), selected byte by byte.
struct TxSeam {
    uint64_t PA, EA, PB, EB;
};

// Source blocks of a seam chunk at a for frame X (payload [PX, EX) in the
// output, source bytes [s0, s0 + len)): the two aligned 16-B blocks of the
// window at SX + a; a block that holds no byte of the source range is replaced
// by `safe16` (its bytes are never selected), so every load is in bounds.
__device__ __forceinline__ void tx_seam_blocks(uint64_t a, uintptr_t SX, uintptr_t s0, uint64_t len, uintptr_t safe16,
                                               uintptr_t &b0, uintptr_t &b1, uint32_t &sh) {
    const uintptr_t sa = SX + (uintptr_t)a;
    sh = (uint32_t)(sa & 15u);
    b0 = sa & ~uintptr_t(15);
    b1 = b0 + 16u;
    if (len == 0 || b0 + 16u <= s0 || b0 >= s0 + len) b0 = safe16;
    if (len == 0 || b1 + 16u <= s0 || b1 >= s0 + len) b1 = safe16;
}

// The frame header as 16 bytes (<= 14 used, rest zero), little-endian dwords:
// b0, b1, the big-endian 16/64-bit length, then the key bytes (masked frames).
__device__ __forceinline__ u32x4 tx_hdr_vec(const fws_tx_desc &d) {
    const uint32_t b0 = ((uint32_t)(d.fin != 0) << 7) | (d.opcode & 15u);
    const uint32_t m = d.masked ? 0x80u : 0u;
    const uint32_t k = d.masked ? d.key : 0u;
    const uint64_t L = d.len;
    if (L < 126u) return u32x4{b0 | ((m | (uint32_t)L) << 8) | ((k & 0xFFFFu) << 16), k >> 16, 0u, 0u};
    if (L <= 65535u)
        return u32x4{b0 | ((m | 126u) << 8) | ((uint32_t)((L >> 8) & 0xFFu) << 16) | ((uint32_t)(L & 0xFFu) << 24), k,
                     0u, 0u};
    const uint32_t hi = __builtin_bswap32((uint32_t)(L >> 32)), lo = __builtin_bswap32((uint32_t)L);
    // bytes 2..9 = L big endian = bswap(hi32) bswap(lo32)
    return u32x4{b0 | ((m | 127u) << 8) | (hi << 16), (hi >> 16) | (lo << 16), (lo >> 16) | ((k & 0xFFFFu) << 16),
                 k >> 16};
}

// 16 bytes of v as seen from byte offset off (-16 < off < 16): byte i of the
// result is v's byte i + off, zero outside v.
__device__ __forceinline__ u32x4 tx_bytes_at(const u32x4 &v, int off) {
    const u32x4 z{0u, 0u, 0u, 0u};
    return off >= 0 ? tx_shr_bytes(v, z, (uint32_t)off) : tx_shr_bytes(z, v, (uint32_t)(16 + off));
}

// x clipped to [a, a + 16), as an offset from a.
__device__ __forceinline__ uint32_t tx_rel(uint64_t x, uint64_t a) {
    return x <= a ? 0u : (x >= a + 16u ? 16u : (uint32_t)(x - a));
}

// Byte-select mask of the chunk's bytes [lo, hi) (offsets 0..16) for dword i.
__device__ __forceinline__ uint32_t tx_sel(uint32_t lo, uint32_t hi, int i) {
    const uint32_t o = 4u * (uint32_t)i;
    if (hi <= o || lo >= o + 4u) return 0u;
    const uint32_t s = lo > o ? lo - o : 0u, e = hi < o + 4u ? o + 4u - hi : 0u;
    return (0xFFFFFFFFu << (8u * s)) & (0xFFFFFFFFu >> (8u * e));
}

// The seam chunk at a: A's header, A's payload (pA: keyed source window), B's
// header, B's payload (pB), each selected on its byte range; 32-bit offsets.
__device__ __forceinline__ u32x4 tx_seam_combine(uint64_t a, const fws_tx_desc &dA, uint64_t OA, const fws_tx_desc &dB,
                                                 uint64_t OB, bool two, const TxSeam &z, uint64_t total,
                                                 const u32x4 &pA, const u32x4 &pB) {
    const uint32_t t = tx_rel(total, a);
    const uint32_t oa = tx_rel(OA, a), pa = tx_rel(z.PA, a), ea = tx_rel(z.EA, a);
    const uint32_t pb = two ? tx_rel(z.PB, a) : ea, eb = two ? tx_rel(z.EB, a) : ea;
    const int hoA = (int)((int64_t)a - (int64_t)OA), hoB = (int)((int64_t)a - (int64_t)OB);
    const u32x4 HA = (hoA > -16 && hoA < 16) ? tx_bytes_at(tx_hdr_vec(dA), hoA) : u32x4{0u, 0u, 0u, 0u};
    const u32x4 HB = (two && hoB > -16 && hoB < 16) ? tx_bytes_at(tx_hdr_vec(dB), hoB) : u32x4{0u, 0u, 0u, 0u};
    const uint32_t ha[4] = {HA.x, HA.y, HA.z, HA.w}, hb[4] = {HB.x, HB.y, HB.z, HB.w};
    const uint32_t wa[4] = {pA.x, pA.y, pA.z, pA.w}, wb[4] = {pB.x, pB.y, pB.z, pB.w};
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t live = tx_sel(0u, t, i);
        w[i] = live & ((ha[i] & tx_sel(oa, pa, i)) | (wa[i] & tx_sel(pa, ea, i)) | (hb[i] & tx_sel(ea, pb, i)) |
                       (wb[i] & tx_sel(pb, eb, i)));
    }
    return u32x4{w[0], w[1], w[2], w[3]};
}

// The output bytes [a, min(a + 16, total)) of x (the output's last chunk).
__device__ __forceinline__ void tx_store_tail(uint8_t *out, uint64_t a, uint64_t total, const u32x4 &x) {
    const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
    for (uint64_t b = a; b < total && b < a + 16u; ++b) out[b] = (uint8_t)(xw[(b - a) >> 2] >> (8u * ((b - a) & 3u)));
}

// One 4 KiB output unit of a wave: lane chunks a0 + 1024 j (j < 4). Frames flo
// .. fhi (indices into d / obase, which may be global or a workgroup's LDS copy)
// cover the unit; chunks at or past own_end belong to another unit owner and are
// skipped; no byte at or past total is written.
// kDpp (r06): one nontemporal load per full chunk; the window's second block is
// the next lane's first (DPP wave shift; lane 63: lane 0's of the next chunk,
// or for the last chunk a load of its own) or the next lane's A-window seam
// block (the left neighbour of a seam chunk). A full chunk with neither (rare:
// the chunk before the batch's last) is built by the seam path afterwards.
template <bool kDpp = false, bool kSeamsOut = false, bool kSeamRec = false, typename DescP,
          typename OffP>
__device__ __forceinline__ void tx_unit(uint8_t *__restrict__ out, const uint8_t *__restrict__ src, DescP d,
                                        OffP obase, uint32_t flo, uint32_t fhi, const fws_tx_desc dA,
                                        const fws_tx_desc dB, uint64_t OA, uint64_t OB, uint64_t a0,
                                        uint64_t own_end, uint64_t total, const uint32_t *__restrict__ rec = nullptr,
                                        uint32_t n_frames = 0) {
    if (fhi - flo >= 2u) {                             // small frames: bytewise with a search
        for (int j = 0; j < 4; ++j) {
            const uint64_t a = a0 + (uint64_t)j * 1024u;
            if (a >= own_end) break;
            const uint32_t f = find_frame(obase, flo, fhi, a);
            tx_bytes(out, src, d, obase, f, a, total);
        }
        return;
    }
    // at most two frames: uniform metadata (dA, dB = d[flo], d[fhi] at OA, OB, by value);
    // payload k of frame X covers [PX, EX)
    TxSeam z;
    z.PA = OA + tx_hdr_len(dA);
    z.EA = z.PA + dA.len;
    z.PB = OB + tx_hdr_len(dB);
    z.EB = z.PB + dB.len;
    const bool two = fhi != flo;
    const bool any_pay = dA.len != 0 || (two && dB.len != 0);          // wave-uniform
    const uint8_t *const safe = src + (dA.len != 0 ? dA.src_off : dB.src_off);
    const uintptr_t safe16 = (uintptr_t)safe & ~uintptr_t(15);
    const uintptr_t SA = (uintptr_t)(src + dA.src_off) - (uintptr_t)z.PA;   // src of output byte a: S + a
    const uintptr_t SB = (uintptr_t)(src + dB.src_off) - (uintptr_t)z.PB;
    uintptr_t sb[4];
    uint32_t sh[4], rk[4];
    uint32_t full = 0, seam = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t a = a0 + (uint64_t)j * 1024u;
        const bool own = a < own_end, whole = a + 16 <= total;   // a chunk crossing `total` is built as a seam
        const bool inA = own && whole && a >= z.PA && a + 16 <= z.EA;
        const bool inB = own && whole && two && a >= z.PB && a + 16 <= z.EB;
        if (inA || inB) full |= 1u << j;
        else if (!kSeamsOut && own && a < total) seam |= 1u << j;
        const uintptr_t sa = (inB ? SB : SA) + (uintptr_t)a;
        sb[j] = (inA || inB) ? (sa & ~uintptr_t(15)) : safe16;
        sh[j] = (uint32_t)(sa & 15u);
        const fws_tx_desc &dx = inB ? dB : dA;
        const uint32_t ph = (uint32_t)(a - (inB ? z.PB : z.PA));
        rk[j] = dx.masked ? rotr32(dx.key, 8u * (ph & 3u)) : 0u;
    }
    // one batch of loads: the full chunks' two aligned source blocks and the
    // A and B source blocks of this lane's first seam chunk
    u32x4 v0[4], v1[4], sa0, sa1, sb0, sb1;
    const int js = seam ? __builtin_ctz(seam) : 0;
    const uint64_t as = a0 + (uint64_t)js * 1024u;
    const uintptr_t sA0 = (uintptr_t)(src + dA.src_off), sB0 = (uintptr_t)(src + dB.src_off);
    uintptr_t qa0, qa1, qb0, qb1;
    uint32_t sha, shb;
    tx_seam_blocks(as, SA, sA0, dA.len, safe16, qa0, qa1, sha);
    tx_seam_blocks(as, SB, sB0, two ? dB.len : 0, safe16, qb0, qb1, shb);
    uint32_t late = 0;
    // kSeamRec: this lane's first seam chunk from the plan's record (tx_seam_records:
    // the owner is the first frame whose header meets the chunk; a record exists
    // when the chunk's bytes end within that frame's payload or at the output's end)
    uint32_t rslot = ~0u;
    if constexpr (kSeamRec) {
        if (seam) {
            const uint32_t hA = tx_hdr_len(dA), hB = tx_hdr_len(dB);
            const bool mA = OA + hA > as && OA < as + 16u;
            const bool mB = two && OB + hB > as && OB < as + 16u;
            if (mA || mB) {
                const uint32_t g = mA ? flo : fhi;
                const uint64_t Og = mA ? OA : OB, Eg = mA ? z.EA : z.EB;
                if (as + 16u <= Eg || g + 1u == n_frames) rslot = 2u * g + (as != (Og & ~uint64_t(15)) ? 1u : 0u);
            } else {
                rslot = 2u * n_frames;                 // the output's last chunk
            }
        }
    }
    u32x4 rv{0u, 0u, 0u, 0u};
    if constexpr (kSeamRec) rv = gload16<false>((uintptr_t)(rec + 4u * (rslot != ~0u ? rslot : 0u)));
    if constexpr (kDpp) {
        const int lane = threadIdx.x & 63;
        u32x4 last = u32x4{0u, 0u, 0u, 0u};
        if (any_pay) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v0[j] = gload16<true>(sb[j]);
            if (lane == 63) last = gload16<true>(((full >> 3) & 1u) && sh[3] ? sb[3] + 16u : sb[3]);
            if constexpr (kSeamsOut) {
                sa0 = sa1 = sb0 = sb1 = u32x4{0u, 0u, 0u, 0u};
                qa0 = 1;                               // no lane's block: the A-window hand-over is off
            } else {
                sa0 = gload16<false>(qa0);
                sa1 = gload16<false>(qa1);
                sb0 = gload16<false>(qb0);
                sb1 = gload16<false>(qb1);
            }
            __builtin_amdgcn_sched_barrier(0);      // keep every load ahead of the first use
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) v0[j] = u32x4{0u, 0u, 0u, 0u};
            sa0 = sa1 = sb0 = sb1 = u32x4{0u, 0u, 0u, 0u};
        }
        // the next lane's A-window seam block (lane 63: lane 0's)
        uint64_t nq = wave_shl1_64(qa0);
        u32x4 wq = wave_shl1(sa0);
        const uint64_t q0 = lane0_of64(qa0);
        const u32x4 w0 = lane0_of(sa0);
        if (lane == 63) {
            nq = q0;
            wq = w0;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint64_t nsb = wave_shl1_64(sb[j]);
            u32x4 w1 = wave_shl1(v0[j]);
            if (j < 3) {
                const uint64_t n0 = lane0_of64(sb[j < 3 ? j + 1 : 0]);
                const u32x4 x0 = lane0_of(v0[j < 3 ? j + 1 : 0]);
                if (lane == 63) {
                    nsb = n0;
                    w1 = x0;
                }
            } else if (lane == 63) {
                nsb = sb[3] + 16u;
                w1 = last;
            }
            // lane 63's seam candidate for chunk j is lane 0's block of chunk j + 1
            const uint64_t need = sb[j] + 16u;
            if (nsb != need && nq == need) w1 = wq;
            if ((full >> j) & 1u) {                  // stored here: v0[j] and w1 die
                if (sh[j] == 0u || nsb == need || nq == need)
                    gstore16<true>((uintptr_t)(out + a0 + (uint64_t)j * 1024u),
                                   tx_shr_bytes(v0[j], w1, sh[j]) ^ rk[j]);
                else
                    late |= 1u << j;
            }
        }
        full = 0;
    } else if (any_pay) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            // default-policy loads: the second block of lane L is the first of lane
            // L + 1, so it must stay in cache (a nontemporal pair reads it twice)
            uintptr_t s1 = sh[j] && ((full >> j) & 1u) ? sb[j] + 16u : sb[j];
            asm volatile("" : "+v"(s1));            // opaque: no "same address as v0" copy
            v0[j] = gload16<false>(sb[j]);          // (a copy would wait for the load)
            v1[j] = gload16<false>(s1);
        }
        if constexpr (kSeamsOut || kSeamRec) {
            sa0 = sa1 = sb0 = sb1 = u32x4{0u, 0u, 0u, 0u};
        } else {
            sa0 = gload16<false>(qa0);
            sa1 = gload16<false>(qa1);
            sb0 = gload16<false>(qb0);
            sb1 = gload16<false>(qb1);
        }
        __builtin_amdgcn_sched_barrier(0);          // keep every load ahead of the first use
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v0[j] = v1[j] = u32x4{0u, 0u, 0u, 0u};
        sa0 = sa1 = sb0 = sb1 = u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if ((full >> j) & 1u)
            gstore16<true>((uintptr_t)(out + a0 + (uint64_t)j * 1024u), tx_shr_bytes(v0[j], v1[j], sh[j]) ^ rk[j]);
    auto seam_chunk = [&](uint64_t a, const u32x4 &A0, const u32x4 &A1, uint32_t shA, const u32x4 &B0,
                          const u32x4 &B1, uint32_t shB) {
        const uint32_t rka = dA.masked ? rotr32(dA.key, 8u * ((uint32_t)(a - z.PA) & 3u)) : 0u;
        const uint32_t rkb = dB.masked ? rotr32(dB.key, 8u * ((uint32_t)(a - z.PB) & 3u)) : 0u;
        const u32x4 x = tx_seam_combine(a, dA, OA, dB, OB, two, z, total, tx_shr_bytes(A0, A1, shA) ^ rka,
                                        tx_shr_bytes(B0, B1, shB) ^ rkb);
        if (a + 16u <= total) gstore16<true>((uintptr_t)(out + a), x);
        else tx_store_tail(out, a, total, x);
    };
#ifdef FWS_TX_ABL_SEAM
    return;                                            // ablation build only: no seam chunks (wrong bytes)
#endif
    if constexpr (kSeamRec) {
        if (seam && rslot != ~0u) {
            if (as + 16u <= total) gstore16<true>((uintptr_t)(out + as), rv);
            else tx_store_tail(out, as, total, rv);
            seam &= seam - 1u;
        }
    } else if (seam) {
        seam_chunk(as, sa0, sa1, sha, sb0, sb1, shb);
        seam &= seam - 1u;
    }
    seam |= late;                                      // kDpp: full chunks without a neighbour block
    if (!__any(seam)) return;                          // a lane with a second seam chunk (rare)
#pragma unroll 1
    for (int j = 0; j < 4; ++j) {
        if (!((seam >> j) & 1u)) continue;
        const uint64_t a = a0 + (uint64_t)j * 1024u;
        tx_seam_blocks(a, SA, sA0, dA.len, safe16, qa0, qa1, sha);
        tx_seam_blocks(a, SB, sB0, two ? dB.len : 0, safe16, qb0, qb1, shb);
        seam_chunk(a, gload16<true>(qa0), gload16<true>(qa1), sha, gload16<true>(qb0), gload16<true>(qb1), shb);
    }
}

// fws_tx_desc from its six words (include/fws_gpu.h layout)
__device__ __forceinline__ fws_tx_desc tx_desc_of(const uint32_t (&w)[6]) {
    fws_tx_desc x;
    x.src_off = w[0] | ((uint64_t)w[1] << 32);
    x.len = w[2] | ((uint64_t)w[3] << 32);
    x.key = w[4];
    x.opcode = (uint8_t)w[5];
    x.fin = (uint8_t)(w[5] >> 8);
    x.masked = (uint8_t)(w[5] >> 16);
    x.pad = (uint8_t)(w[5] >> 24);
    return x;
}

template <bool kDpp = false, bool kSeamsOut = false, bool kSeamRec = false>
__device__ __forceinline__ void tx_encode_body(uint8_t *__restrict__ out, const uint8_t *__restrict__ src,
                                                      const fws_tx_desc *__restrict__ d, uint32_t n,
                                                      const uint64_t *__restrict__ obase,
                                                      const uint32_t *__restrict__ unit_first, uint64_t unit_cap,
                                                      const uint64_t *__restrict__ total_ptr,
                                                      const uint32_t *__restrict__ rec = nullptr) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * (kBlock / 64);
    const uint64_t ufirst = (uint64_t)blockIdx.x * (kBlock / 64) + wave;
    // one scalar round: the total and this wave's first unit map entries (clamped in bounds)
    const uint64_t uc = ufirst + 1 < unit_cap ? ufirst : (unit_cap >= 2 ? unit_cap - 2 : 0);
    uint32_t uf0 = unit_first[uc], uf1 = unit_first[uc + 1];
    const uint64_t total = *total_ptr;
    // (issued together, one wait: the loop test on total had the map loads wait
    // for it in a round of their own)
    asm volatile("" ::"s"(uf0), "s"(uf1), "s"((uint32_t)total));
    const uint64_t n_units = (total + kTxUnit - 1) / kTxUnit;
    for (uint64_t u = ufirst; u < n_units; u += nw) {
        if (u != ufirst || u + 1 >= unit_cap) {       // past the map's capacity: searched (obase)
            uf0 = unit_owner(unit_first, unit_cap, obase, n, u, u * kTxUnit);
            uf1 = u + 1 < n_units ? unit_owner(unit_first, unit_cap, obase, n, u + 1, (u + 1) * kTxUnit) : 0u;
        }
        const uint32_t flo = uf0;
        const uint32_t fhi = (u + 1 < n_units) ? uf1 : n - 1;
        // (copies: a reference into `d` would be re-read after every store to `out`)
        // r06: both descriptors and both offsets as raw words in one scalar round,
        // fields unpacked after it -- loaded as structs, the byte-field unpacking of
        // d[flo] was scheduled before d[fhi]'s loads and the offsets', three
        // dependent rounds per unit, each a full memory latency while HBM is busy
        const uint32_t *wa = reinterpret_cast<const uint32_t *>(d + flo);
        const uint32_t *wb = reinterpret_cast<const uint32_t *>(d + fhi);
        uint32_t ra[6], rb[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            ra[i] = wa[i];
            rb[i] = wb[i];
        }
        const uint64_t OA = obase[flo], OB = obase[fhi];
        // (all four issued, then one wait: an empty asm that takes a word of each --
        // a sched_barrier alone left the loads sunk into the two-frame branch)
        asm volatile("" ::"s"(ra[0]), "s"(ra[5]), "s"(rb[0]), "s"(rb[5]), "s"((uint32_t)OA), "s"((uint32_t)OB));
        const fws_tx_desc dA = tx_desc_of(ra), dB = tx_desc_of(rb);
        tx_unit<kDpp, kSeamsOut, kSeamRec>(out, src, d, obase, flo, fhi, dA, dB, OA, OB,
                                                   u * kTxUnit + (uint64_t)lane * 16u, total, total, rec, n);
    }
}

// ------------------------------------------------------------ one launch
// fws_gpu_encode_frames without the plan launch (r05): frame-major. Workgroup
// b (in ticket order) takes frames [F b, F b + F): one block scan of their
// sizes (+ up to kTxLook frames after them, whose bytes can share the span's
// last 16-B chunk), a decoupled look-back over the workgroups' sums for the
// span's output offset O0 (plan_common.h: the k_out_plan words), then the
// span's 16-B chunks whose first byte lies in [O0, O1) in 4 KiB units, one per
// wave at a time, through tx_unit with the frames' descriptors and offsets in
// LDS. Every chunk has one owner (the workgroup holding its first byte), so
// all but the batch's last chunk are full 16-B stores.
__device__ __forceinline__ uint64_t sgpr64(uint64_t v) {   // a wave-uniform value into SGPRs
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);   // (int results: no sign extension)
}
__device__ __forceinline__ void sgpr_copy(const fws_tx_desc &x, fws_tx_desc &y) {
    static_assert(sizeof(fws_tx_desc) == 24, "6 words");
    const uint32_t *a = reinterpret_cast<const uint32_t *>(&x);
    uint32_t *b = reinterpret_cast<uint32_t *>(&y);
#pragma unroll
    for (int i = 0; i < 6; ++i) b[i] = __builtin_amdgcn_readfirstlane(a[i]);
}

constexpr uint32_t kTxLook = 8;        // frames >= 2 B: 8 of them cover a chunk's 15 bytes past O1
constexpr uint32_t kTxOneMaxF = kBlock - kTxLook;

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(5))) void k_tx_one(
    uint8_t *__restrict__ out, const uint8_t *__restrict__ src, const fws_tx_desc *__restrict__ d, uint32_t n,
    uint32_t F, uint64_t out_cap, uint64_t *__restrict__ out_len, uint64_t *__restrict__ status,
    uint32_t *__restrict__ ticket, uint32_t epoch) {
    __shared__ fws_tx_desc s_d[kBlock];
    __shared__ uint64_t s_ob[kBlock + 1];
    __shared__ uint64_t s_wsum[kBlock / kWave];
    const uint32_t blk = plan_block_order(ticket);
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const uint64_t fb = (uint64_t)blk * F;
    const uint32_t nf = (uint32_t)(n - fb < F ? n - fb : F);                     // this span's frames
    const uint32_t nl = (uint32_t)(n - fb < (uint64_t)nf + kTxLook ? n - fb : nf + kTxLook);   // + look-ahead
    uint64_t sz = 0;
    if (threadIdx.x < nl) {
        const fws_tx_desc x = d[fb + threadIdx.x];
        s_d[threadIdx.x] = x;
        sz = out_size(x);
    }
    const uint64_t inc = wave_incl_scan64(sz, lane);
    if (lane == kWave - 1) s_wsum[w] = inc;
    __syncthreads();
    uint64_t rel = inc - sz;                           // offset of frame t from O0
#pragma unroll
    for (int i = 0; i < kBlock / kWave; ++i) rel += i < w ? s_wsum[i] : 0;
    // s_ob[t] = frame t's offset from O0; s_ob[nl] = the end of the loaded frames,
    // written by the thread of the last loaded frame (nl can be kBlock: there is
    // no thread nl then -- r05 read that entry unwritten, a flaky k_tx_one)
    if (threadIdx.x < nl) s_ob[threadIdx.x] = rel;
    if (threadIdx.x + 1u == nl) s_ob[nl] = rel + sz;
    __syncthreads();
    const uint64_t agg = sgpr64(s_ob[nf]);             // the span's own bytes
    bool unused;
    const uint64_t O0 = sgpr64(block_lookback(status, blk, agg, true, epoch, &unused));
    const uint64_t O1 = O0 + agg, Lend = O0 + sgpr64(s_ob[nl]);
    const bool last = fb + nf >= n;
    if (last && threadIdx.x == 0) *out_len = O1 <= out_cap ? O1 : ~0ull;
    __syncthreads();                                   // every thread read s_ob[nf], s_ob[nl]
    if (threadIdx.x < nl) s_ob[threadIdx.x] += O0;
    if (threadIdx.x + 1u == nl) s_ob[nl] += O0;
    __syncthreads();
    // bytes past the batch (Lend = O1 for the last span) and past out_cap are never written
    const uint64_t clip = Lend < out_cap ? Lend : out_cap;
    const uint64_t A0 = (O0 + 15u) & ~uint64_t(15);    // first chunk whose first byte is ours
    const uint64_t n_units = O1 > A0 ? (O1 - A0 + kTxUnit - 1) / kTxUnit : 0;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint64_t k = wave; k < n_units; k += kBlock / kWave) {
        const uint64_t U0 = A0 + k * kTxUnit;
        if (U0 >= clip) break;                         // wave-uniform
        const uint64_t Ue = (U0 + kTxUnit < clip ? U0 + kTxUnit : clip) - 1u;   // the unit's last byte
        // the frames holding U0 and Ue: count the offsets <= pos (nl + 1 of them, 4 per lane)
        uint32_t flo = 0, fhi = 0;
#pragma unroll
        for (int q = 0; q < kBlock / kWave; ++q) {
            const uint32_t i = (uint32_t)q * kWave + (uint32_t)lane;
            const uint64_t o = i < nl ? s_ob[i] : ~0ull;
            flo += (uint32_t)__popcll(__ballot(o <= U0));
            fhi += (uint32_t)__popcll(__ballot(o <= Ue));
        }
        flo -= 1u;
        fhi -= 1u;
        // the two frames' words from LDS into SGPRs (wave-uniform; LDS loads land in VGPRs)
        fws_tx_desc dA, dB;
        sgpr_copy(s_d[flo], dA);
        sgpr_copy(s_d[fhi], dB);
        const uint64_t OA = sgpr64(s_ob[flo]), OB = sgpr64(s_ob[fhi]);
        tx_unit(out, src, (const fws_tx_desc *)s_d, (const uint64_t *)s_ob, flo, fhi, dA, dB, OA, OB,
                U0 + (uint64_t)lane * 16u, O1, clip);
    }
}

// 4 waves per SIMD (107 VGPRs) as the compiler allocates it, or 5 (96 VGPRs,
// no spill with ROCm 7.2): 5 is the default (C2 TX step 96 -> 90 us, order-
// swapped A/B, profiles/r03/session3/tx_w5_ab.jsonl; 6 waves spill 18 VGPRs);
// tuning hook below.
__global__ __launch_bounds__(kBlock) void k_tx_encode(uint8_t *__restrict__ out, const uint8_t *__restrict__ src,
                                                      const fws_tx_desc *__restrict__ d, uint32_t n,
                                                      const uint64_t *__restrict__ obase,
                                                      const uint32_t *__restrict__ unit_first, uint64_t unit_cap,
                                                      const uint64_t *__restrict__ total_ptr) {
    tx_encode_body(out, src, d, n, obase, unit_first, unit_cap, total_ptr);
}
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(5))) void k_tx_encode_w5(
    uint8_t *__restrict__ out, const uint8_t *__restrict__ src, const fws_tx_desc *__restrict__ d, uint32_t n,
    const uint64_t *__restrict__ obase, const uint32_t *__restrict__ unit_first, uint64_t unit_cap,
    const uint64_t *__restrict__ total_ptr) {
    tx_encode_body(out, src, d, n, obase, unit_first, unit_cap, total_ptr);
}
// r06: one nontemporal load per full chunk (tx_unit<true>), at kW waves per SIMD
template <int kW>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kW))) void k_tx_encode_dpp(
    uint8_t *__restrict__ out, const uint8_t *__restrict__ src, const fws_tx_desc *__restrict__ d, uint32_t n,
    const uint64_t *__restrict__ obase, const uint32_t *__restrict__ unit_first, uint64_t unit_cap,
    const uint64_t *__restrict__ total_ptr) {
    tx_encode_body<true>(out, src, d, n, obase, unit_first, unit_cap, total_ptr);
}
// r06: full chunks only (kSeamsOut; the seam chunks are k_tx_seams's), the
// two-load form (kDpp false) or one load + DPP, at kW waves per SIMD
template <bool kDpp, int kW>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kW))) void k_tx_encode_so(
    uint8_t *__restrict__ out, const uint8_t *__restrict__ src, const fws_tx_desc *__restrict__ d, uint32_t n,
    const uint64_t *__restrict__ obase, const uint32_t *__restrict__ unit_first, uint64_t unit_cap,
    const uint64_t *__restrict__ total_ptr) {
    tx_encode_body<kDpp, true>(out, src, d, n, obase, unit_first, unit_cap, total_ptr);
}

// The seam chunks of a batch (k_tx_encode_so wrote the rest): one thread per
// frame f builds the 16-B output chunks that meet its header [OB, OB + hB) and
// that no earlier frame's header meets (so every chunk has one writer), from
// frame f - 1's payload tail, the header and frame f's payload head -- its
// keyed source windows loaded once, bytes selected in registers (the
// tx_seam_combine of the unit walk); a chunk reaching past frame f's payload
// into frame f + 1 (frames under 16 B) goes bytewise. The last frame's thread
// also writes the output's last chunk when it ends inside a payload. Nothing
// is written when the plan's total is 0 (the batch exceeds out_cap).
__global__ __launch_bounds__(kBlock) void k_tx_seams(uint8_t *__restrict__ out, const uint8_t *__restrict__ src,
                                                     const fws_tx_desc *__restrict__ d, uint32_t n,
                                                     const uint64_t *__restrict__ obase,
                                                     const uint64_t *__restrict__ total_ptr) {
    const uint32_t f = blockIdx.x * kBlock + threadIdx.x;
    const uint64_t total = *total_ptr;
    if (f >= n || total == 0) return;
    const bool hasA = f > 0;
    const fws_tx_desc dB = d[f];
    const uint64_t OB = obase[f];
    fws_tx_desc dA = dB;
    uint64_t OA = OB;
    if (hasA) {
        dA = d[f - 1];
        OA = obase[f - 1];
    }
    const uint32_t hA = tx_hdr_len(dA), hB = tx_hdr_len(dB);
    TxSeam z;
    z.PA = OA + hA;
    z.EA = z.PA + dA.len;
    z.PB = OB + hB;
    z.EB = z.PB + dB.len;
    const uintptr_t sA0 = (uintptr_t)(src + dA.src_off), sB0 = (uintptr_t)(src + dB.src_off);
    const uintptr_t SA = sA0 - (uintptr_t)z.PA, SB = sB0 - (uintptr_t)z.PB;
    const bool payA = hasA && dA.len != 0, payB = dB.len != 0;
    const uintptr_t safe16 = (payB ? sB0 : sA0) & ~uintptr_t(15);
    auto chunk = [&](uint64_t c) {
        const uint64_t ce = c + 16u < total ? c + 16u : total;
        if (ce > z.EB) {                               // meets frame f + 1 too: bytewise
            tx_bytes(out, src, d, obase, c < OB ? f - 1u : f, c, total);
            return;
        }
        u32x4 pA{0u, 0u, 0u, 0u}, pB{0u, 0u, 0u, 0u};
        uintptr_t b0, b1;
        uint32_t sh;
        if (payA && c < z.EA) {
            tx_seam_blocks(c, SA, sA0, dA.len, safe16, b0, b1, sh);
            const uint32_t rk = dA.masked ? rotr32(dA.key, 8u * ((uint32_t)(c - z.PA) & 3u)) : 0u;
            pA = tx_shr_bytes(gload16<true>(b0), gload16<true>(b1), sh) ^ rk;
        }
        if (payB && ce > z.PB) {
            tx_seam_blocks(c, SB, sB0, dB.len, safe16, b0, b1, sh);
            const uint32_t rk = dB.masked ? rotr32(dB.key, 8u * ((uint32_t)(c - z.PB) & 3u)) : 0u;
            pB = tx_shr_bytes(gload16<true>(b0), gload16<true>(b1), sh) ^ rk;
        }
        // (frame 0: A is B itself, one frame)
        const u32x4 x = hasA ? tx_seam_combine(c, dA, OA, dB, OB, true, z, total, pA, pB)
                             : tx_seam_combine(c, dB, OB, dB, OB, false, TxSeam{z.PB, z.EB, z.PB, z.EB}, total, pB,
                                               pB);
        if (c + 16u <= total) gstore16<true>((uintptr_t)(out + c), x);
        else tx_store_tail(out, c, total, x);
    };
    const uint64_t c0 = OB & ~uint64_t(15), c1 = (OB + hB - 1u) & ~uint64_t(15);
    for (uint64_t c = c0; c <= c1 && c < total; c += 16u)
        if (!hasA || OA + hA <= c) chunk(c);           // else frame f - 1's header meets it: its chunk
    if (f == n - 1u && (total & 15u) != 0u) {          // the output's last chunk, when no header meets it
        const uint64_t ct = (total - 1u) & ~uint64_t(15);
        if (ct > c1) chunk(ct);
    }
}

// ------------------------------------------------- seam chunks from the plan
// r06 (kSeamRec): the plan launch builds every seam chunk -- the 16-B output
// chunks meeting a frame header, and the output's last chunk when it ends inside
// a payload -- into a side buffer (never into `out`, so nothing is written when
// the batch exceeds out_cap), one thread per frame, the windows and the byte
// select amortized over a wave of frames; the encode's seam lane copies its
// record. rec[2 f + k]: chunk k (0: the one holding the header's first byte, 1:
// its last byte's when another) of frame f, written when frame f owns it (no
// earlier header meets it) and its bytes end within frame f's payload (or the
// output); rec[2 n]: the last chunk. The encode tests the same two conditions.
__device__ __forceinline__ void tx_seam_records(const uint8_t *__restrict__ src, const fws_tx_desc *__restrict__ d,
                                                uint32_t n, uint32_t f, uint64_t OB, uint32_t *__restrict__ rec) {
    const bool hasA = f > 0, last = f + 1u == n;
    const fws_tx_desc dB = d[f];
    const fws_tx_desc dA = hasA ? d[f - 1u] : dB;
    const uint32_t hB = tx_hdr_len(dB), hA = tx_hdr_len(dA);
    const uint64_t OA = hasA ? OB - out_size(dA) : OB;
    TxSeam z;
    z.PA = OA + hA;
    z.EA = z.PA + dA.len;
    z.PB = OB + hB;
    z.EB = z.PB + dB.len;
    const uint64_t total = last ? z.EB : ~0ull;         // only the last frame's chunks can reach the end
    const uintptr_t sA0 = (uintptr_t)(src + dA.src_off), sB0 = (uintptr_t)(src + dB.src_off);
    const uintptr_t SA = sA0 - (uintptr_t)z.PA, SB = sB0 - (uintptr_t)z.PB;
    const bool payA = hasA && dA.len != 0, payB = dB.len != 0;
    const uintptr_t safe16 = (payB ? sB0 : sA0) & ~uintptr_t(15);
    auto build = [&](uint64_t c, uint32_t slot) {
        u32x4 pA{0u, 0u, 0u, 0u}, pB{0u, 0u, 0u, 0u};
        uintptr_t b0, b1;
        uint32_t sh;
        if (payA && c < z.EA) {
            tx_seam_blocks(c, SA, sA0, dA.len, safe16, b0, b1, sh);
            const uint32_t rk = dA.masked ? rotr32(dA.key, 8u * ((uint32_t)(c - z.PA) & 3u)) : 0u;
            pA = tx_shr_bytes(gload16<true>(b0), gload16<true>(b1), sh) ^ rk;
        }
        if (payB && c + 16u > z.PB) {
            tx_seam_blocks(c, SB, sB0, dB.len, safe16, b0, b1, sh);
            const uint32_t rk = dB.masked ? rotr32(dB.key, 8u * ((uint32_t)(c - z.PB) & 3u)) : 0u;
            pB = tx_shr_bytes(gload16<true>(b0), gload16<true>(b1), sh) ^ rk;
        }
        const u32x4 x = hasA ? tx_seam_combine(c, dA, OA, dB, OB, true, z, total, pA, pB)
                             : tx_seam_combine(c, dB, OB, dB, OB, false, TxSeam{z.PB, z.EB, z.PB, z.EB}, total, pB,
                                               pB);
        gstore16<false>((uintptr_t)(rec + 4u * slot), x);
    };
    const uint64_t c0 = OB & ~uint64_t(15), c1 = (OB + hB - 1u) & ~uint64_t(15);
    for (uint64_t c = c0; c <= c1; c += 16u)
        if ((!hasA || OA + hA <= c) && (c + 16u <= z.EB || last)) build(c, 2u * f + (c != c0 ? 1u : 0u));
    if (last && (z.EB & 15u) != 0u) {                  // the output's last chunk, when no header meets it
        const uint64_t ct = (z.EB - 1u) & ~uint64_t(15);
        if (ct > c1) build(ct, 2u * n);
    }
}

// the TX plan (out_plan_block) and the seam records of its frames, one launch
template <int kF>
__global__ __launch_bounds__(kBlock) void k_tx_plan_seams(const fws_tx_desc *__restrict__ d, uint32_t n,
                                                          OutPlanArgs a, const uint8_t *__restrict__ src,
                                                          uint32_t *__restrict__ rec) {
    const uint32_t blk = plan_block_order(a.ticket);
    out_plan_block<fws_tx_desc, kF>(d, n, a, blk);
    const uint64_t f = uint64_t(blk) * kF + threadIdx.x;
    if (threadIdx.x < (uint32_t)kF && f < n)            // base[f]: this thread's own store in out_plan_block
        tx_seam_records(src, d, n, (uint32_t)f, a.base[f], rec);
}

// r06: full chunks from the source, seam chunks from the plan's records
// (kSeamRec), two loads per chunk, at kW waves per SIMD
template <int kW>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kW))) void k_tx_encode_sr(
    uint8_t *__restrict__ out, const uint8_t *__restrict__ src, const fws_tx_desc *__restrict__ d, uint32_t n,
    const uint64_t *__restrict__ obase, const uint32_t *__restrict__ unit_first, uint64_t unit_cap,
    const uint64_t *__restrict__ total_ptr, const uint32_t *__restrict__ rec) {
    tx_encode_body<false, false, true>(out, src, d, n, obase, unit_first, unit_cap, total_ptr, rec);
}


}  // namespace fwsk

// tuning hook: k_tx_encode grid cap (0 = one wave per output unit, the default:
// 2-8 x the resident workgroups with a grid-stride loop measured 0.091-0.104
// against 0.0906 ms, profiles/r04/ab_tx.jsonl)
static int g_tx_blocks = 0;
extern "C" __attribute__((visibility("default"))) int fws_internal_set_tx_blocks(int blocks) {
    const int old = g_tx_blocks;
    g_tx_blocks = blocks > 0 ? blocks : 0;
    return old;
}

// tuning hook: 1 = k_tx_encode_w5 (default), 0 = the compiler's 4 waves,
// 2 = k_tx_encode_dpp<5> (one load + DPP), 3 / 4 = k_tx_encode_so two loads / DPP
// (full chunks only) + k_tx_seams, 5 = k_tx_plan_seams + k_tx_encode_sr<5> (seam
// chunks built by the plan). r06, four rotating sources: none beat 1 (DESIGN
// §4.6); measured and removed: DPP at 6 / 7 / 8 waves and the two-load form at 6
// / 7 (spills, 0.140-0.250 ms), late seam windows at 6 / 8 waves (0.105 / 0.122),
// the so / sr forms at 6 / 8 waves (0.102-0.149).
static int g_tx_w5 = 1;
extern "C" __attribute__((visibility("default"))) int fws_internal_set_tx_w5(int on) {
    const int old = g_tx_w5;
    g_tx_w5 = on >= 0 && on <= 5 ? on : 1;
    return old;
}

// tuning hook: the one-launch form k_tx_one (1: for batches whose frames
// average <= kTxOneMaxAvg bytes of out_cap; 2 = for every batch, tests) or plan +
// encode (0, the default); and the output bytes per k_tx_one workgroup (its
// frames F = span / average frame). Measured on the C2 TX shape (r05,
// profiles/r05/ab_tx.jsonl, one process, order alternated): plan + encode
// 0.105 ms, k_tx_one 0.132 ms at 128 KiB per workgroup, 0.141 at 64 / 256 KiB,
// 0.169 at 32 KiB. A frame-major grid has one wave per ~span / 4 workgroup
// units: at 128 KiB spans 2,048 waves (2 per SIMD) stream the whole batch, too
// few to keep HBM busy; smaller spans add workgroups whose look-back chains
// (read 256 predecessors a round) grow with the grid. The unit-major kernel
// keeps one wave per 4 KiB unit (65,668) and pays one plan launch.
static int g_tx_one = 0;   // off: measured slower (tools/ab_tx.py, profiles/r05/ab_tx.jsonl)
static uint64_t g_tx_one_span = 64u << 10;
constexpr uint64_t kTxOneMaxAvg = 16u << 10;
extern "C" __attribute__((visibility("default"))) int fws_internal_set_tx_one(int on, int span_kib) {
    const int old = g_tx_one;
    g_tx_one = on < 0 ? 0 : (on > 2 ? 2 : on);
    if (span_kib > 0) g_tx_one_span = (uint64_t)span_kib << 10;
    return old;
}

using namespace fwsk;

extern "C" {

void fws_tx_next(uint32_t frame_type, int last_frame_if_possible, uint8_t *last_msg_not_fin, uint8_t *opcode,
                 uint8_t *fin) {
    // w_socket.h:845-848, 903-913: a data frame continuing an unfinished message
    // is a continuation (opcode 0); control frames neither use nor change the state.
    const bool is_last = last_frame_if_possible != 0;
    const bool is_control = (frame_type & 8u) != 0;
    uint8_t op = 0;
    if (!*last_msg_not_fin || is_control) op = (uint8_t)frame_type;
    if (!is_control) *last_msg_not_fin = is_last ? 0 : 1;
    *opcode = op;
    *fin = is_last ? 1 : 0;
}

int fws_gpu_encode_frames(fws_gpu_ctx *ctx, void *dev_out, uint64_t out_cap, const void *dev_src,
                          const fws_tx_desc *dev_descs, uint32_t n, uint64_t *dev_out_len, void *stream) {
    if (!ctx || !dev_out_len || (n && (!dev_out || !dev_src || !dev_descs))) return FWS_ERR_INVALID;
    if (((uintptr_t)dev_out & 15u) != 0) return FWS_ERR_INVALID;
    hipStream_t s = (hipStream_t)stream;
    int r = fws_hip_status(hipSetDevice(ctx->device));
    if (r) return r;
    if (n == 0) return fws_hip_status(hipMemsetAsync(dev_out_len, 0, sizeof(uint64_t), s));
    const uint64_t units = out_cap / kTxUnit + 2;
    const uint64_t avg = out_cap / n;
    if (g_tx_one == 2 || (g_tx_one == 1 && avg <= kTxOneMaxAvg)) {
        // one launch: ~g_tx_one_span output bytes (F frames) per workgroup
        if ((r = fws_ctx_ensure_plan(ctx, n, 2))) return r;
        fws_plan_ws &ws = ctx->plan;
        uint64_t F = g_tx_one_span / (avg ? avg : 1u);
        if (F < 8u) F = 8u;
        if (F > kTxOneMaxF) F = kTxOneMaxF;
        const uint64_t nb = (n + F - 1) / F;
        if (nb > ws.status_cap || nb > (1u << 30)) return FWS_ERR_CAPACITY;
        if ((r = fws_plan_next_epoch(ws, s))) return r;
        hipLaunchKernelGGL(k_tx_one, dim3((unsigned)nb), dim3(kBlock), 0, s, (uint8_t *)dev_out,
                           (const uint8_t *)dev_src, dev_descs, n, (uint32_t)F, out_cap, dev_out_len, ws.status,
                           ws.ticket, ws.epoch);
        return fws_hip_status(hipGetLastError());
    }
    if ((r = fws_ctx_ensure_plan(ctx, n, units))) return r;
    fws_plan_ws &ws = ctx->plan;
    const bool seam_rec = g_tx_w5 == 5;
    if (seam_rec) {                                    // the plan with the seam chunks (outplan_kernels.hip's shape)
        const bool small = n <= 16384u;
        const uint32_t nb = small ? (n + 63u) / 64u : (n + kBlock - 1) / kBlock;
        if (nb > ws.status_cap) return FWS_ERR_CAPACITY;
        if ((r = fws_plan_next_epoch(ws, s))) return r;
        OutPlanArgs pa{ws.cbase, ws.unit_first, ws.unit_cap, ws.total, dev_out_len, out_cap, ws.status, ws.ticket,
                       ws.epoch};
        if (small)
            hipLaunchKernelGGL((k_tx_plan_seams<64>), dim3(nb), dim3(kBlock), 0, s, dev_descs, n, pa,
                               (const uint8_t *)dev_src, ws.tx_seam);
        else
            hipLaunchKernelGGL((k_tx_plan_seams<kBlock>), dim3(nb), dim3(kBlock), 0, s, dev_descs, n, pa,
                               (const uint8_t *)dev_src, ws.tx_seam);
        if ((r = fws_hip_status(hipGetLastError()))) return r;
    } else if ((r = fws_launch_tx_plan(dev_descs, n, ws, out_cap, dev_out_len, s))) {
        return r;
    }
    uint64_t u = units < ws.unit_cap ? units : ws.unit_cap;
    uint64_t blocks = (u + 3) / 4;
    // one wave per unit in one pass (a cap at 16 384 workgroups left a C2-shaped
    // TX batch's last 129 units to a second round of a few waves)
    if (blocks > (1u << 30)) blocks = 1u << 30;
    if (g_tx_blocks && blocks > (uint64_t)g_tx_blocks) blocks = (uint64_t)g_tx_blocks;
    const void *k = g_tx_w5 == 0   ? (const void *)k_tx_encode
                    : g_tx_w5 == 2 ? (const void *)k_tx_encode_dpp<5>
                    : g_tx_w5 == 3 ? (const void *)k_tx_encode_so<false, 5>
                    : g_tx_w5 == 4 ? (const void *)k_tx_encode_so<true, 5>
                    : g_tx_w5 == 5 ? (const void *)k_tx_encode_sr<5>
                                   : (const void *)k_tx_encode_w5;
    uint8_t *o = (uint8_t *)dev_out;
    const uint8_t *sp = (const uint8_t *)dev_src;
    const uint32_t *rec = ws.tx_seam;
    void *args[] = {&o, &sp, &dev_descs, &n, &ws.cbase, &ws.unit_first, &ws.unit_cap, &ws.total, &rec};
    void *args8[] = {&o, &sp, &dev_descs, &n, &ws.cbase, &ws.unit_first, &ws.unit_cap, &ws.total};
    if ((r = fws_hip_status(hipLaunchKernel(k, dim3((unsigned)blocks), dim3(kBlock), seam_rec ? args : args8, 0, s))))
        return r;
    if (g_tx_w5 == 3 || g_tx_w5 == 4)                  // the seam chunks the encode left
        hipLaunchKernelGGL(k_tx_seams, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, o, sp, dev_descs, n,
                           (const uint64_t *)ws.cbase, (const uint64_t *)ws.total);
    return fws_hip_status(hipGetLastError());
}

}  // extern "C"
