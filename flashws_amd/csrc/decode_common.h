// decode_common.h -- constants and node encodings shared by the stream-decode
// kernels: k_scan (decode_kernels.hip) and the resolve (merge_kernels.hip).
#pragma once

#include "fws_device.h"
#include "fws_internal.h"

namespace fwsk {

constexpr uint32_t kTile = 2048;             // bytes per scan tile (one wavefront)
constexpr uint32_t kHalo = 16;               // header bytes past the tile end
constexpr uint16_t kDead = 0xFFFF;
constexpr uint16_t kLeaf = 0x8000;           // kLeaf | offset: chain ends at this header

constexpr uint32_t kNone = 0xFFFFFFFFu;           // "no node" (memset 0xFF)
constexpr uint32_t kTermEnd = 0xFFFFFFFEu;        // chain reaches / passes the stream end
constexpr uint32_t kTermDead = 0xFFFFFFFDu;       // next header offset is not a survivor
constexpr uint32_t kTermIncomplete = 0xFFFFFFFCu; // incomplete header at the stream end
__device__ __forceinline__ bool is_term(uint32_t v) { return v >= kTermIncomplete; }

// dec.counters[] (zeroed before every decode)
enum Counter {
    kCntSurv = 0,        // survivors (sum of the tiles' counts)
    kCntOverflow = 1,    // bit 0: k_scan's survivor spill capacity exceeded
    kCntDenseTiles = 2,  // tiles k_scan left to dense_tile() (diagnostic)
    kCntFrames = 3,      // frames emitted (device frame count, read by the unmask)
    kCntRoot = 4,        // k_merge (super tile 0) on the header at offset 0: 0 = not recorded (the
                         //   big-ST paths), 1 = no survivor there, 2 + kind = this survivor's chain:
    kCntRootSid = 5,     //   its slot id,
    kCntRootTail = 6,    //   fws_node_res::tail and
    kCntSpill = 7,       // survivors spilled by dense tiles
    kCntEmitDoubling = 8, // super tiles whose k_emit marked the chain by pointer doubling (diagnostic)
    kCntFallback = 9,    // the resolve failed (workspace capacity): the result says so, k_emit skips
    kCntTicket = 10,     // k_link workgroups finished (the last one resolves the path)
    kCntTails = 11,      // super-tile exit tails appended by k_merge
    kCntBig = 12,        // super tiles that took k_merge's big-ST path (diagnostic)
    kCntScanDense = 13,  // tiles k_scan marked kDenseTile (k_merge rewrites their counts: its early
                         //   landing lookups need a stream with none)
    // 14..17: unused
    kCntRootCnt = 18,    //   ::cnt (ent is 0) -- resolve_path skips four dependent loads
    kCntCount = 19
};
// Spill runs: k_scan wavefront gw reserves from region gw % kSpillRegions (its
// own counter at kCntRegion0 + region * kRegionStride, one 128-B line each: no
// hot atomic or hot line when every tile spills), then from the shared second
// half (kCntSpill; dense_tile uses only that)
constexpr uint32_t kSpillRegions = 64;
constexpr uint32_t kCntRegion0 = 64;
constexpr uint32_t kRegionStride = 32;
constexpr uint32_t kCntStride = kCntRegion0 + kSpillRegions * kRegionStride;   // words per counter set
static_assert(kCntRegion0 >= kCntCount, "counter layout");
// [0, half): kSpillRegions regions of region_size; [half, s_cap): shared
__device__ __forceinline__ uint32_t spill_half(uint32_t s_cap) { return s_cap / 2u; }
__device__ __forceinline__ uint32_t spill_region_size(uint32_t s_cap) { return spill_half(s_cap) / kSpillRegions; }
// a shared spill run of ns records, or kNone (capacity exceeded: kCntOverflow set)
__device__ __forceinline__ uint32_t spill_shared(uint32_t *counters, uint32_t s_cap, uint32_t ns) {
    const uint32_t off = atomicAdd(&counters[kCntSpill], ns);
    const uint32_t room = s_cap - spill_half(s_cap);
    if (off > room || room - off < ns) {
        atomicOr(&counters[kCntOverflow], 1u);
        return kNone;
    }
    return spill_half(s_cap) + off;
}
static_assert(kCntFrames == kDecodeFramesCounter, "fws_internal.h names the frame counter");

constexpr uint32_t kSlots = 8;               // per-tile survivor slots before spilling
constexpr uint32_t kDenseTile = 0xFFFFFFFEu; // tile_count mark: k_scan left the tile to k_scan_dense (which overwrites it)

__device__ __forceinline__ uint64_t exit_of(const fws_frame_info &fi) {
    return fi.hdr_off + fi.hdr_len + fi.payload_len;
}


// Exclusive scan over a kT-thread workgroup; *total = the workgroup sum.
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

}  // namespace fwsk
