// fws_internal.h -- host-side internals of libfws_gpu (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fws_gpu.h"

// Map a HIP error to the ABI's negative range (fws_gpu.h FWS_ERR_HIP_BASE).
static inline int fws_hip_status(hipError_t e) {
    return e == hipSuccess ? 0 : (FWS_ERR_HIP_BASE - (int)e);
}

// One-launch decode of a small read (small_kernels.hip): streams of at most
// kSmallMax bytes (16-B aligned base) with at most kSmallFrames headers;
// more headers -> res->status = FWS_SMALL_DECLINED, nothing else written.
constexpr uint64_t kSmallMax = 128u << 10;
constexpr uint32_t kSmallFrames = 256;
constexpr int FWS_SMALL_DECLINED = -30;
int fws_resolve_mode();   // decode_kernels.hip test hook (fws_internal_set_resolve_mode)
int fws_launch_decode_small(uint8_t *wire, uint64_t N, fws_frame_info *frames, uint32_t cap,
                            fws_decode_result *res, hipStream_t s);
// One segment of a multi-connection batch (fws_rx_mux, rx_session.cpp): the
// continuation bytes [cont_off, cont_off + u) unmasked with `key` (rotated to
// their first byte), then the header stream [hs_off, hs_off + L) decoded into
// frames[fbase, fbase + fcap) and res[segment]. Both offsets 16-B aligned.
struct fws_seg_desc {
    uint64_t cont_off;
    uint64_t hs_off;
    uint32_t u;
    uint32_t key;
    uint32_t L;                        // <= kSmallMax
    uint32_t fcap;
    uint32_t fbase;
    uint32_t pad;
};
// flag (optional, host memory): `seq` is stored there once every segment's
// results are visible to the host; ctr (with flag): a monotonic device counter,
// target = its value once this launch's n workgroups have counted
int fws_launch_decode_segments(uint8_t *batch, const fws_seg_desc *segs, uint32_t n, fws_frame_info *frames,
                               fws_decode_result *res, hipStream_t s, uint32_t *ctr = nullptr, uint32_t target = 0,
                               uint32_t *flag = nullptr, uint32_t seq = 0);
// registered host memory (fws_gpu_host_register, rx_pipe.cpp): the device
// address of [p, p + n) when it lies inside one registered range, else null
uint8_t *fws_host_alias(const void *p, uint64_t n);
void fws_host_registry_add(const uint8_t *host, uint64_t bytes, uint8_t *dev);
void fws_host_registry_remove(const uint8_t *host);
// one segment, its descriptor by value (the RX session's staged read)
int fws_launch_decode_one(uint8_t *batch, const fws_seg_desc &d, fws_frame_info *frames, fws_decode_result *res,
                          hipStream_t s, uint32_t *flag = nullptr, uint32_t seq = 0);
// wait for a host_done flag (small_kernels.hip): spin briefly, then
// synchronize the stream (which also reports a failed launch)
int fws_wait_flag(const volatile uint32_t *flag, uint32_t seq, hipStream_t s);

// ---- the persistent receive service (r05; small_kernels.hip k_rx_service,
// rx_session.cpp fws_rx_service): the small-read decodes of fws_rx_session and
// fws_rx_mux without a kernel launch per read. One lingering grid: a poller
// workgroup reads a mailbox in coherent pinned memory and republishes each
// request in device memory; `workers` workgroups decode its segments
// (decode_segment, as k_decode_segments does) and the last one stores the
// request's host flag. state = (seq << 1) | running: the host publishes a
// request by a CAS from (s, running) to (s + 1, running), and launches a new
// grid when the running bit is clear; the poller clears it by a CAS after
// `linger` ticks without a request (or once `life` ticks have passed), so an
// idle grid always exits and a request is never lost between the two.
struct fws_svc_req {
    uint64_t base;                     // segment offsets are relative to it (mod 2^64)
    uint64_t descs;                    // fws_seg_desc[nseg] (host or device memory), or 0: `one`
    uint64_t frames;                   // fws_frame_info*
    uint64_t res;                      // fws_decode_result[nseg]
    uint64_t flag;                     // uint32_t* in host memory: flag_seq is stored there when done
    uint64_t out;                      // kind 2: where the decoded bytes [0, span) of base go (host memory)
    uint32_t nseg, flag_seq, kind, span;   // kind 1: quit; 2: a pushed read (base: device staging)
    fws_seg_desc one;
};
static_assert(sizeof(fws_svc_req) % 8 == 0, "8-B words");
// One 128-B line: the poller's wave reads all of it with one coalesced load per
// poll (one PCIe round trip for the state and the request together). `tag` =
// the request's seq, written with the request (a later 64-B half than the
// state word): a read that sees the new state and the new tag saw the whole
// request, since the host writes the request, then the tag, then CASes state.
// Push mode (large-BAR devices, r05): the line the poller reads lives in
// fine-grained device memory and the host writes it -- and a pushed read's
// bytes, into the staging after it -- with CPU stores, an sfence before the
// state word and one after it (write-combining buffers otherwise hold them).
// The running bit keeps its CAS protocol on the pinned host line's state word.
struct alignas(128) fws_svc_mail {     // coherent pinned host memory (or device memory: push mode)
    uint64_t state;
    fws_svc_req req;                   // written before the CAS that publishes its seq
    uint64_t tag;
    uint64_t pad[1];
};
static_assert(sizeof(fws_svc_mail) == 128, "one line");
struct alignas(128) fws_svc_dev {      // device memory, zeroed before each launch
    uint64_t seqn;                     // the request's seq | its segment count << 32 (one word: a worker
                                       //   without a segment of it needs no fence)
    uint32_t quit, ctr, pad[28];
    fws_svc_req req;
};
// mail: the pinned line (its state word's running bit); poll: the line the
// poller reads (mail, or the device-memory line in push mode)
int fws_launch_rx_service(fws_svc_mail *mail, const fws_svc_mail *poll, fws_svc_dev *dv, uint32_t seq0,
                          uint32_t workers, uint64_t linger_ticks, uint64_t life_ticks, uint32_t trace, hipStream_t s);
int fws_rx_service_trace_read(unsigned long long *out8);
struct fws_rx_service;
// the context's service (created on first use when enabled), or null: not enabled
fws_rx_service *fws_ctx_rx_service(fws_gpu_ctx *ctx);
void fws_rx_service_destroy(fws_rx_service *v);
// one request through the service, waited for: segments [0, nseg) of `descs`
// (or the one `*one`) relative to base; returns 0 once flag == flag_seq
int fws_rx_service_run(fws_rx_service *v, uint8_t *base, const fws_seg_desc *descs, const fws_seg_desc *one,
                       uint32_t nseg, fws_frame_info *frames, fws_decode_result *res, uint32_t *flag,
                       uint32_t flag_seq);
// The same request published and not waited for (fws_rx_mux_submit); the next
// request on the service, or fws_rx_service_wait(flag, flag_seq), waits for it.
int fws_rx_service_post(fws_rx_service *v, uint8_t *base, const fws_seg_desc *descs, uint32_t nseg,
                        fws_frame_info *frames, fws_decode_result *res, uint32_t *flag, uint32_t flag_seq);
int fws_rx_service_wait(fws_rx_service *v, uint32_t *flag, uint32_t flag_seq);
// Push mode: can a read of `span` staged bytes be pushed (the service runs in
// push mode and its device staging holds them)?
bool fws_rx_service_can_push(const fws_rx_service *v, uint64_t span);
uint32_t fws_rx_service_workers(const fws_rx_service *v);   // its decode workgroups (0: none)
// One pushed read, waited for: the host bytes src[0, span) are copied into the
// service's device staging with CPU stores, decoded there as segment `d`
// (offsets relative to the staging, 16-B aligned layout), and the decoded bytes
// are written to out_dev[0, span) (host memory the device addresses: a
// registered alias or pinned memory) before the flag.
int fws_rx_service_push(fws_rx_service *v, const uint8_t *src, uint64_t span, uint8_t *out_dev, const fws_seg_desc &d,
                        fws_frame_info *frames, fws_decode_result *res, uint32_t *flag, uint32_t flag_seq);

// Device workspace for the chunk plan of one descriptor batch.
// Descriptor batches are planned two ways in one launch (k_plan): chunk space
// (cbase / unit_first: any descriptor order) and byte space (unit_first_s:
// sorted, non-overlapping payloads, one owner per 16-B chunk, no partial
// stores inside the batch). mode[] tells k_unmask_desc which one holds.
struct fws_plan_ws {
    uint64_t *block_sums = nullptr;   // ceil(n / 1024): gather plan (text_kernels.hip)
    uint64_t *cbase = nullptr;        // n + 1
    uint32_t *unit_first = nullptr;   // units (total chunks / 256) + 1
    uint32_t *unit_rec = nullptr;     // byte-space units + 1, 4 words each (fws_unit_rec, k_plan)
    uint64_t *total = nullptr;        // 1
    uint64_t *status = nullptr;       // ceil(n / 1024): k_plan look-back words (epoch-tagged)
    uint32_t *ticket = nullptr;       // k_plan's ordered block ticket (reset by its last block)
    uint64_t *mode = nullptr;         // kPlanModeWords: fws_plan_mode
    uint32_t *tx_seam = nullptr;      // TX seam chunks built by the plan: 2 per frame + the tail, 4 words each
    uint64_t status_cap = 0;
    uint32_t epoch = 0;               // tag of the last k_plan's status words (1..0xFFFF)
    uint64_t unit_cap = 0;            // capacity of unit_first / unit_first_s (writes are clamped)
};

// k_plan's result for the run (device words, base-relative offsets).
struct fws_plan_mode {
    uint64_t byte_space;              // 1: unit_first_s holds (sorted, non-overlapping, dense)
    uint64_t s0;                      // base offset of byte-space unit 0 (first payload, 16-B floor)
    uint64_t first_po;                // first payload byte of the batch
    uint64_t last_pe;                 // end of the last payload of the batch
    uint64_t n_units;                 // byte-space units
    uint64_t pad[3];
};

// Super-tile resolve records (merge_kernels.hip).
struct fws_node_res {                 // per survivor: its chain inside its super tile
    uint32_t tail;                    // EXIT: tail-list index; else the chain's tail survivor
                                      //   (ST-local index, or slot id on the big-ST path)
    uint32_t cnt;                     // frames from this survivor up to and including the tail
    uint32_t ent;                     // this survivor as its ST's entry: ST-local index / slot id
    uint32_t kind;                    // merge_kernels.hip kKind* | kBigBit
};
struct fws_tail_rec {                 // one EXIT tail: a chain leaving its super tile
    uint64_t exit;                    // offset of the next header
    uint32_t id;                      // slot id of the tail survivor
    uint32_t w;                       // slot id of the survivor at `exit`, or DEAD
    uint32_t wst;                     // super tile of `exit`
    uint32_t pad;
};

// one survivor in its super tile's table (k_merge -> k_emit)
struct fws_st_node {
    uint32_t sid;                     // slot id of the record
    uint16_t nx;                      // in-ST next (local index) or exit code
    uint16_t tail;                    // local index of its chain's tail in the ST
    uint16_t cnt;                     // frames from it up to and including the tail
    uint8_t wt;                       // 1: a frame; 0: incomplete header
    uint8_t pad0;
    uint32_t pad1;
};

// Stream-decode workspace (decode_kernels.hip, merge_kernels.hip).
struct fws_decode_ws {
    uint64_t max_tiles = 0;
    uint64_t max_surv = 0;            // capacity of the spill survivor arrays
    uint32_t *tile_count = nullptr;   // survivors per tile
    uint32_t *counters = nullptr;     // this call's set (decode_common.h Counter)
    uint32_t *cnt_base = nullptr;     // two sets of kCntStride words: a call uses one, its k_emit
    uint32_t parity = 0;              //   launch zeroes the other for the next call (no memset launch)
    bool cnt_dirty = true;            // zero this call's set first (new allocation, failed call)
    fws_frame_info *stage_info = nullptr;  // per-tile survivor slots (k_scan)
    fws_frame_info *spill_info = nullptr;  // survivors of dense tiles
    uint32_t *tile_spill = nullptr;        // spill offset of a dense tile, or ~0
    uint32_t scan_grid = 0;                // persistent k_scan workgroups
    uint32_t *scan_dummy = nullptr;        // one 64-B line per k_scan wavefront (idle-lane stores)
    // super-tile resolve (merge_kernels.hip)
    uint64_t max_nodes = 0;                // slot ids: tiles * 8 + spill capacity
    uint64_t max_st = 0;
    uint32_t tail_cap = 0;
    fws_node_res *nres = nullptr;          // [max_nodes]
    fws_tail_rec *tails = nullptr;         // [tail_cap]
    uint32_t *gnx = nullptr;               // [tail_cap] next tail / terminal
    uint64_t *tpk = nullptr;               // [2 * tail_cap] per tail: the landing entry, its frame
                                           //   count, end record, ST (k_link -> its last workgroup)
    uint32_t *tmark = nullptr;             // [tail_cap / 32 + 1] tails that are some tail's next
    uint32_t *comp = nullptr;              // [fws_merge_comp_cap()] marked tails, compacted
    fws_st_node *st_nodes = nullptr;       // [max_st * kStCap] survivors per super tile (8 B each)
    uint32_t *st_n = nullptr;              // [max_st] survivors per super tile
    uint32_t *st_nt = nullptr;             // [max_st] EXIT tails in the super tile's own run (0: overflow area)
    uint32_t *st_entry = nullptr;          // [max_st] the path's first header in the ST (local index / slot id)
    uint32_t *st_fbase = nullptr;          // [max_st] frames before the ST
    // big-ST path: super tiles with more survivors than LDS holds (dense small
    // frames) run the same merge / emit over these, indexed by slot id
    uint32_t *bg_nx = nullptr;             // [max_nodes] in-ST next slot id or exit code
    uint32_t *bg_wt = nullptr;             // [max_nodes] 1: a frame; 0: incomplete header
    uint32_t *bg_lref = nullptr;           // [max_nodes] EXIT tail's index in the ST's tail run
    uint32_t *bg_ptr = nullptr;            // [2][max_nodes] pointer jumping
    uint32_t *bg_sc = nullptr;             // [2][max_nodes] frame counts
    uint32_t *bg_mark = nullptr;           // [max_nodes] k_emit: on the path
};

struct fws_gpu_ctx {
    int device = 0;
    uint64_t cap_frames = 0;
    uint64_t cap_units = 0;
    uint64_t cap_stream = 0;
    fws_plan_ws plan;
    fws_decode_ws dec;
    void *pinned = nullptr;           // host staging for small readbacks
    uint32_t *seam = nullptr;         // fws_gpu_unmask_sorted_utf8: first / last unmasked dword per unit
    uint64_t seam_cap = 0;            // words
    uint64_t *any_q = nullptr;        // fws_gpu_unmask_batch (one launch): queued pieces of long regions
    uint32_t *any_cnt = nullptr;      // 2 words: queue counts by call parity
    uint32_t any_qcap = 0;
    uint32_t any_parity = 0;
    uint32_t svc_workers = 0;         // fws_gpu_ctx_set_rx_persistent: 0 = off
    fws_rx_service *svc = nullptr;
};
int fws_ctx_ensure_seam(fws_gpu_ctx *ctx, uint64_t span);
int fws_ctx_ensure_any(fws_gpu_ctx *ctx);             // the piece queue, sized from the reservation

int fws_ctx_ensure_plan(fws_gpu_ctx *ctx, uint64_t frames, uint64_t units);

// unmask_kernels.hip
int fws_launch_mask_single(void *dev_ptr, uint64_t n, uint32_t key, uint32_t phase, hipStream_t s);
// n_dev (optional, device memory): the actual count, <= n (n is the host-side bound).
int fws_launch_plan(const uint8_t *base, const fws_frame_desc *d, uint32_t n, const uint32_t *n_dev,
                    fws_plan_ws &ws, hipStream_t s);
int fws_launch_unmask(uint8_t *base, const fws_frame_desc *d, uint32_t n, const uint32_t *n_dev,
                      const fws_plan_ws &ws, uint64_t max_chunks, hipStream_t s);
// fws_gpu_unmask_batch in one launch (descriptor-major) + the queued pieces of
// regions over 64 KiB; qcnt / qnext: this call's and the next call's count
bool fws_unmask_any_on();
int fws_launch_unmask_any(uint8_t *base, const fws_frame_desc *d, uint32_t n, uint64_t *queue, uint32_t qcap,
                          uint32_t *qcnt, uint32_t *qnext, uint32_t piece_grid, hipStream_t s);
int fws_launch_unmask_sorted(uint8_t *base, const fws_frame_desc *d, uint32_t n, uint64_t max_span,
                             hipStream_t s);
// *bad = the first index breaking the sorted / disjoint contract, or ~0 (device word)
int fws_launch_check_sorted(const fws_frame_desc *d, uint32_t n, uint32_t *bad, hipStream_t s);
// seam (2 words per 4 KiB unit of the span + 4): the first and last unmasked dword of
// every unit, written by the unmask and read by the unit-seam UTF-8 check
// (seam_words: its capacity; units past seam_words / 2 -- a batch wider than the
// context's reservation -- write no words and the seam check reads the stream)
int fws_launch_unmask_sorted_utf8(uint8_t *base, const fws_frame_desc *d, uint32_t n, uint64_t max_span,
                                  uint8_t *ok, uint32_t *seam, uint64_t seam_words, hipStream_t s);
// Decoded stream in stream-byte space: unit_first[u] = frame spanning byte 4 KiB * u (the decode's plan).
// utf8_ok (optional): per-frame flags, preset by the resolve to TEXT && FIN && complete; cleared here on
// a UTF-8 error found while the payload is in registers (+ k_utf8_seam for unit seams).
// seam (utf8_ok only; 2 words per 4 KiB unit + 4): each unit's first / last unmasked dword
// for the unit-seam check.
int fws_launch_unmask_stream(uint8_t *base, uint64_t N, const fws_frame_info *frames, uint32_t cap,
                             const uint32_t *n_dev, const uint32_t *unit_first, uint8_t *utf8_ok,
                             uint32_t *seam, hipStream_t s);

// outplan_kernels.hip: one-launch output-space plans (base = ws.cbase, unit map, total)
int fws_plan_next_epoch(fws_plan_ws &ws, hipStream_t s);
int fws_launch_gather_plan(const fws_frame_desc *d, uint32_t n, fws_plan_ws &ws, hipStream_t s);
int fws_launch_tx_plan(const fws_tx_desc *d, uint32_t n, fws_plan_ws &ws, uint64_t out_cap, uint64_t *out_len,
                       hipStream_t s);

// text_kernels.hip
int fws_launch_utf8_descs(const uint8_t *base, const fws_frame_desc *descs, uint32_t n, uint8_t *ok,
                          hipStream_t s);
int fws_launch_gather(uint8_t *dst, const uint8_t *src, const fws_frame_desc *d, uint32_t n, fws_plan_ws &ws,
                      uint64_t max_bytes, hipStream_t s);

// decode_kernels.hip
constexpr int kDecodeFramesCounter = 3;   // index of the device frame count in dec.counters
int fws_decode_ensure(fws_gpu_ctx *ctx, uint64_t N, uint32_t cap);
// utf8_ok (optional): per-frame UTF-8 flags, preset here, finished by fws_launch_unmask_stream
int fws_launch_decode(fws_gpu_ctx *ctx, uint8_t *wire, uint64_t N, fws_frame_info *frames, uint32_t cap,
                      fws_decode_result *res, uint8_t *utf8_ok, hipStream_t s);
// the same in two halves, which may run on two streams (fws_decode_engine): the
// scan, then -- after it, with nothing else on this context in between -- the
// resolve
int fws_launch_decode_scan(fws_gpu_ctx *ctx, uint8_t *wire, uint64_t N, hipStream_t s);
int fws_launch_decode_resolve(fws_gpu_ctx *ctx, uint8_t *wire, uint64_t N, fws_frame_info *frames, uint32_t cap,
                              fws_decode_result *res, uint8_t *utf8_ok, hipStream_t s);
// fws_gpu_decode_stream's workspace for a stream of len bytes / cap frames (may reallocate)
int fws_decode_prepare(fws_gpu_ctx *ctx, uint64_t len, uint32_t cap, bool utf8);
// its unmask launch (after the resolve, on the resolve's stream)
int fws_decode_unmask(fws_gpu_ctx *ctx, uint8_t *wire, uint64_t len, fws_frame_info *frames, uint32_t cap,
                      uint8_t *utf8_ok, hipStream_t s);
// merge_kernels.hip: from k_scan's survivors to the frame list, the result and the
// unmask plan (k_merge -> k_link + path -> k_emit); no grid barrier anywhere
uint64_t fws_merge_super_tiles(uint64_t n_tiles);
uint64_t fws_merge_super_tiles_cap(uint64_t n_tiles);   // bound over every n <= n_tiles (table sizes)
uint32_t fws_merge_tail_cap(uint64_t n_tiles);
uint64_t fws_merge_st_nodes(uint64_t n_tiles);
uint32_t fws_merge_comp_cap();
int fws_launch_merge(fws_gpu_ctx *ctx, const uint8_t *wire, uint64_t N, uint32_t n_tiles, fws_frame_info *frames,
                     uint32_t cap, fws_decode_result *res, uint8_t *utf8_ok, bool force_big, uint32_t *zero_next,
                     hipStream_t s);
