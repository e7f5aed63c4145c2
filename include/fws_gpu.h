/*
 * fws_gpu.h -- C ABI of flashws_amd: the MI355X (gfx950) receive-path frame
 * decode of flashws (RFC 6455 §5.2 header parse + 4-byte-key XOR unmask).
 *
 * Pure C. No HIP or torch types in the signatures: device memory is `void *`,
 * streams are `void *` (a hipStream_t, NULL = the null stream). Every entry
 * point returns an int status (0 = ok, negative = error, table below); none
 * throws, none frees caller memory, none synchronises the stream unless its
 * comment says so.
 *
 * Reference interfaces replaced (paths relative to flashws include/flashws/):
 *   seam 1  fws::WSMaskBytesFast(uint8_t*, size_t, uint32_t)  crypto/ws_mask.h:175-197
 *           -> fws_gpu_mask / fws_gpu_unmask_batch
 *   seam 2  WSocket<D, is_server, tls>::OnRecvData(IOBuffer&) net/w_socket.h:543-769
 *           (its ParseFrameHdr net/w_socket.h:435-524 and RX state :223-245)
 *           -> fws_gpu_decode_stream (device-resident batch)
 *           -> fws_rx_session_* (host buffers, same on_read() event contract)
 * The reference-side binding a maintainer adds is in INTEGRATION.md.
 */
#ifndef FWS_GPU_H
#define FWS_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FWS_GPU_ABI_VERSION 1

/* ---- status codes ------------------------------------------------------
 * Protocol errors keep the reference's ParseFrameHdr return values
 * (w_socket.h:451-521) so callers can forward them unchanged to
 * WSServerSocket's Close(WS_ABNORMAL_CLOSE, ...) (ws_server_socket.h:176-181). */
enum {
    FWS_OK = 0,
    FWS_ERR_RSV = -1,           /* RSV1-3 set                 w_socket.h:466-470 */
    FWS_ERR_TOO_LARGE = -2,     /* payload_len > 2^32         w_socket.h:493-498 */
    FWS_ERR_NOT_MASKED = -3,    /* server RX, MASK bit clear  w_socket.h:513-515 */
    FWS_ERR_MASKED = -4,        /* client RX, MASK bit set    w_socket.h:518-521 */
    FWS_ERR_OPCODE = -9,        /* opcode not 0-2/8-10        w_socket.h:451-454 */
    FWS_ERR_CONTROL_FRAME = -10,/* host RX session: control frame with payload > 125 B
                                   (RFC 6455 §5.5). The reference does not check
                                   (only a debug FWS_ASSERT, w_socket.h:654) and overflows
                                   its control buffer; the session refuses the frame. */
    FWS_ERR_CAPACITY = -20,     /* an output array is too small (count still reported) */
    FWS_ERR_INVALID = -21,      /* bad argument / not initialised */
    FWS_ERR_NO_DEVICE = -22,    /* no gfx950 device visible */
    FWS_ERR_INTERNAL = -23,     /* device-side failure (decode grid barrier timed out) */
    FWS_ERR_HIP_BASE = -1000    /* -1000 - hipError_t */
};

/* ---- descriptor-mode unmask --------------------------------------------
 * One payload region to unmask in place. Byte i of the region is XORed with
 * key byte ((phase + i) & 3), key = the 4 wire key bytes loaded as a native
 * little-endian uint32 (w_socket.h:504; ws_mask.h:17-28). Continuing a frame
 * at payload offset k is phase = k & 3, the same as the reference's
 * RotateR(key, 8 * (k & 3)) (w_socket.h:756-759). Regions of one batch must
 * not overlap; they may be in any order and any alignment. */
typedef struct fws_frame_desc {
    uint64_t payload_off;   /* byte offset from the batch's device base */
    uint64_t payload_len;   /* bytes to unmask (0 allowed) */
    uint32_t key;
    uint32_t phase;         /* 0..3 */
} fws_frame_desc;           /* 24 bytes */

/* ---- stream decode output ------------------------------------------------
 * One parsed frame of a server-side (client-masked) byte stream. */
typedef struct fws_frame_info {
    uint64_t hdr_off;       /* offset of the frame's first header byte */
    uint64_t payload_len;   /* length field from the header (w_socket.h:473-492) */
    uint32_t key;           /* mask key, native LE u32 of the wire bytes */
    uint8_t opcode;         /* raw opcode of this frame (0 = continuation) */
    uint8_t fin;
    uint8_t hdr_len;        /* 6, 8 or 14 */
    uint8_t flags;          /* FWS_FRAME_TRUNCATED: payload runs past the stream end */
} fws_frame_info;           /* 24 bytes */

#define FWS_FRAME_TRUNCATED 1u

/* Result of one fws_gpu_decode_stream call (written to device memory). */
typedef struct fws_decode_result {
    int32_t status;         /* FWS_OK or the first protocol error on the stream */
    uint32_t n_frames;      /* frames parsed (complete headers), also past capacity */
    uint64_t consumed;      /* bytes consumed: end of last frame part (== len unless a
                               partial header remains, or an error stopped the decode) */
    uint64_t err_off;       /* offset of the failing header when status < 0 */
    uint64_t carry_unread;  /* payload bytes of the last frame still to come */
    uint32_t carry_hdr_len; /* bytes of an incomplete trailing header (<= 13) */
    uint32_t n_survivors;   /* diagnostics: speculative header candidates kept */
} fws_decode_result;        /* 40 bytes */

typedef struct fws_gpu_ctx fws_gpu_ctx;

int fws_gpu_abi_version(void);
int fws_gpu_device_count(int *count);

/* A context owns the device workspace of one device and is used from one
 * host thread at a time (one context per stream/thread; the reference is one
 * FLoop per thread, floop.h:331-345). */
int fws_gpu_ctx_create(int device, fws_gpu_ctx **out);
void fws_gpu_ctx_destroy(fws_gpu_ctx *ctx);
/* Pre-size the workspace so later calls never allocate (hipGraph-capturable). */
int fws_gpu_ctx_reserve(fws_gpu_ctx *ctx, uint64_t max_frames, uint64_t max_stream_bytes);
/* Persistent receive decode (r05): with workers > 0, the small reads of the
 * context's fws_rx_session / fws_rx_mux calls (reads of <= 128 KiB in pinned
 * or registered host memory, the per-read and per-loop-step hot path of
 * OnRecvData, w_socket.h:543-769) are decoded by a resident grid of `workers`
 * workgroups (+ one poller) that the context launches on first use and that
 * exits by itself after ~250 us without a read -- no kernel launch per read
 * while reads keep coming. 0 (the default) = a launch per read. The grid holds
 * `workers` CUs' LDS and one hardware queue while it is resident. On a device
 * with a large BAR the grid polls a mailbox in device memory that the CPU
 * writes, and a session read of <= 16 KiB is copied there by the CPU with its
 * doorbell (push mode; FWS_RX_PUSH=0 in the environment keeps every read a
 * device-side pull over PCIe). Results are the same either way. */
int fws_gpu_ctx_set_rx_persistent(fws_gpu_ctx *ctx, uint32_t workers);

/* seam 1 -- device twin of WSMaskBytesFast (ws_mask.h:175): XOR n bytes at
 * dev_ptr with key, in place, on `stream`. Any alignment, any n. */
int fws_gpu_mask(void *dev_ptr, uint64_t n, uint32_t key, void *stream);

/* Descriptor-mode batch unmask: every region of dev_descs[0..n) (device
 * memory) inside dev_base is unmasked in place. Load-balanced over 4 KiB
 * units, so one launch covers any mix of frame sizes. Regions must not
 * overlap; any order is accepted. When they are sorted by offset (a batch cut
 * from a wire stream) the run works in byte space: non-payload bytes that
 * share a 16-byte aligned chunk with payload bytes, between the batch's first
 * and last payload byte, are written back with their own value (no other
 * writer may change them during the call); bytes outside that span are never
 * written. A permuted batch is planned in chunk space (C2 permuted: 0.142 ms
 * against 0.091 sorted). */
int fws_gpu_unmask_batch(fws_gpu_ctx *ctx, void *dev_base, const fws_frame_desc *dev_descs,
                         uint32_t n, void *stream);

/* One-launch batch unmask for descriptors sorted by payload_off with
 * non-overlapping regions (payload_off_i + payload_len_i <= payload_off_i+1),
 * as a batch cut from a wire stream or fws_gpu_decode_stream's frame list
 * always is. Same result and the same byte-space write rule as
 * fws_gpu_unmask_batch, without its plan launch: each 4 KiB unit finds its
 * frames itself (interpolation guess, binary search on a miss). Unsorted or
 * overlapping descriptors are a contract violation: results are undefined
 * inside [first payload, last payload end), nothing outside it is written.
 * Replaces the per-frame WSMaskBytesFast calls (ws_mask.h:175) of
 * OnRecvData's frame loop (w_socket.h:586,614) for a whole batch. */
int fws_gpu_unmask_sorted(fws_gpu_ctx *ctx, void *dev_base, const fws_frame_desc *dev_descs,
                          uint32_t n, void *stream);

/* The sortedness contract of fws_gpu_unmask_sorted(_utf8), checked on the
 * device in one launch: *dev_bad (a device word) becomes the first i with
 * payload_off_i + payload_len_i > payload_off_i+1 (or an overflowing end), or
 * 0xFFFFFFFF when the batch is sorted and disjoint. With FWS_CHECK_SORTED=1
 * in the environment the sorted entry points run this check first and refuse
 * a violating batch with FWS_ERR_INVALID, writing nothing (a debug mode: it
 * synchronises the stream). */
int fws_gpu_check_sorted(fws_gpu_ctx *ctx, const fws_frame_desc *dev_descs, uint32_t n, uint32_t *dev_bad,
                         void *stream);

/* fws_gpu_unmask_sorted plus per-region UTF-8 validation of the unmasked
 * payloads in the same pass (BASELINE config 5 in descriptor mode):
 * dev_ok[i] = 1 iff region i is well-formed UTF-8 (Unicode Table 3-7), the
 * same flags as fws_gpu_unmask_sorted followed by fws_gpu_validate_utf8.
 * Same sortedness contract as fws_gpu_unmask_sorted. */
int fws_gpu_unmask_sorted_utf8(fws_gpu_ctx *ctx, void *dev_base, const fws_frame_desc *dev_descs, uint32_t n,
                               uint8_t *dev_ok, void *stream);

/* The two halves of fws_gpu_unmask_batch, for callers that reuse one plan
 * (same descriptors) across buffers: _plan builds the chunk plan of the
 * descriptors in ctx, _run unmasks with the last plan built in ctx. */
int fws_gpu_unmask_plan(fws_gpu_ctx *ctx, const void *dev_base, const fws_frame_desc *dev_descs,
                        uint32_t n, void *stream);
int fws_gpu_unmask_run(fws_gpu_ctx *ctx, void *dev_base, const fws_frame_desc *dev_descs,
                       uint32_t n, void *stream);

/* Same, out of place: dst[dst_off_i ..] = src[payload_off_i ..] ^ key, with
 * dst_off = exclusive prefix sum of payload_len (message reassembly, C4). */
int fws_gpu_unmask_gather(fws_gpu_ctx *ctx, void *dev_dst, const void *dev_src,
                          const fws_frame_desc *dev_descs, uint32_t n, void *stream);

/* seam 2 (device-resident) -- fused header parse + unmask of a server-side
 * wire stream dev_wire[0..len) that starts at a frame header. Payloads are
 * unmasked in place; frames are listed in dev_frames (capacity cap) and the
 * outcome in *dev_result (device memory). Semantics are OnRecvData's on one
 * buffer: decoding stops at the first protocol error (frames before it are
 * still unmasked), a truncated last payload is unmasked as far as present, an
 * incomplete trailing header is left for the next call. If dev_utf8_ok is
 * non-NULL, byte i of it is set to 1 iff frame i is TEXT (opcode 1), FIN,
 * complete, and its unmasked payload is well-formed UTF-8 (else 0). */
int fws_gpu_decode_stream(fws_gpu_ctx *ctx, void *dev_wire, uint64_t len,
                          fws_frame_info *dev_frames, uint32_t cap,
                          fws_decode_result *dev_result, uint8_t *dev_utf8_ok, void *stream);

/* ---- batched stream decode: many independent streams ----------------------
 * fws_gpu_decode_stream over a list of independent streams (the buffers of
 * many connections, or successive batches of one: FLoop's loop hands each
 * socket's bytes to its own OnRecvData, floop.h:661-703), with decodes kept
 * in flight on two HIP streams so one job's latency-bound resolve overlaps
 * another's streaming kernels. Each job's frames, result,
 * UTF-8 flags and unmasked bytes equal fws_gpu_decode_stream on that job
 * alone. Jobs must not share memory. The work is ordered after everything
 * already on `stream`, and `stream` waits for all of it (synchronise `stream`
 * to read results). An engine is used from one host thread at a time; it owns
 * its workspaces, sized by max_frames / max_stream_bytes per job (a larger job
 * grows them after draining the engine). */
typedef struct fws_decode_job {
    void *dev_wire;                 /* 16-B aligned, as fws_gpu_decode_stream */
    uint64_t len;
    fws_frame_info *dev_frames;
    uint32_t cap;
    uint32_t reserved;              /* 0 */
    fws_decode_result *dev_result;
    uint8_t *dev_utf8_ok;           /* optional (NULL) */
} fws_decode_job;                   /* 48 bytes */

typedef struct fws_decode_engine fws_decode_engine;
int fws_decode_engine_create(int device, uint64_t max_frames, uint64_t max_stream_bytes, fws_decode_engine **out);
void fws_decode_engine_destroy(fws_decode_engine *e);
int fws_decode_engine_run(fws_decode_engine *e, const fws_decode_job *jobs, uint32_t n, void *stream);

/* Per-frame UTF-8 validation of already-unmasked payloads (Unicode Table
 * 3-7): ok[i] = 1 iff region i is well-formed UTF-8. */
int fws_gpu_validate_utf8(fws_gpu_ctx *ctx, const void *dev_base, const fws_frame_desc *dev_descs,
                          uint32_t n, uint8_t *dev_ok, void *stream);

/* ---- host-buffer RX session: OnRecvData over the GPU ----------------------
 * Mirrors WSocket::OnRecvData (w_socket.h:543-769) for one server
 * connection: reads are host buffers, decode runs on the device, and the
 * on_read() contract (opcode, part, is_frame_end, is_msg_end, is_control) is
 * reported as an event array whose order and values match the reference.
 * Control frames: PING -> a PONG event (the caller sends the reply), CLOSE ->
 * a CLOSE event with status code; their payload bytes are copied to ctl_out. */
typedef struct fws_rx_event {
    uint32_t kind;          /* 0 ON_READ, 1 PONG_TO_SEND, 2 CLOSE_RECEIVED */
    uint32_t opcode;        /* reported opcode (continuations report the first frame's, w_socket.h:626) */
    uint8_t is_ctl;
    uint8_t frame_end;
    uint8_t msg_end;
    uint8_t fin;
    uint32_t code;          /* CLOSE status code (1005 if absent) */
    uint64_t size;          /* bytes in this part */
    uint64_t data_off;      /* ON_READ data part: offset of the part in the read buffer */
    uint64_t ctl_off;       /* control payload copy offset in ctl_out */
    uint64_t capacity;      /* IOBuffer capacity of the view, relative to the read start */
} fws_rx_event;             /* 48 bytes */

/* Carried RX state of a session (w_socket.h:223-245), for inspection. */
typedef struct fws_rx_state {
    int32_t recv_status;    /* 0 WAIT_FRAME_HEAD, 1 WAIT_FRAME_PAYLOAD */
    uint32_t mask_key;      /* last_rx_mask_key_, rotated for the next payload byte */
    uint64_t unread_pl_len;
    uint8_t last_rx_opcode;
    uint8_t last_rx_control_opcode;
    uint8_t last_rx_fin_flag;
    uint8_t is_rx_control_frame;
    uint32_t last_rx_hdr_part_len;
} fws_rx_state;             /* 24 bytes */

typedef struct fws_rx_session fws_rx_session;

int fws_rx_session_create(fws_gpu_ctx *ctx, int is_server, fws_rx_session **out);
void fws_rx_session_destroy(fws_rx_session *s);
/* Decode one read in place (buf is host memory, unmasked on return). Returns
 * 0 or the reference's negative ParseFrameHdr code. buf_capacity: the view's
 * capacity measured from buf (the last part's IOBuffer capacity). */
int fws_rx_session_feed(fws_rx_session *s, uint8_t *buf, uint64_t size, uint64_t buf_capacity,
                        fws_rx_event *events, uint64_t ev_cap, uint64_t *n_events,
                        uint8_t *ctl_out, uint64_t ctl_cap, uint64_t *ctl_used);
int fws_rx_session_state(const fws_rx_session *s, fws_rx_state *out);
/* fws_rx_session_feed with the session's own event and control-payload sinks
 * (grown as needed, no capacity error): *events / *ctl point into the session
 * and stay valid until its next feed. */
int fws_rx_session_feed_view(fws_rx_session *s, uint8_t *buf, uint64_t size, uint64_t buf_capacity,
                             const fws_rx_event **events, uint64_t *n_events, const uint8_t **ctl,
                             uint64_t *ctl_used);
/* The last feed's protocol error (0 if none) and the opcode of the frame it
 * stopped at, for the reference's error text ("Opcode %u is not valid",
 * w_socket.h:452) in the Close reason (ws_server_socket.h:178-181). */
int fws_rx_session_error(const fws_rx_session *s, uint32_t *opcode);

/* ---- many connections, one round trip -----------------
 * FLoop::OneStep (floop.h:661-703) drains every readable socket in one loop
 * iteration and runs each read through its socket's OnRecvData. fws_rx_mux
 * keeps one RX state per connection (the fws_rx_session of each) and decodes
 * the reads of many connections -- each with its own carried state: staged
 * header bytes, unread payload of the frame in progress, rotated key -- with
 * one pinned staging pass, one H2D copy, one launch (one workgroup per read)
 * and one D2H copy, then replays each connection's OnRecvData bookkeeping.
 * Per read the results equal fws_rx_session_feed on that connection alone.
 * A read over 256 KiB, or whose header stream needs the parallel decode (over
 * 128 KiB or 256 headers), goes through that connection's session path. */
typedef struct fws_rx_mux fws_rx_mux;
typedef struct fws_rx_read {
    uint32_t conn;          /* connection slot, < n_conns; at most one read per slot per call */
    uint32_t flags;         /* 0 */
    uint8_t *buf;           /* host memory, unmasked in place */
    uint64_t size;
    uint64_t capacity;      /* the view's capacity from buf (fws_rx_session_feed) */
} fws_rx_read;
typedef struct fws_rx_read_result {
    int32_t ret;            /* fws_rx_session_feed's return for this read */
    uint32_t pad;
    const fws_rx_event *events;   /* the connection's events, valid until its next feed */
    uint64_t n_events;
    const uint8_t *ctl;           /* control payloads the events point into */
    uint64_t ctl_used;
} fws_rx_read_result;
int fws_rx_mux_create(fws_gpu_ctx *ctx, uint32_t n_conns, fws_rx_mux **out);
void fws_rx_mux_destroy(fws_rx_mux *m);
/* slot `conn` starts a new connection (the reference's initial RX state) */
int fws_rx_mux_reset(fws_rx_mux *m, uint32_t conn);
int fws_rx_mux_state(const fws_rx_mux *m, uint32_t conn, fws_rx_state *out);
int fws_rx_mux_error(const fws_rx_mux *m, uint32_t conn, uint32_t *opcode);
/* Decode n reads (distinct connections). Returns 0 (per-read codes in
 * results[i].ret) or FWS_ERR_INVALID / a HIP error for the call itself. */
int fws_rx_mux_feed(fws_rx_mux *m, const fws_rx_read *reads, uint32_t n, fws_rx_read_result *results);
/* fws_rx_mux_feed in two halves, so the host can go on (read more sockets,
 * dispatch an earlier batch's events) while the GPU decodes: submit stages and
 * starts the batch and returns; complete waits for it and fills results[0, n)
 * exactly as feed would. One batch at a time: submit again only after
 * complete. Until complete returns the reads' buffers belong to the mux
 * (unmasked in place), and the connections' state is the state before the
 * batch. Other GPU calls of the context may be made in between (a request of
 * the context's persistent receive decode waits for the batch first). */
int fws_rx_mux_submit(fws_rx_mux *m, const fws_rx_read *reads, uint32_t n);
int fws_rx_mux_complete(fws_rx_mux *m, fws_rx_read_result *results);
/* Non-blocking: 1 when fws_rx_mux_complete would not wait (the submitted
 * batch has decoded, or none is in flight), 0 while it decodes, < 0 on a HIP
 * error. The batched hook's deferred completion polls it (gpu_floop.hpp). */
int fws_rx_mux_ready(fws_rx_mux *m);

/* ---- send path: batch frame builder -------------------
 * The bytes WSocket::SendFrame (w_socket.h:832-944) writes for one frame:
 * b0 = FIN << 7 | opcode, b1 = MASK << 7 | len7, the BE 16 / 64-bit length,
 * for a client frame the key (native LE u32 of the wire bytes) and the payload
 * XORed with it from phase 0 (w_socket.h:858-866). The reference draws the key
 * from SemiSecureRand32 (w_socket.h:860); here the caller supplies it. */
typedef struct fws_tx_desc {
    uint64_t src_off;       /* payload bytes at dev_src + src_off */
    uint64_t len;           /* payload length */
    uint32_t key;           /* mask key (masked frames) */
    uint8_t opcode;         /* wire opcode: 0 continuation, 1 TEXT, 2 BIN, 8 CLOSE, 9 PING, 10 PONG */
    uint8_t fin;
    uint8_t masked;         /* 1: client frame (MASK bit + key + masked payload); 0: server frame */
    uint8_t pad;
} fws_tx_desc;              /* 24 bytes */

/* Opcode and FIN of a connection's next frame by SendFrame's rule
 * (w_socket.h:845-848, 903-913): a data frame that continues an unfinished
 * message is a continuation; control frames neither use nor change the state.
 * frame_type: WSTxFrameType (1 TEXT, 2 BIN, 8 CLOSE, 9 PING, 10 PONG). Host code. */
void fws_tx_next(uint32_t frame_type, int last_frame_if_possible, uint8_t *last_msg_not_fin, uint8_t *opcode,
                 uint8_t *fin);

/* dev_out (16-B aligned) = the frames of dev_descs[0..n) back to back;
 * *dev_out_len (device u64) = their total size, or ~0 if it exceeds out_cap.
 * The default form (plan + encode: k_out_plan, k_tx_encode_w5) writes nothing
 * when the total exceeds out_cap. The opt-in one-launch tuning form (k_tx_one,
 * fws_internal_set_tx_one; measured slower) never writes a
 * byte at or past out_cap, but writes the frames that fit below it. */
int fws_gpu_encode_frames(fws_gpu_ctx *ctx, void *dev_out, uint64_t out_cap, const void *dev_src,
                          const fws_tx_desc *dev_descs, uint32_t n, uint64_t *dev_out_len, void *stream);

/* Host-memory send for one connection: WSocket::SendFrame (w_socket.h:832-944)
 * for its next n frames, in order. Frame i = payloads[i][0..lens[i]) of
 * WSTxFrameType frame_types[i] with last_frame_if_possible = last[i]; a client
 * session (is_server = 0) masks with keys[i] (the reference draws
 * SemiSecureRand32, w_socket.h:860; here the caller supplies it). The frames'
 * wire bytes, back to back, go to out; *out_len = their size. If out_cap is
 * too small: FWS_ERR_CAPACITY, *out_len = the size needed, nothing sent and
 * the sequencing state unchanged. Opcode / FIN sequencing (last_msg_not_fin_,
 * w_socket.h:903-913) is carried across calls. Synchronous; empty control
 * payloads are sent as empty frames (the reference dereferences a null
 * buffer there). */
typedef struct fws_tx_session fws_tx_session;
int fws_tx_session_create(fws_gpu_ctx *ctx, int is_server, fws_tx_session **out);
void fws_tx_session_destroy(fws_tx_session *s);
int fws_tx_session_send(fws_tx_session *s, const uint8_t *const *payloads, const uint64_t *lens,
                        const uint32_t *frame_types, const uint8_t *last, const uint32_t *keys, uint32_t n,
                        uint8_t *out, uint64_t out_cap, uint64_t *out_len);
int fws_tx_session_state(const fws_tx_session *s, uint8_t *last_msg_not_fin);

/* ---- batched, pipelined receive over host memory ---------------------------
 * the reads of one event-loop step (FLoop::OneStep,
 * floop.h:661-703; TCPSocket::Read, tcp_socket.h:387-402) aggregated into one
 * host batch per submit. Each of `depth` slots runs H2D -> decode (header parse
 * + unmask, optional per-frame UTF-8 flags) -> D2H of the unmasked bytes (back
 * into the batch), the frame list and the result on its own stream, so
 * successive batches overlap on the full-duplex link. The batch must stay
 * valid (and should be pinned) until its wait returns; a batch starts at a
 * frame header (the per-connection carry is the session's job). */
typedef struct fws_rx_pipe fws_rx_pipe;

/* Pin / unpin caller memory (e.g. MemPool blocks, flash_alloc.h:44-73) for async copies. */
int fws_gpu_host_register(void *host_ptr, uint64_t bytes);
int fws_gpu_host_unregister(void *host_ptr);

int fws_rx_pipe_create(int device, uint64_t max_batch_bytes, uint32_t max_frames, uint32_t depth, int utf8,
                       fws_rx_pipe **out);
void fws_rx_pipe_destroy(fws_rx_pipe *p);
/* Enqueue a batch; *ticket identifies it. Waits first if its slot is still busy. */
int fws_rx_pipe_submit(fws_rx_pipe *p, uint8_t *batch, uint64_t len, uint64_t *ticket);
/* Block until batch `ticket` is done: the batch holds the unmasked bytes, *frames
 * points at min(n_frames, max_frames) decoded frames (pinned, valid until the
 * slot is reused `depth` submits later), *result is the decode result, and
 * *utf8_ok the per-frame flags (pipes created with utf8 != 0). */
int fws_rx_pipe_wait(fws_rx_pipe *p, uint64_t ticket, const fws_frame_info **frames, uint64_t *n_frames,
                     fws_decode_result *result, const uint8_t **utf8_ok);

/* ---- synthetic workloads (BASELINE configs, not test oracles) ------------ */
typedef struct fws_gen_params {
    uint64_t seed;
    uint32_t kind;          /* 0 fixed-size frames, 1 log-uniform sizes, 2 fragmented message, 3 UTF-8 text */
    uint32_t opcode;        /* data opcode for kinds 0/1 (1 TEXT, 2 BIN) */
    uint64_t n_frames;      /* kinds 0/3: frame count */
    uint64_t payload_min;   /* kind 0/3: the payload size; kinds 1/2: minimum */
    uint64_t payload_max;   /* kinds 1/2: maximum (log-uniform in [min, max]) */
    uint64_t target_bytes;  /* kinds 1/2: stop once the payload total reaches this */
    uint32_t invalid_permille; /* kind 3: frames carrying one invalid UTF-8 sequence */
    uint32_t pad_;
} fws_gen_params;

/* Two-call protocol: with wire == NULL only *wire_len and *n_frames are
 * computed. Otherwise fills wire (cap bytes, host memory) with client-masked
 * frames and descs (payload regions, phase 0) and, for kind 3, utf8_ok
 * (expected per-frame validity). */
int fws_gen_batch(const fws_gen_params *p, uint8_t *wire, uint64_t cap, uint64_t *wire_len,
                  fws_frame_desc *descs, uint64_t descs_cap, uint64_t *n_frames, uint8_t *utf8_ok);

#ifdef __cplusplus
}
#endif
#endif /* FWS_GPU_H */
