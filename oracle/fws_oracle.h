/*
 * fws_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of flashws's receive-path frame decode (RFC 6455 §5.2 header
 * parse + 4-byte-key XOR unmask), used as the parity checker for the HIP path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this; the product path (flashws_amd/) never links or calls it.
 *
 * Parity: pinned. tests/golden/ fixtures were produced by the real reference
 * (oracle/ref_driver.cpp compiled against /root/reference/include, driving
 * WSocket::OnRecvData) and tests/test_oracle_golden.py checks this restatement
 * against every one of them byte-for-byte.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the flashws tree, include/flashws/...).
 */
#ifndef FWS_ORACLE_H
#define FWS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- a5: RotateR  (base/constexpr_math.h:67-82) ---- */
uint32_t orc_rotr32(uint32_t v, uint32_t b);

/* ---- a1..a4: XOR unmask variants (crypto/ws_mask.h) ---- */
void orc_mask1(uint8_t *src, size_t n, uint32_t key);            /* ws_mask.h:32-43  */
void orc_ws_mask_bytes(uint8_t *src, size_t n, uint32_t key);    /* ws_mask.h:15-29  */
void orc_mask_avx2(uint8_t *src, size_t n, uint32_t key);        /* ws_mask.h:52-91  */
void orc_mask_large_chunk_avx2(uint8_t *src, size_t n, uint32_t key); /* ws_mask.h:96-166 */
void orc_ws_mask_fast(uint8_t *src, size_t n, uint32_t key);     /* ws_mask.h:175-197 (GCC dispatch) */

/* ---- a6: ParseFrameHdr  (net/w_socket.h:435-524) ---- */
enum {
    ORC_ERR_RSV = -1,          /* w_socket.h:466-470 */
    ORC_ERR_TOO_LARGE = -2,    /* w_socket.h:493-498 */
    ORC_ERR_NOT_MASKED = -3,   /* w_socket.h:513-515 (server) */
    ORC_ERR_MASKED = -4,       /* w_socket.h:518-521 (client) */
    ORC_ERR_OPCODE = -9        /* w_socket.h:451-454 */
};

/* ---- a8: RX state (net/w_socket.h:223-245) + the control buffer buf_ ---- */
typedef struct orc_rx_state {
    int32_t recv_status;            /* 0 WAIT_FRAME_HEAD, 1 WAIT_FRAME_PAYLOAD */
    uint32_t last_rx_mask_key;
    uint64_t unread_pl_len;
    uint8_t last_rx_opcode;
    uint8_t last_rx_control_opcode;
    uint8_t last_rx_fin_flag;
    uint8_t is_rx_control_frame;
    uint32_t last_rx_hdr_part_len;
    uint8_t rx_ws_hdr_buf[14];
    /* buf_ (control payload staging, w_socket.h:637-658) */
    uint8_t ctl_buf[128];
    uint32_t ctl_size;
    uint8_t ctl_allocated;
    uint8_t is_server;
    uint8_t pad_[2];
} orc_rx_state;

void orc_rx_init(orc_rx_state *st, int is_server);

/* One parse of up to 14 staged header bytes. Returns header length, 0 if
 * incomplete, or a negative ORC_ERR_* (w_socket.h:435-524). Updates the
 * control/opcode bookkeeping in st exactly as the reference member does. */
int orc_parse_frame_hdr(orc_rx_state *st, const uint8_t *data, const uint8_t *data_end,
                        uint32_t *opcode, uint32_t *fin, int *is_control, int *is_masked,
                        uint32_t *mask_key, uint64_t *payload_len);

/* Event emitted by orc_on_recv_data. kind:
 *   0 ON_READ   : user on_read() delivery (data part, or PONG)  w_socket.h:713-747
 *   1 PONG_SENT : a PING completed; the server replies PONG with ctl bytes  w_socket.h:662-666
 *   2 CLOSE_RECV: a CLOSE completed; status + reason in ctl bytes           w_socket.h:667-710
 *   3 FRAME_HDR : a header was parsed (frame bookkeeping, not a reference callback)
 */
typedef struct orc_event {
    uint32_t kind;
    uint32_t opcode;
    uint8_t is_ctl;
    uint8_t frame_end;
    uint8_t msg_end;
    uint8_t fin;
    uint32_t key;           /* FRAME_HDR: mask key; CLOSE_RECV: status code */
    uint64_t size;          /* bytes delivered (ON_READ) / payload_len (FRAME_HDR) */
    uint64_t data_off;      /* offset of the delivered bytes (or header) in the read buffer */
    uint64_t ctl_off;       /* offset into ctl_out for PONG/PING/CLOSE payload copies */
    uint64_t capacity;      /* IOBuffer capacity of the delivered view, relative to buffer start */
} orc_event;

/* a7: OnRecvData (w_socket.h:543-769). buf is the read's payload region
 * (IOBuffer data+start_pos .. +size); it is unmasked in place. buf_capacity is
 * the view's capacity measured from buf (the reference measures from data+0;
 * callers compare relative values). Returns 0 or a negative ORC_ERR_*.
 * Events beyond ev_cap / ctl bytes beyond ctl_cap are dropped but counted. */
int orc_on_recv_data(orc_rx_state *st, uint8_t *buf, size_t size, size_t buf_capacity,
                     orc_event *ev, size_t ev_cap, size_t *n_ev,
                     uint8_t *ctl_out, size_t ctl_cap, size_t *ctl_used);

/* Whole-stream convenience used by the large-size parity tests: decode a
 * complete server-side stream in place, listing every frame header.
 * frames[i] = {hdr_off, payload_len, key, opcode|fin<<8|hdr_len<<16}.
 * Returns 0, or a negative code with *err_off = offset of the failing header.
 * *n_frames counts every parsed frame even when frames_cap is exceeded. */
typedef struct orc_frame {
    uint64_t hdr_off;
    uint64_t payload_len;
    uint32_t key;
    uint8_t opcode;
    uint8_t fin;
    uint8_t hdr_len;
    uint8_t pad_;
} orc_frame;

int orc_decode_stream(uint8_t *buf, size_t size, orc_frame *frames, size_t frames_cap,
                      size_t *n_frames, size_t *err_off, size_t *consumed);

/* C4 (parity anchored on the user-level copy in tests/new-ws-echo/test_ws_server.cpp:205-206):
 * concatenation of the on_read() data parts, in order. Returns bytes written. */
size_t orc_reassemble(const uint8_t *unmasked, const orc_frame *frames, size_t n_frames,
                      uint8_t *out);

/* C5: strict UTF-8 (Unicode Table 3-7 / RFC 3629). Not in the reference
 * (w_socket.h:41 defines 1007 but never checks) -> parity unpinned by the
 * reference; cross-checked against Python's strict decoder in tests. */
int orc_utf8_valid(const uint8_t *s, size_t n);

/* ---- client / server TX ----------------------------------
 * w_socket.h:49-65 GetTxWSFrameHdrSize: 2 + (client ? 4 : 0) + (0 | 2 | 8). */
size_t orc_tx_hdr_size(size_t payload, int is_server);
/* w_socket.h:832-944 SendFrame, the bytes it writes: b0 = FIN << 7 | opcode,
 * where a data frame continuing an unfinished message carries opcode 0
 * (last_msg_not_fin_, :903-913; control frames neither use nor change it);
 * b1 = MASK << 7 | len7, then the BE 16 / 64-bit length, then (client) the key
 * as its native LE bytes (:862-866) and the payload masked with it
 * (WSMaskBytesFast, :861). The reference draws the key from SemiSecureRand32
 * (:860); here it is an argument. Writes hdr + n bytes to out, returns that. */
typedef struct orc_tx_state {
    int last_msg_not_fin;
} orc_tx_state;
size_t orc_tx_frame(orc_tx_state *st, int is_server, const uint8_t *payload, size_t n, uint32_t frame_type,
                    int last_frame_if_possible, uint32_t key, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif
