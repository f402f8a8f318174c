/*
 * xyws.h — C-ABI of the MI355X (gfx950) WebSocket frame-decode path.
 *
 * This is the drop-in boundary that replaces the CPU hot path of xynet's
 * WebSocket layer (paths relative to the xynet reference tree):
 *
 *   reference symbol                                         replaced by
 *   -------------------------------------------------------  ---------------------------
 *   websocket_mask(R&&, uint32_t mask, size_t i) -> size_t   xyws_unmask
 *     include/xynet/http/websocket_frame_mask.h:6-25
 *   websocket_frame_header_parser::parse / result / reset    xyws_decode_stream (parse
 *     include/xynet/http/websocket_frame_header.h:226-385      state carried in xyws_carry)
 *   websocket_recv_data: parse -> result -> websocket_mask   xyws_decode_stream,
 *     example/include/common/websocket.h:110-134               xyws_decode_indexed
 *   enum class websocket_flags                               XYWS_FLAG_* (same encoding)
 *     include/xynet/http/websocket_frame_header.h:42-58
 *
 * The reference has no FFI of its own: it is a header-only C++20 library whose
 * templates are instantiated in the caller's translation unit. A caller (an
 * io_uring/coroutine service in the xynet style) keeps its sockets and
 * buffer_sequence unchanged and hands device-resident recv buffers to these
 * entry points; see INTEGRATION.md for the binding a maintainer would add.
 *
 * Conventions
 *   - Plain C types only. Device pointers are void* / typed pointers into
 *     device memory (hipMalloc or equivalent); `stream` is a hipStream_t passed
 *     as void* (NULL = the legacy default stream).
 *   - Every call is asynchronous on `stream` and returns an int status
 *     (XYWS_OK or a negative XYWS_ERR_*). Device-side results (frame tables,
 *     frame counts, carries) are valid once the stream reaches the call.
 *   - Buffers are owned by the caller. Unmasking mutates the caller's buffer in
 *     place, exactly like websocket_mask (websocket_frame_mask.h:16). The
 *     context owns only its scratch (tile status records, frame tables).
 *   - Parse semantics are the reference's, bit for bit: nothing is rejected
 *     (RSV bits, reserved opcodes, non-minimal or 2^63+ lengths are accepted,
 *     websocket_frame_header.h:305-385); violations are only *reported* in
 *     xyws_frame.status. An unmasked frame has key 0 (the parser's m_mask after
 *     reset(), :274-281), so its payload is left unchanged.
 *   - No CPU fallback: every entry point that computes runs HIP kernels for
 *     gfx950; if no device is present the call fails with XYWS_ERR_HIP.
 */
#ifndef XYWS_H
#define XYWS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XYWS_ABI_VERSION 1

/* ---- status codes -------------------------------------------------------- */
#define XYWS_OK              0
#define XYWS_ERR_INVALID    -1  /* bad argument (null ctx, misaligned length, ...) */
#define XYWS_ERR_HIP        -2  /* a HIP runtime call failed (no device, launch error) */
#define XYWS_ERR_NOMEM      -3  /* device scratch allocation failed */
#define XYWS_ERR_CAPACITY   -4  /* batch larger than xyws_ctx_reserve() allowed while capturing */
#define XYWS_ERR_DEVICE     -5  /* a device-side bound tripped (see xyws_ctx_last_device_error) */

/* ---- websocket_flags encoding (websocket_frame_header.h:42-58) ----------- */
#define XYWS_FLAG_OP_CONTINUE 0x00
#define XYWS_FLAG_OP_TEXT     0x01
#define XYWS_FLAG_OP_BINARY   0x02
#define XYWS_FLAG_OP_CLOSE    0x08
#define XYWS_FLAG_OP_PING     0x09
#define XYWS_FLAG_OP_PONG     0x0A
#define XYWS_FLAG_OP_MASK     0x0F
#define XYWS_FLAG_FIN         0x10
#define XYWS_FLAG_HAS_MASK    0x20

/* Largest header: calc_frame_header_size(WS_HAS_MASK, UINT32_MAX)
 * (websocket_frame_header.h:111-134). */
#define XYWS_MAX_FRAME_HEADER_SIZE 14

/* ---- per-frame status bits (informational; never change the output) ----- */
#define XYWS_ST_PAYLOAD_INCOMPLETE 0x01 /* payload runs past the batch end (continues in carry) */
#define XYWS_ST_RSV                0x02 /* RSV1..3 set (parser drops them, :315) */
#define XYWS_ST_RESERVED_OPCODE    0x04 /* opcode 3-7 or 11-15 */
#define XYWS_ST_NONMINIMAL_LENGTH  0x08 /* 126/127 form used for a length that fits a shorter form */
#define XYWS_ST_LENGTH_MSB         0x10 /* 64-bit length with the most significant bit set */
#define XYWS_ST_BAD_CONTROL        0x20 /* control frame (opcode >= 8) with FIN=0 or length > 125 */
#define XYWS_ST_UNMASKED           0x40 /* MASK bit clear (client frames must be masked) */
#define XYWS_ST_OVERLAP            0x80 /* indexed mode: frame overlaps the next caller-supplied start;
                                           its unmask is clipped at that start */

/* ---- decode options ----------------------------------------------------- */
#define XYWS_OPT_PARSE_ONLY     0x1u /* build the frame table, leave payload bytes untouched */
#define XYWS_OPT_UNMASKED_HINT  0x2u /* stream mode: speculate on server->client (MASK=0) framing */
#define XYWS_OPT_SERIAL_SCAN    0x4u /* stream mode: one-lane serial boundary chase (debug/reference
                                        shape; exact, slow). Default is the fused tile kernel. */

/* One decoded frame. 32 bytes, naturally aligned; written to device memory. */
typedef struct xyws_frame {
  int64_t  frame_off;   /* header byte 0 relative to the batch start (< 0: header began in
                           an earlier batch and was completed from xyws_carry.hdr)        */
  int64_t  payload_off; /* payload byte 0 relative to the batch start                      */
  uint64_t payload_len; /* raw parsed length (websocket_frame_header_parser::length())    */
  uint8_t  key[4];      /* masking key, wire order (== bytes of mask_uint32_t(), :259-262) */
  uint8_t  flags;       /* websocket_flags: opcode | FIN 0x10 | HAS_MASK 0x20             */
  uint8_t  hdr_len;     /* 2..14: value parse() returns when fed from the frame start     */
  uint8_t  status;      /* XYWS_ST_* bits                                                  */
  uint8_t  reserved;
} xyws_frame;

/*
 * Decoder state carried across batch boundaries — the device-side analogue of
 * websocket_mask's returned phase `i` (websocket_frame_mask.h:14,24) and of the
 * parser's incremental npos protocol (websocket_frame_header.h:230,383-384).
 * A byte stream split at ANY point into consecutive batches decodes to the same
 * bytes and the same frames as the unsplit stream. A zero-filled carry is the
 * state at a frame boundary (a fresh parser).
 */
typedef struct xyws_carry {
  uint64_t payload_remaining; /* payload bytes of the open frame not yet seen (0 = at a boundary) */
  uint64_t phase;             /* websocket_mask phase for the next payload byte of the open frame */
  uint64_t frames_total;      /* frames whose header completed in all earlier batches             */
  uint8_t  key[4];            /* key of the open frame (wire order)                               */
  uint8_t  hdr_len;           /* bytes of an incomplete header held in hdr[] (0..13)              */
  uint8_t  hdr[14];           /* the incomplete header's bytes                                    */
  uint8_t  reserved[21];
} xyws_carry;                 /* 64 bytes */

typedef struct xyws_ctx xyws_ctx;

/* ---- library / context --------------------------------------------------- */
int         xyws_abi_version(void);
const char* xyws_strerror(int code);

/* Bind a context to HIP device `device`. One context per (thread, device). */
int xyws_ctx_create(int device, xyws_ctx** out);
int xyws_ctx_destroy(xyws_ctx* ctx);
/* Pre-size scratch for batches up to `max_batch_bytes` (and, for indexed mode,
 * `max_frames` caller starts) so that later calls allocate nothing and can be
 * captured into a hipGraph. Calls on larger batches grow scratch lazily. */
int xyws_ctx_reserve(xyws_ctx* ctx, uint64_t max_batch_bytes, uint64_t max_frames);
/* Device-side error word of the last completed call (0 = none). Synchronizes
 * the context's device. */
int xyws_ctx_last_device_error(xyws_ctx* ctx, uint32_t* out);

/* ---- hot path ------------------------------------------------------------ */

/* websocket_mask (websocket_frame_mask.h:6-25) on device memory: in place,
 * dev[j] ^= key[(phase + j) % 4] for j in [0, len). *phase_out (host pointer,
 * nullable) receives phase + len, the reference's return value. */
int xyws_unmask(xyws_ctx* ctx, void* dev, uint64_t len, const uint8_t key[4],
                uint64_t phase, uint64_t* phase_out, void* stream);

/* Frames at caller-known offsets (ascending, non-overlapping) inside one
 * device buffer: parse each header as websocket_frame_header_parser::parse
 * does from a fresh parser, then unmask its payload in place (clipped to the
 * buffer). A header that does not fit in the buffer yields hdr_len = 0 and is
 * left untouched. `dev_frames` (nullable) receives n descriptors. */
int xyws_decode_indexed(xyws_ctx* ctx, void* dev_buf, uint64_t len,
                        const uint64_t* dev_starts, uint64_t n,
                        xyws_frame* dev_frames, uint32_t opts, void* stream);

/* Back-to-back frames in one device buffer, boundaries discovered on device:
 * the batched websocket_recv_data (websocket.h:110-134) without its caller
 * policy. Starting from `dev_carry_in` (nullable = fresh stream), every frame
 * is parsed with a fresh parser and its payload unmasked in place; a frame or
 * header cut by the batch end is continued through `dev_carry_out`
 * (nullable). Up to `cap` descriptors go to `dev_frames` (nullable); the frame
 * count (which may exceed cap) goes to `dev_nframes` (nullable). All
 * pointers except ctx are device pointers. dev_carry_in may equal
 * dev_carry_out. */
int xyws_decode_stream(xyws_ctx* ctx, void* dev_buf, uint64_t len,
                       const xyws_carry* dev_carry_in, xyws_carry* dev_carry_out,
                       xyws_frame* dev_frames, uint64_t cap, uint64_t* dev_nframes,
                       uint32_t opts, void* stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* XYWS_H */
