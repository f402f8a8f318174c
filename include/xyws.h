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
 *   websocket_frame_header_parser (incremental, one header)  xyws_parser_* (runs the stream
 *     include/xynet/http/websocket_frame_header.h:226-385      decoder in parse-only mode)
 *   detail::websocket_frame_header_builder                   xyws_header_build (one header),
 *     include/xynet/http/websocket_frame_header.h:136-175      xyws_encode_frames (batched, device)
 *   echo_once: header{FIN|TEXT, len} + send(header, data)    xyws_encode_frames
 *     example/websocket/websocket_echo.cpp:18-27
 *   websocket_check_parser_result (close policy)             xyws_classify_frames
 *     example/include/common/websocket.h:81-108
 *   (new) FIN=0 message reassembly + UTF-8 validation        xyws_reassemble
 *   recv_all / io_service remote-queue eventfd               xyws_arena_* (pinned recv arena,
 *     include/xynet/socket/impl/recv_all.h:86-121              H2D -> decode -> D2H, completion
 *     include/xynet/io_service.h:362-381                       written to an eventfd)
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

#define XYWS_ABI_VERSION 2

/* ---- status codes -------------------------------------------------------- */
#define XYWS_OK              0
#define XYWS_ERR_INVALID    -1  /* bad argument (null ctx, misaligned length, ...) */
#define XYWS_ERR_HIP        -2  /* a HIP runtime call failed (no device, launch error) */
#define XYWS_ERR_NOMEM      -3  /* device scratch allocation failed */
#define XYWS_ERR_CAPACITY   -4  /* batch larger than xyws_ctx_reserve() allowed while capturing */
#define XYWS_ERR_DEVICE     -5  /* a device-side bound tripped (see xyws_ctx_last_device_error) */
#define XYWS_ERR_AGAIN      -6  /* not complete yet (xyws_arena_poll) / no free slot (xyws_arena_submit) */

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
/* Pre-size scratch for batches up to `max_batch_bytes` (and, for indexed mode
 * and frame descriptors, `max_frames` frames) so that later calls allocate
 * nothing and can be captured into a hipGraph. The per-frame tables go to the
 * streams already used on the context and to one spare: the first stream new
 * to the context may be captured at once; a second new stream needs one
 * uncaptured call first (or XYWS_ERR_CAPACITY). Calls on larger batches grow
 * scratch lazily. */
int xyws_ctx_reserve(xyws_ctx* ctx, uint64_t max_batch_bytes, uint64_t max_frames);
/* The staging buffer of xyws_decode_stream_iov for sequences of up to
 * `max_total_bytes` in all, in the slots of the streams already used on the
 * context and in one spare (as xyws_ctx_reserve's per-frame tables): with
 * xyws_ctx_reserve(ctx, max_total_bytes, ...) before it, an iov decode that
 * fits allocates nothing and can be captured into a hipGraph. */
int xyws_ctx_reserve_iov(xyws_ctx* ctx, uint64_t max_total_bytes);
/* Device-side error word of the last completed call (0 = none). Synchronizes
 * the context's device. */
int xyws_ctx_last_device_error(xyws_ctx* ctx, uint32_t* out);

/* ---- hot path ------------------------------------------------------------ */

/* websocket_mask (websocket_frame_mask.h:6-25) on device memory: in place,
 * dev[j] ^= key[(phase + j) % 4] for j in [0, len). *phase_out (host pointer,
 * nullable) receives phase + len, the reference's return value. Eager calls
 * claim 64 KiB tiles from a counter in the stream's scratch slot (reset by
 * the launch itself); a call captured into a graph needs no reserve and
 * leaves no state outside its launch (static tiles), so its replays may run
 * on any stream, concurrently with each other. */
int xyws_unmask(xyws_ctx* ctx, void* dev, uint64_t len, const uint8_t key[4],
                uint64_t phase, uint64_t* phase_out, void* stream);

/* websocket_mask(R&& data, uint32_t mask, size_t i) with the reference's
 * contract (websocket_frame_mask.h:14, called by websocket_recv_data at
 * example/include/common/websocket.h:131): `data` is host or device memory,
 * and the bytes are unmasked when the call returns (it synchronizes
 * `stream`). Host bytes are staged through the context's device buffer (a
 * compatibility path: two copies per call); device bytes go to xyws_unmask.
 * Not allowed during stream capture (XYWS_ERR_CAPACITY). */
int xyws_mask_bytes(xyws_ctx* ctx, void* data, uint64_t len, const uint8_t key[4],
                    uint64_t phase, uint64_t* phase_out, void* stream);
/* xyws_mask_bytes refuses device memory of another device than ctx's
 * (XYWS_ERR_INVALID; xyws_unmask takes ctx's device memory only, unchecked:
 * no pointer query on the hot path). xyws_pointer_device: *device = the HIP device whose
 * memory `p` points into, or -1 for host memory (pinned, registered or
 * pageable); the shim uses it to pick the per-device context. */
int xyws_pointer_device(const void* p, int* device);

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

/* One piece of a buffer sequence: device memory. */
typedef struct xyws_iov {
  void*    base;
  uint64_t len;
} xyws_iov;
#define XYWS_IOV_MAX 64u
/* xyws_decode_stream over a buffer sequence — what one recv into a
 * multi-buffer `buffer_sequence` fills (include/xynet/buffer.h:94-110,
 * socket/impl/recv_all.h:99-121): the `niov` pieces (a HOST array of device
 * pieces, at most XYWS_IOV_MAX, any lengths and alignments, 0-length pieces
 * allowed) are ONE stream, decoded as if concatenated; every piece is
 * unmasked in place. Descriptor offsets count bytes across the pieces in
 * order (piece k starts at the sum of the earlier pieces' lengths). Three
 * launches whatever niov (gather into the stream's staging buffer, one
 * decode, scatter back); the staging buffer grows to the largest total seen
 * (XYWS_ERR_CAPACITY under capture before it has, or before
 * xyws_ctx_reserve_iov reserved it). XYWS_OPT_SERIAL_SCAN is refused
 * (XYWS_ERR_INVALID). */
int xyws_decode_stream_iov(xyws_ctx* ctx, const xyws_iov* iov, uint32_t niov,
                           const xyws_carry* dev_carry_in, xyws_carry* dev_carry_out,
                           xyws_frame* dev_frames, uint64_t cap, uint64_t* dev_nframes,
                           uint32_t opts, void* stream);


/* ==== ABI 2: the rest of the frame interface ============================ */

#define XYWS_NPOS UINT64_MAX /* websocket_frame_header_parser::npos (:230) */

/* ---- websocket_frame_header_parser (websocket_frame_header.h:226-385) ---
 * The reference's incremental one-header parser. parse() feeds `len` bytes
 * (host or device memory); *consumed receives the bytes consumed in THIS call
 * up to the end of the header, or XYWS_NPOS while the header is incomplete.
 * Once a header completed, further input returns XYWS_NPOS until reset()
 * (:378-384). The bytes are parsed on the device by the stream decoder in
 * parse-only mode with a device-resident carry; parse() is synchronous on
 * `stream` (it returns the reference's answer). result() before a header
 * completed returns what the reference's state machine holds at that point
 * (:305-385): flags from the first byte, HAS_MASK and the 7-bit length from
 * the second (0 for the 126/127 forms), the extended length accumulated over
 * the bytes received, the mask bytes received so far (checked against the
 * reference's parser corpus, tests/golden/parse_corpus.json). */
typedef struct xyws_parser xyws_parser;
int xyws_parser_create(xyws_ctx* ctx, xyws_parser** out);
int xyws_parser_destroy(xyws_parser* p);
int xyws_parser_reset(xyws_parser* p);
int xyws_parser_parse(xyws_parser* p, const void* data, uint64_t len, uint64_t* consumed, void* stream);
int xyws_parser_result(const xyws_parser* p, uint8_t* flags, uint8_t key[4], uint64_t* length);

/* ---- header build (detail::websocket_frame_header_builder, :136-175) ----
 * One header into out[14] (host memory, no device work); returns its length
 * H. With XYWS_FLAG_HAS_MASK the 4 key bytes are written only when `key` is
 * non-null, as the reference builder does (:168-173); with key == NULL they
 * are zero, which is what class websocket_frame_header's masked constructors
 * produce (:183-202). */
uint64_t xyws_header_build(uint8_t flags, const uint8_t* key, uint64_t len, uint8_t out[14]);

/* ---- batched encode on the device (echo replies, client-role frames) ----
 * For every frame i < n_eff (n_eff = min(n, *dev_n) when dev_n is given) of
 * a decoded frame table, writes a reply frame = header(flags_i, len_i) +
 * payload bytes dev_src[payload_off .. +payload_len) into dev_out, replies
 * back to back in frame order (the iovec pair echo_once sends, as one
 * buffer). flags_i = `flags`, or with XYWS_ENC_FRAME_OPCODE the frame's own
 * opcode and FIN (a ping answered as a pong) plus `flags`' HAS_MASK bit.
 * With HAS_MASK and dev_keys (4 bytes per frame, wire order) the header
 * carries key i and the payload is masked with it (client role); with
 * HAS_MASK and dev_keys == NULL the key bytes are zero (the reference
 * class's form) and the payload is copied unchanged. dev_verdicts (nullable,
 * from xyws_classify_frames) with `action_mask` (bit 1<<action) selects which
 * frames get a reply (others: none). dev_offsets (nullable) receives n_eff+1
 * reply offsets; *dev_out_len (nullable) the total reply bytes. Bytes past
 * out_cap are not written (compare *dev_out_len with out_cap); payload bytes
 * past src_len read as zero and set bit 0x100 of the device error word. */
#define XYWS_ENC_FRAME_OPCODE 0x1u
typedef struct xyws_verdict xyws_verdict;
int xyws_encode_frames(xyws_ctx* ctx, const void* dev_src, uint64_t src_len,
                       const xyws_frame* dev_frames, uint64_t n, const uint64_t* dev_n,
                       uint8_t flags, uint32_t enc_opts, const uint8_t* dev_keys,
                       const xyws_verdict* dev_verdicts, uint32_t action_mask,
                       void* dev_out, uint64_t out_cap, uint64_t* dev_offsets,
                       uint64_t* dev_out_len, void* stream);

/* ---- close policy per frame (websocket_check_parser_result) -------------
 * websocket.h:81-108 checks, in order: close frame -> 1000, FIN=0 -> 1003,
 * unmasked -> 1008, length > max -> 1009. Here without its opcode bug (the
 * bit-3 test `flags & WS_OP_CLOSE` there also closes on ping and pong):
 * pings and pongs are actions of their own. Policy bits relax or tighten the
 * reference's checks. *dev_first_close (nullable) receives the index of the
 * first frame with a close code, or UINT64_MAX. */
#define XYWS_ACT_DATA   0 /* text/binary/continuation frame to deliver */
#define XYWS_ACT_PING   1 /* answer with a pong carrying the same payload */
#define XYWS_ACT_PONG   2 /* unsolicited or answering pong: nothing to do */
#define XYWS_ACT_CLOSE  3 /* the connection closes with close_code */
#define XYWS_POL_FRAGMENTS  0x1u /* accept FIN=0 data frames (reassembly) instead of closing 1003 */
#define XYWS_POL_UNMASKED   0x2u /* accept unmasked frames instead of closing 1008 */
#define XYWS_POL_STRICT     0x4u /* RFC 6455 protocol errors (RSV, reserved opcode, fragmented or
                                    >125-byte control frame) close 1002 (the reference accepts them) */
#define XYWS_POL_REFERENCE  0x8u /* the reference's own close test, bug included: `flags & WS_OP_CLOSE`
                                    (websocket.h:87) is bit 3 of the opcode, so ping, pong and opcodes
                                    0xB-0xF close 1000 like a close frame (echo_once answers nothing else) */
struct xyws_verdict {
  uint16_t close_code; /* 0, or the code the connection closes with */
  uint16_t peer_code;  /* close frames: the peer's status code (1005 if none) */
  uint8_t  action;     /* XYWS_ACT_* */
  uint8_t  reserved[3];
};
int xyws_classify_frames(xyws_ctx* ctx, const void* dev_src, uint64_t src_len,
                         const xyws_frame* dev_frames, uint64_t n, const uint64_t* dev_n,
                         uint64_t max_payload, uint32_t policy, xyws_verdict* dev_verdicts,
                         uint64_t* dev_first_close, void* stream);

/* ---- message reassembly (FIN=0 chains) + UTF-8 validation ---------------
 * A message is a text/binary frame followed by continuation frames up to the
 * first one with FIN (control frames may sit between fragments and are not
 * part of it). Every message's payload is gathered into dev_out back to back
 * (frame payloads must be complete in dev_src: decoded, unmasked); its
 * record goes to dev_msgs[m] in order; *dev_nmsgs receives the count. With
 * XYWS_REASM_UTF8 every text message is validated (RFC 3629: no overlongs,
 * surrogates or code points above U+10FFFF). A continuation outside a
 * message is dropped and reported with XYWS_MSG_ORPHANS on the next message
 * (bit 0x200 of the device error word if none follows). */
#define XYWS_REASM_UTF8 0x1u
#define XYWS_MSG_COMPLETE   0x1u /* the FIN fragment is in this batch */
#define XYWS_MSG_UTF8_BAD   0x2u /* text message: invalid UTF-8 (a sequence cut by the end of an
                                    incomplete message is not counted) */
#define XYWS_MSG_INTERRUPTED 0x4u /* a new text/binary frame started before the FIN fragment */
#define XYWS_MSG_TRUNCATED  0x8u /* the payload did not fit in out_cap */
#define XYWS_MSG_ORPHANS    0x10u /* continuation frames without a message preceded this one */
typedef struct xyws_message {
  uint64_t first_frame; /* index of the text/binary frame that starts it */
  uint64_t nframes;     /* its data frames */
  uint64_t out_off;     /* its payload in dev_out */
  uint64_t length;      /* total payload bytes */
  uint32_t status;      /* XYWS_MSG_* */
  uint8_t  opcode;      /* XYWS_FLAG_OP_TEXT or XYWS_FLAG_OP_BINARY */
  uint8_t  reserved[3];
} xyws_message;         /* 40 bytes */
int xyws_reassemble(xyws_ctx* ctx, const void* dev_src, uint64_t src_len,
                    const xyws_frame* dev_frames, uint64_t n, const uint64_t* dev_n, uint32_t opts,
                    void* dev_out, uint64_t out_cap, xyws_message* dev_msgs, uint64_t msg_cap,
                    uint64_t* dev_nmsgs, void* stream);

/* ---- recv arenas: the io_uring side (recv_all.h:86-121, io_service.h:362-381)
 * One arena per connection: a receive area in pinned host memory (allocated
 * here, or the caller's buffer registered with hipHostRegister, e.g. the
 * memory an io_uring registered-buffer ring hands to recv), a device mirror,
 * a device-resident carry and up to XYWS_ARENA_SLOTS submissions in flight on
 * one of the context's arena streams (arenas share 8 streams round robin, so
 * any number of connections binds at most 8 scratch slots; an arena's
 * submissions stay in order). xyws_arena_submit(offset, len) enqueues
 * H2D -> xyws_decode_stream (carry chained across submissions, so a frame cut
 * by a recv boundary decodes as if unsplit) -> D2H of the unmasked bytes back
 * into the same host range (in place, like websocket_mask) and of the frame
 * table and count, then a host callback that marks the submission complete
 * and writes 1 to the arena's eventfd (when one is given): the ring keeps a
 * poll_add on that fd exactly as io_service does for its remote-queue eventfd
 * and never blocks on the GPU. xyws_arena_poll() returns XYWS_ERR_AGAIN until
 * the submission completed. Submissions complete in order. A submission's
 * results stay valid until its slot is reused, which happens only after
 * poll() or wait() returned them: submit() returns XYWS_ERR_AGAIN while
 * XYWS_ARENA_SLOTS submissions are in flight or unclaimed. wait() blocks on
 * that submission's own completion event, not on the shared stream (other
 * connections' later work is not waited for). Arenas that share a stream
 * share its scratch slot, so the decoder choice one arena's batches steer
 * (which decoder, which geometry: speed only, never bytes) applies to the
 * next batch of any arena on that stream. */
#define XYWS_ARENA_SLOTS 8
/* A submit that fails before anything was enqueued leaves the arena as it
 * was; one that fails later (the decode or a copy back could not be
 * enqueued) leaves it failed: the device carry may have moved past bytes no
 * result reports, so every later submit returns XYWS_ERR_HIP (destroy it). */
typedef struct xyws_arena xyws_arena;
typedef struct xyws_arena_result {
  uint64_t seq;              /* the submission */
  uint64_t offset, len;      /* its host range (now unmasked in place) */
  uint64_t nframes;          /* frames whose header completed in it */
  const xyws_frame* frames;  /* min(nframes, max_frames) descriptors, pinned host memory, offsets
                                relative to `offset`; valid until the slot is reused */
  xyws_carry carry;          /* the connection's carry after it */
} xyws_arena_result;
/* host == NULL: allocate `bytes` of pinned memory; else register the caller's
 * host range (unregistered at destroy). eventfd < 0: no notification. */
int xyws_arena_create(xyws_ctx* ctx, void* host, uint64_t bytes, uint64_t max_frames, int eventfd,
                      xyws_arena** out);
int xyws_arena_destroy(xyws_arena* a);
void* xyws_arena_host(xyws_arena* a);
int xyws_arena_submit(xyws_arena* a, uint64_t offset, uint64_t len, uint32_t opts, uint64_t* seq);
int xyws_arena_poll(xyws_arena* a, uint64_t seq, xyws_arena_result* out);
int xyws_arena_wait(xyws_arena* a, uint64_t seq, xyws_arena_result* out);
/* The completion notifier on its own (no device): what the arena's host
 * callback runs. Exposed so the eventfd handshake can be exercised on a host
 * without a GPU. */
typedef struct xyws_notifier xyws_notifier;
int xyws_notifier_create(int eventfd, xyws_notifier** out);
int xyws_notifier_destroy(xyws_notifier* n);
int xyws_notifier_signal(xyws_notifier* n, uint64_t seq); /* marks seq complete, writes the fd */
uint64_t xyws_notifier_completed(const xyws_notifier* n); /* highest completed seq + 1 */

/* ---- one batch across several devices -----------------
 * Frames are independent, so a batch of back-to-back frames splits across
 * devices at frame boundaries with no exchange between them. xyws_shard_plan
 * cuts `len` bytes of host memory (what a recv buffer_sequence holds,
 * buffer.h:94-224 / recv_all.h:99-121 of the reference) into n_shards
 * contiguous ranges bounds[k] .. bounds[k+1] (n_shards + 1 entries, bounds[0]
 * = 0, bounds[n_shards] = len) balanced by bytes: bounds[k] is the frame
 * start nearest to k * len / n_shards (each shard is within one frame of
 * len / n_shards). Shard 0 continues from `carry_in` (nullable = a fresh
 * stream); every other shard starts at a frame boundary, so it decodes on its
 * own device with a fresh carry (xyws_decode_stream, dev_carry_in = NULL) to
 * exactly the bytes and frames of the unsplit decode; only the last shard can
 * end inside a frame (its carry out continues the stream). The headers are
 * walked on the host (one header read per frame, parsed as
 * websocket_frame_header_parser::parse, websocket_frame_header.h:305-385):
 * a planner, not a decode — no payload byte is touched. A shard may be empty
 * when one frame is larger than len / n_shards. */
int xyws_shard_plan(const void* host_batch, uint64_t len, const xyws_carry* carry_in, uint32_t n_shards,
                    uint64_t* bounds);
/* The same from a frame table in host memory (frame_off ascending: e.g. the
 * descriptors of a parse-only decode, or the table a generator or a framing
 * layer already holds): the candidate boundaries are the frame_off >= 0
 * values (a negative frame_off, a header carried in, is not one) and len. */
int xyws_shard_plan_frames(const xyws_frame* frames, uint64_t n, uint64_t len, uint32_t n_shards,
                           uint64_t* bounds);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* XYWS_H */
