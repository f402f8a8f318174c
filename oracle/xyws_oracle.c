/*
 * xyws_oracle.c — CPU ORACLE for the WebSocket frame-decode path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline). The product path (xynet_amd/, libxyws.so) never
 * links, loads or calls it.
 *
 * What it is: a plain-C restatement of the reference hot path
 * (xuanyi-fu/xynet, paths relative to the reference tree):
 *   - websocket_frame_header_parser::parse state machine
 *       include/xynet/http/websocket_frame_header.h:285-292 (states), :305-385 (parse)
 *   - result()/mask_uint32_t()/reset()      :259-281
 *   - detail::calc_frame_header_size         :111-126
 *   - detail::websocket_frame_header_builder :136-175
 *   - websocket_mask                         include/xynet/http/websocket_frame_mask.h:6-25
 *   - websocket_check_parser_result's policy example/include/common/websocket.h:81-108
 *   - echo_once's reply (header + payload)   example/websocket/websocket_echo.cpp:18-27
 * and the batch semantics this build defines on top of them: every frame of a
 * back-to-back batch parsed by a fresh parser and its payload unmasked in
 * place from phase 0, as websocket_recv_data does for one frame
 * (example/include/common/websocket.h:110-134), with a carry so a stream cut
 * at any byte decodes identically.
 *
 * Pinning: tests/test_oracle.py checks this restatement against the golden
 * vectors in tests/golden/, which tests/golden/gen_golden.py produced from the
 * REAL reference headers compiled in the survey container (oracle/_ref), and
 * against the reference's own test cases (test/websocket_frame_test.cpp:10-89)
 * and the RFC 6455 §5.7 "Hello" example.
 */
#include <pthread.h>
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>
#include "xyws.h"
#include "xyws_synth.h"

#define ORACLE_NPOS ((size_t)-1) /* websocket_frame_header_parser::npos, :230 */

enum { S_START = 0, S_HEAD, S_LENGTH, S_MASK, S_FINISHED }; /* :285-292 */

typedef struct oracle_parser {
  uint32_t state;
  uint8_t  flags;
  uint8_t  mask[4];
  uint8_t  pad[3];
  uint64_t length;
  uint64_t require;
} oracle_parser;

void oracle_parser_reset(oracle_parser* p) { /* reset(), :274-281 */
  p->state = S_START;
  p->flags = 0;
  memset(p->mask, 0, 4);
  p->length = 0;
  p->require = 0;
}

/* parse(const unsigned char*, size_t), :305-385. Returns the bytes consumed
 * in THIS call up to the end of the header, or npos while incomplete. Once
 * finished, further input returns npos until reset (default branch, :378). */
size_t oracle_parser_parse(oracle_parser* p, const uint8_t* data, size_t len) {
  const uint8_t* q = data;
  const uint8_t* end = data + len;
  for (; q != end; q++) {
    switch (p->state) {
      case S_START: /* :313-322; note m_mask is NOT cleared here */
        p->length = 0;
        p->flags = (uint8_t)(*q & XYWS_FLAG_OP_MASK); /* RSV bits dropped, :315 */
        if (*q & 0x80u) p->flags |= XYWS_FLAG_FIN;
        p->state = S_HEAD;
        break;
      case S_HEAD: /* :323-346 */
        p->length = (uint64_t)(*q & 0x7Fu);
        if (*q & 0x80u) p->flags |= XYWS_FLAG_HAS_MASK;
        if (p->length >= 126) {
          p->require = (p->length == 127) ? 8 : 2;
          p->length = 0;
          p->state = S_LENGTH;
        } else if (p->flags & XYWS_FLAG_HAS_MASK) {
          p->state = S_MASK;
          p->require = 4;
        } else {
          p->state = S_FINISHED;
          return (size_t)(q - data) + 1;
        }
        break;
      case S_LENGTH: /* :347-365, big-endian accumulate */
        while (q < end && p->require) {
          p->length = (p->length << 8) | (uint64_t)(*q);
          p->require--;
          q++;
        }
        q--;
        if (!p->require) {
          if (p->flags & XYWS_FLAG_HAS_MASK) {
            p->state = S_MASK;
            p->require = 4;
          } else {
            p->state = S_FINISHED;
            return (size_t)(q - data) + 1;
          }
        }
        break;
      case S_MASK: /* :366-377, key kept in wire order */
        while (q < end && p->require) {
          p->mask[4 - p->require] = *q;
          p->require--;
          q++;
        }
        q--;
        if (!p->require) {
          p->state = S_FINISHED;
          return (size_t)(q - data) + 1;
        }
        break;
      default:
        break;
    }
  }
  return ORACLE_NPOS; /* incomplete, :383-384 */
}

/* mask_uint32_t(), :259-262: the four wire bytes reinterpreted as a host
 * (little-endian) integer. */
uint32_t oracle_parser_mask_u32(const oracle_parser* p) {
  return (uint32_t)p->mask[0] | ((uint32_t)p->mask[1] << 8) |
         ((uint32_t)p->mask[2] << 16) | ((uint32_t)p->mask[3] << 24);
}
uint8_t oracle_parser_flags(const oracle_parser* p) { return p->flags; }
uint64_t oracle_parser_length(const oracle_parser* p) { return p->length; }

/* websocket_mask, websocket_frame_mask.h:6-25: in place,
 * data[j] ^= ((const byte*)&mask)[(i + j) % 4]; returns i + len. On the
 * little-endian hosts this targets, byte t of `mask` is (mask >> 8t). */
uint64_t oracle_mask(uint8_t* data, uint64_t len, uint32_t mask, uint64_t i) {
  for (uint64_t j = 0; j < len; j++) {
    data[j] ^= (uint8_t)(mask >> (8u * (uint32_t)((i + j) % 4)));
  }
  return i + len;
}

/* detail::calc_frame_header_size, :111-126 */
uint64_t oracle_calc_frame_header_size(uint8_t flags, uint64_t len) {
  uint64_t size = 2;
  if (len >= 126) size += (len > 0xFFFF) ? 8 : 2;
  if (flags & XYWS_FLAG_HAS_MASK) size += 4;
  return size;
}

/* detail::websocket_frame_header_builder, :136-175. Key bytes are copied
 * only when `mask` is non-null (:168-171). */
uint64_t oracle_header_build(uint8_t* frame, uint8_t flags, const uint8_t* mask, uint64_t len) {
  uint64_t off = 0;
  frame[0] = 0;
  frame[1] = 0;
  if (flags & XYWS_FLAG_FIN) frame[0] = 0x80;
  frame[0] |= (uint8_t)(flags & XYWS_FLAG_OP_MASK);
  if (flags & XYWS_FLAG_HAS_MASK) frame[1] = 0x80;
  if (len < 126) {
    frame[1] |= (uint8_t)len;
    off = 2;
  } else if (len <= 0xFFFF) {
    frame[1] |= 126;
    frame[2] = (uint8_t)(len >> 8);
    frame[3] = (uint8_t)(len & 0xFF);
    off = 4;
  } else {
    frame[1] |= 127;
    for (int b = 0; b < 8; b++) frame[2 + b] = (uint8_t)(len >> (56 - 8 * b));
    off = 10;
  }
  if (flags & XYWS_FLAG_HAS_MASK) {
    if (mask) memcpy(&frame[off], mask, 4);
    off += 4;
  }
  return off;
}

/* Informational RFC 6455 checks on a complete header (never change output). */
static uint8_t oracle_header_status(const uint8_t* hdr, uint64_t plen) {
  uint8_t st = 0;
  uint8_t b0 = hdr[0], b1 = hdr[1];
  uint8_t op = b0 & 0x0F;
  uint8_t l7 = b1 & 0x7F;
  if (b0 & 0x70) st |= XYWS_ST_RSV;
  if ((op >= 3 && op <= 7) || op >= 11) st |= XYWS_ST_RESERVED_OPCODE;
  if ((l7 == 126 && plen < 126) || (l7 == 127 && plen <= 0xFFFF)) st |= XYWS_ST_NONMINIMAL_LENGTH;
  if (l7 == 127 && (plen >> 63)) st |= XYWS_ST_LENGTH_MSB;
  if (op >= 8 && (!(b0 & 0x80) || plen > 125)) st |= XYWS_ST_BAD_CONTROL;
  if (!(b1 & 0x80)) st |= XYWS_ST_UNMASKED;
  return st;
}

/*
 * Batch decode with carry (the semantics xyws_decode_stream implements).
 * Returns the number of frames whose header completed in this batch.
 */
uint64_t oracle_decode_stream(uint8_t* buf, uint64_t len, const xyws_carry* cin,
                              xyws_carry* cout, xyws_frame* frames, uint64_t cap) {
  xyws_carry c;
  if (cin) c = *cin; else memset(&c, 0, sizeof c);
  uint64_t pos = 0, n = 0;
  if (c.payload_remaining) {
    uint64_t take = c.payload_remaining < len ? c.payload_remaining : len;
    uint32_t k = (uint32_t)c.key[0] | ((uint32_t)c.key[1] << 8) | ((uint32_t)c.key[2] << 16) |
                 ((uint32_t)c.key[3] << 24);
    c.phase = oracle_mask(buf, take, k, c.phase);
    c.payload_remaining -= take;
    pos = take;
    if (!c.payload_remaining) { c.phase = 0; memset(c.key, 0, 4); }
  }
  while (pos < len) {
    oracle_parser p;
    oracle_parser_reset(&p);
    int64_t frame_off = (int64_t)pos;
    uint8_t hdr[XYWS_MAX_FRAME_HEADER_SIZE];
    uint32_t h0 = c.hdr_len;
    if (h0) {
      memcpy(hdr, c.hdr, h0);
      (void)oracle_parser_parse(&p, c.hdr, h0); /* npos by construction */
      frame_off = (int64_t)pos - (int64_t)h0;
    }
    size_t r = oracle_parser_parse(&p, buf + pos, len - pos);
    if (r == ORACLE_NPOS) { /* incomplete header: keep its bytes */
      uint64_t have = len - pos;
      memcpy(c.hdr + h0, buf + pos, have);
      c.hdr_len = (uint8_t)(h0 + have);
      pos = len;
      break;
    }
    memcpy(hdr + h0, buf + pos, r);
    uint64_t payload_off = pos + r;
    uint64_t plen = p.length;
    xyws_frame f;
    memset(&f, 0, sizeof f);
    f.frame_off = frame_off;
    f.payload_off = (int64_t)payload_off;
    f.payload_len = plen;
    memcpy(f.key, p.mask, 4);
    f.flags = p.flags;
    f.hdr_len = (uint8_t)(h0 + r);
    f.status = oracle_header_status(hdr, plen);
    c.hdr_len = 0;
    memset(c.hdr, 0, sizeof c.hdr);
    uint64_t avail = len - payload_off;
    uint32_t key = oracle_parser_mask_u32(&p);
    if (plen <= avail) {
      oracle_mask(buf + payload_off, plen, key, 0);
      pos = payload_off + plen;
    } else {
      c.phase = oracle_mask(buf + payload_off, avail, key, 0);
      c.payload_remaining = plen - avail;
      memcpy(c.key, p.mask, 4);
      f.status |= XYWS_ST_PAYLOAD_INCOMPLETE;
      pos = len;
    }
    if (frames && n < cap) frames[n] = f;
    n++;
  }
  c.frames_total += n;
  if (cout) *cout = c;
  return n;
}

/* Indexed decode (the semantics of xyws_decode_indexed): caller-supplied,
 * ascending frame starts; each frame parsed by a fresh parser, payload
 * clipped to the buffer and to the next start. */
void oracle_decode_indexed(uint8_t* buf, uint64_t len, const uint64_t* starts, uint64_t n,
                           xyws_frame* frames) {
  for (uint64_t i = 0; i < n; i++) {
    uint64_t s = starts[i];
    xyws_frame f;
    memset(&f, 0, sizeof f);
    f.frame_off = (int64_t)s;
    f.payload_off = (int64_t)s;
    oracle_parser p;
    oracle_parser_reset(&p);
    size_t r = (s < len) ? oracle_parser_parse(&p, buf + s, len - s) : ORACLE_NPOS;
    if (r != ORACLE_NPOS) {
      uint64_t ps = s + r, plen = p.length;
      f.payload_off = (int64_t)ps;
      f.payload_len = plen;
      memcpy(f.key, p.mask, 4);
      f.flags = p.flags;
      f.hdr_len = (uint8_t)r;
      f.status = oracle_header_status(buf + s, plen);
      uint64_t lim = len;
      if (i + 1 < n && starts[i + 1] < lim) lim = starts[i + 1];
      uint64_t end = (plen > UINT64_MAX - ps) ? UINT64_MAX : ps + plen; /* saturating */
      uint64_t pe = (plen > len - ps) ? len : ps + plen;
      if (plen > len - ps) f.status |= XYWS_ST_PAYLOAD_INCOMPLETE;
      if (i + 1 < n && end > starts[i + 1]) f.status |= XYWS_ST_OVERLAP;
      if (pe > lim) pe = lim;
      if (pe > ps) oracle_mask(buf + ps, pe - ps, oracle_parser_mask_u32(&p), 0);
    }
    if (frames) frames[i] = f;
  }
}

/* ---- the callers either side of the path (xyws_frames.hip's semantics) ---- */

/* echo_once's reply for every selected frame (websocket_echo.cpp:22-26):
 * header_build(flags_i, key_i or NULL, len_i) + payload bytes (masked with
 * key_i when keys are given), back to back. Returns the total reply bytes;
 * bytes past out_cap are not written; offsets (nullable) gets n + 1 entries. */
uint64_t oracle_encode_frames(const uint8_t* src, uint64_t src_len, const xyws_frame* frames, uint64_t n,
                              uint8_t flags, uint32_t enc_opts, const uint8_t* keys, const xyws_verdict* verd,
                              uint32_t amask, uint8_t* out, uint64_t out_cap, uint64_t* offsets) {
  uint64_t pos = 0;
  for (uint64_t i = 0; i < n; i++) {
    if (offsets) offsets[i] = pos;
    if (verd && !((amask >> verd[i].action) & 1u)) continue;
    const xyws_frame* f = &frames[i];
    uint8_t fl = flags;
    if (enc_opts & XYWS_ENC_FRAME_OPCODE) {
      uint8_t op = f->flags & XYWS_FLAG_OP_MASK;
      if (op == XYWS_FLAG_OP_PING) op = XYWS_FLAG_OP_PONG;
      fl = (uint8_t)(op | (f->flags & XYWS_FLAG_FIN) | (flags & XYWS_FLAG_HAS_MASK));
    }
    const uint8_t* key = (keys && (fl & XYWS_FLAG_HAS_MASK)) ? keys + 4 * i : NULL;
    uint8_t hdr[XYWS_MAX_FRAME_HEADER_SIZE] = {0};  /* (zero key bytes without a key, as the
                                                        class's zero-initialised array, :221) */
    uint64_t h = oracle_header_build(hdr, fl, key, f->payload_len);
    for (uint64_t j = 0; j < h; j++, pos++)
      if (pos < out_cap) out[pos] = hdr[j];
    for (uint64_t j = 0; j < f->payload_len; j++, pos++) {
      uint64_t sp = (uint64_t)f->payload_off + j;
      uint8_t b = sp < src_len ? src[sp] : 0;
      if (key) b ^= key[j & 3];
      if (pos < out_cap) out[pos] = b;
    }
  }
  if (offsets) offsets[n] = pos;
  return pos;
}

/* websocket_check_parser_result (websocket.h:81-108): close -> 1000, FIN=0 ->
 * 1003, unmasked -> 1008, length > max -> 1009, first match wins; without its
 * bit-3 test (`flags & WS_OP_CLOSE` is also true for ping and pong). Policy
 * bits: XYWS_POL_FRAGMENTS skips the FIN test, XYWS_POL_UNMASKED the mask
 * test, XYWS_POL_STRICT puts RFC protocol errors (1002) first, XYWS_POL_REFERENCE
 * restores the bit-3 test (websocket.h:87: ping, pong, 0xB-0xF close 1000). *first: the
 * first closing frame, or UINT64_MAX. */
void oracle_classify(const uint8_t* src, uint64_t src_len, const xyws_frame* frames, uint64_t n,
                     uint64_t max_payload, uint32_t policy, xyws_verdict* out, uint64_t* first) {
  if (first) *first = UINT64_MAX;
  for (uint64_t i = 0; i < n; i++) {
    const xyws_frame* f = &frames[i];
    uint8_t op = f->flags & XYWS_FLAG_OP_MASK;
    xyws_verdict v;
    memset(&v, 0, sizeof v);
    v.action = op == XYWS_FLAG_OP_PING ? XYWS_ACT_PING : op == XYWS_FLAG_OP_PONG ? XYWS_ACT_PONG : XYWS_ACT_DATA;
    int proto = (f->status & (XYWS_ST_RSV | XYWS_ST_RESERVED_OPCODE | XYWS_ST_BAD_CONTROL)) != 0;
    uint16_t code = 0;
    if ((policy & XYWS_POL_STRICT) && proto) code = 1002;
    else if (op == XYWS_FLAG_OP_CLOSE || ((policy & XYWS_POL_REFERENCE) && (op & 8u))) code = 1000;
    else if (!(f->flags & XYWS_FLAG_FIN) && !(policy & XYWS_POL_FRAGMENTS)) code = 1003;
    else if (!(f->flags & XYWS_FLAG_HAS_MASK) && !(policy & XYWS_POL_UNMASKED)) code = 1008;
    else if (f->payload_len > max_payload) code = 1009;
    if (op == XYWS_FLAG_OP_CLOSE) {
      v.action = XYWS_ACT_CLOSE;
      uint64_t p = (uint64_t)f->payload_off;
      v.peer_code = 1005;
      if (f->payload_len >= 2 && p + 2 <= src_len) v.peer_code = (uint16_t)((src[p] << 8) | src[p + 1]);
    }
    if (code) {
      v.close_code = code;
      v.action = XYWS_ACT_CLOSE;
      if (first && *first == UINT64_MAX) *first = i;
    }
    out[i] = v;
  }
}

/* RFC 3629 UTF-8 over s[0, len): 1 if valid. With complete == 0 a sequence
 * cut by the end is accepted (the message continues later). */
int oracle_utf8_valid(const uint8_t* s, uint64_t len, int complete) {
  uint64_t i = 0;
  while (i < len) {
    uint8_t c = s[i];
    if (c < 0x80) { i++; continue; }
    uint32_t L = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 0;
    if (L == 0 || c == 0xC0 || c == 0xC1 || c >= 0xF5) return 0;
    for (uint32_t d = 1; d < L; d++) {
      if (i + d >= len) return complete ? 0 : 1;
      uint8_t x = s[i + d];
      if ((x & 0xC0) != 0x80) return 0;
      if (d == 1) {
        if (c == 0xE0 && x < 0xA0) return 0;
        if (c == 0xED && x > 0x9F) return 0;
        if (c == 0xF0 && x < 0x90) return 0;
        if (c == 0xF4 && x > 0x8F) return 0;
      }
    }
    i += L;
  }
  return 1;
}

/* Messages of a decoded batch (the semantics of xyws_reassemble): a text or
 * binary frame opens a message, continuations join it up to the first with
 * FIN; control frames between fragments are skipped; a continuation with no
 * open message is dropped (XYWS_MSG_ORPHANS on the next message). Payloads
 * are gathered into out back to back. Returns the message count. */
uint64_t oracle_reassemble(const uint8_t* src, uint64_t src_len, const xyws_frame* frames, uint64_t n,
                           uint32_t opts, uint8_t* out, uint64_t out_cap, xyws_message* msgs, uint64_t msg_cap) {
  uint64_t nm = 0, pos = 0;
  int64_t open = -1;
  int orphans = 0;
  for (uint64_t i = 0; i < n; i++) {
    const xyws_frame* f = &frames[i];
    uint8_t op = f->flags & XYWS_FLAG_OP_MASK;
    if (op > XYWS_FLAG_OP_BINARY) continue;
    int64_t m;
    if (op != XYWS_FLAG_OP_CONTINUE) {
      if (open >= 0 && (uint64_t)open < msg_cap) msgs[open].status |= XYWS_MSG_INTERRUPTED;
      m = (int64_t)nm++;
      if ((uint64_t)m < msg_cap) {
        memset(&msgs[m], 0, sizeof msgs[m]);
        msgs[m].first_frame = i;
        msgs[m].out_off = pos;
        msgs[m].opcode = op;
        msgs[m].status = orphans ? XYWS_MSG_ORPHANS : 0;
      }
      orphans = 0;
      open = m;
    } else {
      if (open < 0) { orphans = 1; continue; }
      m = open;
    }
    for (uint64_t j = 0; j < f->payload_len; j++, pos++) {
      uint64_t sp = (uint64_t)f->payload_off + j;
      if (pos < out_cap) out[pos] = sp < src_len ? src[sp] : 0;
    }
    if ((uint64_t)m < msg_cap) {
      msgs[m].nframes++;
      msgs[m].length += f->payload_len;
    }
    if (f->flags & XYWS_FLAG_FIN) {
      if ((uint64_t)m < msg_cap) msgs[m].status |= XYWS_MSG_COMPLETE;
      open = -1;
    }
  }
  uint64_t lim = nm < msg_cap ? nm : msg_cap;
  for (uint64_t m = 0; m < lim; m++) {
    xyws_message* M = &msgs[m];
    if (M->out_off + M->length > out_cap) M->status |= XYWS_MSG_TRUNCATED;
    if ((opts & XYWS_REASM_UTF8) && M->opcode == XYWS_FLAG_OP_TEXT) {
      uint64_t avail = M->out_off >= out_cap ? 0 : out_cap - M->out_off;
      uint64_t len = M->length < avail ? M->length : avail;
      int complete = (M->status & XYWS_MSG_COMPLETE) && !(M->status & XYWS_MSG_TRUNCATED);
      if (!oracle_utf8_valid(out + M->out_off, len, complete)) M->status |= XYWS_MSG_UTF8_BAD;
    }
  }
  return nm;
}

/* ---- synthetic batches + digest (shared spec: include/xyws_synth.h) ------ */

uint64_t oracle_digest(const uint8_t* buf, uint64_t len) {
  uint64_t sum = 0, i = 0;
  for (; (i + 1) * 8 <= len; i++) {
    uint64_t w;
    memcpy(&w, buf + i * 8, 8);
    sum += xyws_digest_term(i, w);
  }
  if (i * 8 < len) {
    uint64_t w = 0;
    memcpy(&w, buf + i * 8, len - i * 8);
    sum += xyws_digest_term(i, w);
  }
  return xyws_digest_finish(sum, len);
}

void oracle_fill_uniform(uint8_t* buf, uint64_t nframes, uint64_t plen, uint8_t b0, uint64_t seed) {
  uint64_t H = xyws_synth_hdr_len(plen, 1), S = H + plen;
  uint64_t dpf = xyws_synth_draws_per_frame(plen);
  for (uint64_t f = 0; f < nframes; f++) {
    uint8_t* fr = buf + f * S;
    uint64_t d = f * dpf;
    uint32_t key = xyws_synth_key(seed, d);
    for (uint32_t i = 0; i < H; i++) fr[i] = xyws_synth_hdr_byte(b0, plen, key, i);
    uint8_t* pl = fr + H;
    uint64_t j = 0;
    for (; j + 8 <= plen; j += 8) {
      uint64_t w = xyws_sm64_at(seed, d + 1 + j / 8);
      for (int b = 0; b < 8; b++) pl[j + b] = (uint8_t)(w >> (8 * b)) ^ (uint8_t)(key >> (8 * ((j + b) & 3)));
    }
    for (; j < plen; j++) pl[j] = xyws_synth_plain_byte(seed, d, j) ^ (uint8_t)(key >> (8 * (j & 3)));
  }
}

uint64_t oracle_mixed_table(uint64_t seed, uint64_t target, xyws_synth_frame* out, uint64_t cap,
                            uint64_t* total) {
  return xyws_synth_mixed_table(seed, target, out, cap, total);
}

void oracle_fill_mixed(uint8_t* buf, const xyws_synth_frame* tab, uint64_t n, uint64_t seed) {
  for (uint64_t f = 0; f < n; f++) {
    const xyws_synth_frame* fr = &tab[f];
    uint8_t* p = buf + fr->off;
    uint32_t key = xyws_synth_key(seed, fr->draw);
    for (uint32_t i = 0; i < fr->hlen; i++) p[i] = xyws_synth_hdr_byte(fr->b0, fr->plen, key, i);
    uint8_t* pl = p + fr->hlen;
    for (uint64_t j = 0; j < fr->plen; j++)
      pl[j] = xyws_synth_plain_byte(seed, fr->draw, j) ^ (uint8_t)(key >> (8 * (j & 3)));
  }
}

/* ---- CPU baseline (bench.py cpu_baseline, kind "port") --------------------
 * The reference's per-frame work on a batch held in host memory, on `threads`
 * host threads: one thread walks the headers with the parser above (boundary
 * discovery is serial by nature: websocket_frame_header.h:305-385), then the
 * frames' payloads are unmasked with oracle_mask (websocket_frame_mask.h:6-25)
 * by `threads` workers over byte-balanced contiguous frame ranges. Whole
 * frames only (a trailing partial frame is ignored). Returns the frame count. */
typedef struct { uint64_t ps, plen; uint32_t mask; } oracle_span;
typedef struct { uint8_t* buf; const oracle_span* fs; uint64_t a, b; } oracle_work;

static void* oracle_worker(void* arg) {
  const oracle_work* w = (const oracle_work*)arg;
  for (uint64_t i = w->a; i < w->b; i++) oracle_mask(w->buf + w->fs[i].ps, w->fs[i].plen, w->fs[i].mask, 0);
  return NULL;
}

uint64_t oracle_decode_batch_mt(uint8_t* buf, uint64_t len, int threads) {
  uint64_t cap = 1024, n = 0, pos = 0;
  oracle_span* fs = (oracle_span*)malloc(cap * sizeof *fs);
  if (!fs) return 0;
  while (pos < len) {
    oracle_parser p;
    oracle_parser_reset(&p);
    size_t r = oracle_parser_parse(&p, buf + pos, len - pos);
    if (r == ORACLE_NPOS || p.length > len - (pos + r)) break;
    if (n == cap) {
      oracle_span* g = (oracle_span*)realloc(fs, 2 * cap * sizeof *fs);
      if (!g) break;
      fs = g;
      cap *= 2;
    }
    fs[n].ps = pos + r;
    fs[n].plen = p.length;
    fs[n].mask = oracle_parser_mask_u32(&p);
    n++;
    pos += r + p.length;
  }
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  oracle_work w[256];
  uint64_t per = pos / (uint64_t)threads + 1, a = 0;
  int nt = 0;
  for (int t = 0; t < threads && a < n; t++) {
    uint64_t b = a, lim = (uint64_t)(t + 1) * per;
    while (b < n && (fs[b].ps < lim || b == a)) b++;
    if (t == threads - 1) b = n;
    w[nt].buf = buf; w[nt].fs = fs; w[nt].a = a; w[nt].b = b;
    if (threads == 1 || pthread_create(&tid[nt], NULL, oracle_worker, &w[nt]) != 0) {
      oracle_worker(&w[nt]);
    } else {
      nt++;
    }
    a = b;
  }
  for (int t = 0; t < nt; t++) pthread_join(tid[t], NULL);
  free(fs);
  return n;
}
