// xyws_device.h — device helpers shared by the gfx950 decode kernels.
//
// Header semantics restate websocket_frame_header_parser::parse
// (include/xynet/http/websocket_frame_header.h:305-385) for a parser fed
// from the frame start: byte 0 -> opcode | FIN (RSV dropped, :313-322),
// byte 1 -> MASK + 7-bit length (:323-346), 0/2/8 big-endian length bytes
// (:347-365), 4 key bytes in wire order (:366-377).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "xyws.h"

#define XYWS_DEV __device__ __forceinline__

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// All positions inside the kernels are byte offsets relative to `base`, a
// 16-byte-aligned address at or below the caller's buffer. The caller's bytes
// are [lo, hi) in that coordinate system (lo = buf & 15).

// A workgroup-uniform value read from LDS, moved to scalar registers (values
// loaded from LDS live in VGPRs otherwise, where the store loops need them).
XYWS_DEV uint32_t uniform32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// (the lane builtins return int: each half goes through uint32_t, or the low
// half's bit 31 would sign-extend over the high half)
XYWS_DEV uint64_t uniform64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
}

// Rotate a little-endian key word so byte t of the result XORs a byte whose
// payload index is congruent to t + c (mod 4).
XYWS_DEV uint32_t rotr8(uint32_t k, uint32_t c) {
  c &= 3u;
  return c ? ((k >> (8u * c)) | (k << (32u - 8u * c))) : k;
}

// Key word to XOR into any 4-byte-aligned word of a frame whose payload starts
// at position ps with mask phase ph (websocket_mask's i): payload index of byte
// t of the word at aligned a is a + t - ps, key byte K[(ph + a + t - ps) % 4];
// a % 4 == 0, so the rotation is the constant (ph - ps) mod 4.
XYWS_DEV uint32_t aligned_key(uint32_t key, uint64_t ps, uint64_t ph) {
  return rotr8(key, (uint32_t)(ph - ps));
}

// Byte-select mask of the bytes of the word at aligned position a that lie in
// [lo, hi).
XYWS_DEV uint32_t range_mask(uint64_t a, uint64_t lo, uint64_t hi) {
  if (hi <= a || lo >= a + 4) return 0u;
  uint32_t l = lo > a ? (uint32_t)(lo - a) : 0u;
  uint32_t h = hi < a + 4 ? (uint32_t)(hi - a) : 4u;
  uint32_t mh = h >= 4 ? 0xFFFFFFFFu : ((1u << (8u * h)) - 1u);
  uint32_t ml = (1u << (8u * l)) - 1u;  // l <= 3
  return mh & ~ml;
}

struct hdr_info {
  uint64_t plen;     // parsed payload length (raw, up to 2^64-1)
  uint32_t key;      // wire key bytes as a little-endian word (mask_uint32_t)
  uint32_t hlen;     // header length 2..14; 0 = incomplete
  uint8_t  flags;    // websocket_flags
  uint8_t  status;   // XYWS_ST_* (informational)
};

// Parse a header from up to 14 bytes b[0..avail). avail < needed -> hlen = 0.
XYWS_DEV hdr_info parse_header_bytes(const uint8_t* b, uint32_t avail) {
  hdr_info h;
  h.plen = 0; h.key = 0; h.hlen = 0; h.flags = 0; h.status = 0;
  if (avail < 2) return h;
  uint32_t b0 = b[0], b1 = b[1];
  uint32_t l7 = b1 & 0x7Fu;
  uint32_t ext = l7 == 126 ? 2u : (l7 == 127 ? 8u : 0u);
  uint32_t masked = b1 >> 7;
  uint32_t need = 2u + ext + 4u * masked;
  if (avail < need) return h;
  uint64_t len = l7;
  if (ext) {
    len = 0;
    for (uint32_t i = 0; i < ext; i++) len = (len << 8) | b[2 + i];
  }
  uint32_t key = 0;
  if (masked) {
    const uint8_t* k = b + 2 + ext;
    key = (uint32_t)k[0] | ((uint32_t)k[1] << 8) | ((uint32_t)k[2] << 16) | ((uint32_t)k[3] << 24);
  }
  uint32_t op = b0 & 0x0Fu;
  uint8_t st = 0;
  if (b0 & 0x70u) st |= XYWS_ST_RSV;
  if ((op >= 3 && op <= 7) || op >= 11) st |= XYWS_ST_RESERVED_OPCODE;
  if ((l7 == 126 && len < 126) || (l7 == 127 && len <= 0xFFFFull)) st |= XYWS_ST_NONMINIMAL_LENGTH;
  if (l7 == 127 && (len >> 63)) st |= XYWS_ST_LENGTH_MSB;
  if (op >= 8 && (!(b0 & 0x80u) || len > 125)) st |= XYWS_ST_BAD_CONTROL;
  if (!masked) st |= XYWS_ST_UNMASKED;
  h.plen = len;
  h.key = key;
  h.hlen = need;
  h.flags = (uint8_t)(op | ((b0 & 0x80u) ? XYWS_FLAG_FIN : 0u) | (masked ? XYWS_FLAG_HAS_MASK : 0u));
  h.status = st;
  return h;
}

// frame end = ps + plen, saturating at UINT64_MAX (a 2^63+ length never ends
// inside any batch).
XYWS_DEV uint64_t sat_add(uint64_t a, uint64_t b) {
  uint64_t s = a + b;
  return s < a ? ~0ull : s;
}

// The same parse from 16 little-endian bytes held in four dwords w[0..3]
// (byte i = w[i/4] >> 8*(i%4)), of which `avail` are valid: register-only,
// no byte array (the kernels read headers as dwords from LDS or memory).
XYWS_DEV hdr_info parse_header_words(const uint32_t w[4], uint32_t avail) {
  hdr_info h;
  h.plen = 0; h.key = 0; h.hlen = 0; h.flags = 0; h.status = 0;
  if (avail < 2) return h;
  const uint32_t b0 = w[0] & 0xFF, b1 = (w[0] >> 8) & 0xFF;
  const uint32_t l7 = b1 & 0x7Fu;
  const uint32_t ext = l7 == 126 ? 2u : (l7 == 127 ? 8u : 0u);
  const uint32_t masked = b1 >> 7;
  const uint32_t need = 2u + ext + 4u * masked;
  if (avail < need) return h;
  // bytes 2..9 as a big-endian length; bytes k..k+3 as the key (k = 2 + ext)
  const uint64_t lo8 = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  const uint64_t hi8 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  const uint64_t b2_9 = (lo8 >> 16) | (hi8 << 48);  // bytes 2..9, little-endian
  uint64_t len = l7;
  if (ext == 2) len = ((b2_9 & 0xFF) << 8) | ((b2_9 >> 8) & 0xFF);
  else if (ext == 8) len = __builtin_bswap64(b2_9);
  uint32_t key = 0;
  if (masked) {
    const uint32_t k = 2 + ext;  // 2, 4 or 10
    key = (k == 2) ? __builtin_amdgcn_alignbyte(w[1], w[0], 2)
        : (k == 4) ? w[1] : __builtin_amdgcn_alignbyte(w[3], w[2], 2);
  }
  const uint32_t op = b0 & 0x0Fu;
  uint8_t st = 0;
  if (b0 & 0x70u) st |= XYWS_ST_RSV;
  if ((op >= 3 && op <= 7) || op >= 11) st |= XYWS_ST_RESERVED_OPCODE;
  if ((l7 == 126 && len < 126) || (l7 == 127 && len <= 0xFFFFull)) st |= XYWS_ST_NONMINIMAL_LENGTH;
  if (l7 == 127 && (len >> 63)) st |= XYWS_ST_LENGTH_MSB;
  if (op >= 8 && (!(b0 & 0x80u) || len > 125)) st |= XYWS_ST_BAD_CONTROL;
  if (!masked) st |= XYWS_ST_UNMASKED;
  h.plen = len;
  h.key = key;
  h.hlen = need;
  h.flags = (uint8_t)(op | ((b0 & 0x80u) ? XYWS_FLAG_FIN : 0u) | (masked ? XYWS_FLAG_HAS_MASK : 0u));
  h.status = st;
  return h;
}
