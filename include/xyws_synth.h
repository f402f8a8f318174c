/*
 * xyws_synth.h — synthetic masked-frame batches and the batch digest.
 *
 * TEST/BENCH INFRASTRUCTURE, not part of the decode path. Compiles as C (gcc,
 * the oracle and the golden generator) and as HIP (hipcc, the device-side
 * generator used by bench.py), so both sides build bit-identical batches.
 *
 * Random numbers: splitmix64, used counter-style so the device can generate in
 * parallel: draw k of the stream seeded with s is mix(s + (k+1)*gamma), which
 * is exactly the (k+1)-th output of the sequential splitmix64 generator.
 *
 * Uniform batch (SURVEY.md §8(d) configs 1,2,3,5): N frames of P payload bytes,
 * byte 0 = b0 (0x81 text / 0x82 binary, FIN set), MASK set, minimal length
 * form (header = calc_frame_header_size, websocket_frame_header.h:111-126).
 * Frame f occupies [f*S, (f+1)*S), S = H + P. Its draws start at
 * d_f = f * (1 + ceil(P/8)): key = low 32 bits of draw d_f (wire order = its
 * little-endian bytes), plaintext word j = draw d_f + 1 + j. The wire payload
 * is plaintext XOR key (RFC 6455 §5.3), so a correct unmask restores the
 * plaintext.
 *
 * Digest: position-keyed sum over little-endian 8-byte words (last word zero
 * padded) — order-independent to compute, so the device reduces it in parallel:
 *   D = mix(len) + sum_i mix(w_i ^ (i * 0xD1B54A32D192ED03))   (mod 2^64)
 */
#ifndef XYWS_SYNTH_H
#define XYWS_SYNTH_H

#include <stdint.h>
#include <stddef.h>

#if defined(__HIPCC__)
#define XYWS_HD __host__ __device__ static inline
#else
#define XYWS_HD static inline
#endif

#define XYWS_SM64_GAMMA 0x9E3779B97F4A7C15ULL
#define XYWS_DIGEST_GAMMA 0xD1B54A32D192ED03ULL

XYWS_HD uint64_t xyws_sm64_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

/* k-th (0-based) output of splitmix64 seeded with `seed`. */
XYWS_HD uint64_t xyws_sm64_at(uint64_t seed, uint64_t k) {
  return xyws_sm64_mix(seed + (k + 1) * XYWS_SM64_GAMMA);
}

/* Header size for a masked/unmasked frame of payload length len
 * (restates calc_frame_header_size, websocket_frame_header.h:111-126). */
XYWS_HD uint32_t xyws_synth_hdr_len(uint64_t len, int masked) {
  uint32_t h = 2;
  if (len >= 126) h += (len > 0xFFFF) ? 8 : 2;
  if (masked) h += 4;
  return h;
}

/* Byte `i` (0 <= i < hlen) of a masked header with first byte b0, payload
 * length len and key (low byte = first wire key byte). */
XYWS_HD uint8_t xyws_synth_hdr_byte(uint8_t b0, uint64_t len, uint32_t key, uint32_t i) {
  if (i == 0) return b0;
  uint32_t ext = (len >= 126) ? ((len > 0xFFFF) ? 8 : 2) : 0;
  if (i == 1) return (uint8_t)(0x80u | (ext == 0 ? (uint32_t)len : (ext == 2 ? 126u : 127u)));
  if (i < 2 + ext) {
    uint32_t sh = 8u * (ext - 1u - (i - 2u));
    return (uint8_t)(len >> sh);
  }
  return (uint8_t)(key >> (8u * (i - 2u - ext)));
}

XYWS_HD uint64_t xyws_synth_draws_per_frame(uint64_t plen) { return 1 + (plen + 7) / 8; }

/* Plaintext payload byte j of a frame whose draws start at `draw_base`. */
XYWS_HD uint8_t xyws_synth_plain_byte(uint64_t seed, uint64_t draw_base, uint64_t j) {
  return (uint8_t)(xyws_sm64_at(seed, draw_base + 1 + j / 8) >> (8u * (uint32_t)(j & 7)));
}

XYWS_HD uint32_t xyws_synth_key(uint64_t seed, uint64_t draw_base) {
  return (uint32_t)xyws_sm64_at(seed, draw_base);
}

/* Wire byte at offset q of a uniform batch (N frames, payload P, first byte b0). */
XYWS_HD uint8_t xyws_synth_uniform_byte(uint64_t seed, uint64_t P, uint8_t b0, uint64_t q) {
  uint64_t H = xyws_synth_hdr_len(P, 1);
  uint64_t S = H + P;
  uint64_t f = q / S, r = q - f * S;
  uint64_t d = f * xyws_synth_draws_per_frame(P);
  uint32_t key = xyws_synth_key(seed, d);
  if (r < H) return xyws_synth_hdr_byte(b0, P, key, (uint32_t)r);
  uint64_t j = r - H;
  return (uint8_t)(xyws_synth_plain_byte(seed, d, j) ^ (uint8_t)(key >> (8u * (uint32_t)(j & 3))));
}

/* One digest term: word index i, value w. */
XYWS_HD uint64_t xyws_digest_term(uint64_t i, uint64_t w) {
  return xyws_sm64_mix(w ^ (i * XYWS_DIGEST_GAMMA));
}

XYWS_HD uint64_t xyws_digest_finish(uint64_t sum, uint64_t len) {
  return sum + xyws_sm64_mix(len ^ 0xA0761D6478BD642FULL);
}

/* Frame record of a mixed batch (config 4); built on the host, filled on either side. */
typedef struct xyws_synth_frame {
  uint64_t off;   /* offset of header byte 0 */
  uint64_t plen;  /* payload length */
  uint64_t draw;  /* first draw index (key) */
  uint8_t  b0;    /* header byte 0 */
  uint8_t  hlen;  /* header length */
  uint8_t  pad[6];
} xyws_synth_frame;  /* 32 bytes */

#if !defined(__HIP_DEVICE_COMPILE__)
/*
 * Mixed batch structure (config 4), sequential splitmix64 over `seed`:
 * frames until the batch holds >= target bytes. Payload P is log-uniform over
 * [1, 2^20]: octave e uniform in 0..20, then uniform inside [2^e, 2^(e+1))
 * (e = 20 gives exactly 2^20); integer-only so every compiler agrees. With probability 1/4 a frame opens
 * a fragmented message of 2..8 frames (first opcode 2 FIN=0, middle opcode 0
 * FIN=0, last opcode 0 FIN=1); between fragments a masked ping (0x89, payload
 * 0..125) is inserted with probability 1/64. Other frames are 0x82. Every
 * frame has its own key; draws for keys/payload come from the same stream
 * (record.draw). Returns the frame count; writes at most cap records and the
 * total batch length to *total.
 */
static inline uint64_t xyws_synth_mixed_table(uint64_t seed, uint64_t target,
                                              xyws_synth_frame* out, uint64_t cap,
                                              uint64_t* total) {
  uint64_t k = 0;                /* structure-stream counter */
  uint64_t sseed = seed ^ 0x5851F42D4C957F2DULL;
  uint64_t draw = 0, off = 0, n = 0;
#define XYWS_NEXT() xyws_sm64_at(sseed, k++)
  /* log-uniform payload length: octave e uniform in 0..20, uniform inside it */
#define XYWS_PLEN() __extension__({ uint64_t e_ = XYWS_NEXT() % 21;              \
    e_ == 20 ? (1ULL << 20) : ((1ULL << e_) | (XYWS_NEXT() & ((1ULL << e_) - 1))); })
#define XYWS_EMIT(B0, P) do {                                              \
    uint64_t p_ = (P);                                                    \
    if (n < cap && out) {                                                 \
      out[n].off = off; out[n].plen = p_; out[n].draw = draw;             \
      out[n].b0 = (uint8_t)(B0); out[n].hlen = (uint8_t)xyws_synth_hdr_len(p_, 1); \
    }                                                                     \
    off += xyws_synth_hdr_len(p_, 1) + p_;                                \
    draw += xyws_synth_draws_per_frame(p_);                               \
    n++;                                                                  \
  } while (0)
  while (off < target) {
    uint64_t P = XYWS_PLEN();
    int frag = (XYWS_NEXT() & 3u) == 0;
    if (!frag) {
      XYWS_EMIT(0x82, P);
    } else {
      uint64_t m = 2 + XYWS_NEXT() % 7;
      for (uint64_t i = 0; i < m; i++) {
        uint8_t b0 = (uint8_t)((i == 0 ? 0x02 : 0x00) | (i == m - 1 ? 0x80 : 0x00));
        uint64_t Pi = (i == 0) ? P : XYWS_PLEN();
        XYWS_EMIT(b0, Pi);
        if (i + 1 < m && (XYWS_NEXT() & 63u) == 0) {
          XYWS_EMIT(0x89, XYWS_NEXT() % 126);
        }
      }
    }
  }
#undef XYWS_NEXT
#undef XYWS_PLEN
#undef XYWS_EMIT
  if (total) *total = off;
  return n;
}
#endif

/* Wire byte r (0 <= r < hlen + plen) of a mixed-batch frame. */
XYWS_HD uint8_t xyws_synth_frame_byte(uint64_t seed, const xyws_synth_frame* fr, uint64_t r) {
  uint32_t key = xyws_synth_key(seed, fr->draw);
  if (r < fr->hlen) return xyws_synth_hdr_byte(fr->b0, fr->plen, key, (uint32_t)r);
  uint64_t j = r - fr->hlen;
  return (uint8_t)(xyws_synth_plain_byte(seed, fr->draw, j) ^ (uint8_t)(key >> (8u * (uint32_t)(j & 3))));
}

#endif /* XYWS_SYNTH_H */
