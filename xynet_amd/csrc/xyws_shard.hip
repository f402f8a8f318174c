// xyws_shard.hip — host-side shard planner: one batch of back-to-back frames
// cut into per-device ranges at frame boundaries (C-ABI in
// include/xyws.h). No kernels: the plan is a walk over the headers (one read
// per frame), the decode of each range is xyws_decode_stream on its device.
//
// A frame starts at X, its header is parsed as
// websocket_frame_header_parser::parse does from a fresh parser
// (include/xynet/http/websocket_frame_header.h:305-385: 2 bytes, 0/2/8
// big-endian length bytes, 4 key bytes when MASK is set; nothing rejected),
// and the next frame starts at X + header + payload length.
#include <stdint.h>
#include <string.h>

#include "xyws.h"

namespace {

constexpr uint64_t U64MAX = ~0ull;

uint64_t sat_add_h(uint64_t a, uint64_t b) {
  const uint64_t s = a + b;
  return s < a ? U64MAX : s;
}

// Header size and payload length of the header whose first `avail` bytes are
// b[0..avail); false when they do not complete it.
bool header_span(const uint8_t* b, uint64_t avail, uint64_t* hlen, uint64_t* plen) {
  if (avail < 2) return false;
  const uint32_t l7 = b[1] & 0x7Fu;
  const uint32_t ext = l7 == 126 ? 2u : (l7 == 127 ? 8u : 0u);
  const uint64_t need = 2u + ext + ((b[1] & 0x80u) ? 4u : 0u);
  if (avail < need) return false;
  uint64_t len = l7;
  if (ext) {
    len = 0;
    for (uint32_t i = 0; i < ext; i++) len = (len << 8) | b[2 + i];
  }
  *hlen = need;
  *plen = len;
  return true;
}

// The first frame start at or after the batch start given the carry: after
// the carried payload, or after the frame whose carried header the batch
// completes. U64MAX when the batch holds no frame start.
uint64_t first_start(const uint8_t* p, uint64_t len, const xyws_carry* c) {
  if (!c) return 0;
  if (c->payload_remaining) return c->payload_remaining < len ? c->payload_remaining : U64MAX;
  if (!c->hdr_len) return 0;
  uint8_t hb[XYWS_MAX_FRAME_HEADER_SIZE];
  const uint64_t h0 = c->hdr_len < XYWS_MAX_FRAME_HEADER_SIZE ? c->hdr_len : XYWS_MAX_FRAME_HEADER_SIZE;
  memcpy(hb, c->hdr, h0);
  uint64_t n = h0;
  for (; n < XYWS_MAX_FRAME_HEADER_SIZE && n - h0 < len; n++) hb[n] = p[n - h0];
  uint64_t hl = 0, pl = 0;
  if (!header_span(hb, n, &hl, &pl)) return U64MAX;
  const uint64_t x = sat_add_h(hl - h0, pl);
  return x < len ? x : U64MAX;
}

// Chooses bounds[1..n-1] from an ascending stream of candidate boundaries
// (frame starts, then len): for target t_k = k * len / n the candidate
// nearest to it (the lower one on a tie), never below the previous bound.
struct chooser {
  uint64_t len;
  uint32_t n, k = 1;
  uint64_t* bounds;
  uint64_t prev = U64MAX;  // the last candidate at or below the current target (U64MAX: none yet)
  uint64_t target() const {
    return (uint64_t)(((unsigned __int128)len * k) / n);
  }
  void offer(uint64_t c) {
    while (k < n) {
      const uint64_t t = target();
      if (c <= t) { prev = c; return; }
      // c is the first candidate past t: prev or c, whichever is nearer
      bounds[k] = (prev != U64MAX && t - prev <= c - t) ? prev : c;
      k++;
    }
  }
  void close() {  // (only after len was offered: every target is at most len)
    for (; k < n; k++) bounds[k] = prev != U64MAX ? prev : len;
  }
};

}  // namespace

extern "C" {

int xyws_shard_plan(const void* host_batch, uint64_t len, const xyws_carry* carry_in, uint32_t n_shards,
                    uint64_t* bounds) {
  if (!bounds || !n_shards || (!host_batch && len)) return XYWS_ERR_INVALID;
  const uint8_t* p = static_cast<const uint8_t*>(host_batch);
  bounds[0] = 0;
  bounds[n_shards] = len;
  chooser ch{len, n_shards, 1, bounds};
  for (uint64_t x = first_start(p, len, carry_in); x < len;) {
    ch.offer(x);
    uint64_t hl = 0, pl = 0;
    const uint64_t room = len - x;
    if (!header_span(p + x, room < XYWS_MAX_FRAME_HEADER_SIZE ? room : XYWS_MAX_FRAME_HEADER_SIZE, &hl, &pl))
      break;  // a header cut by the batch end: x was the last start
    x = sat_add_h(x + hl, pl);
  }
  ch.offer(len);
  ch.close();
  return XYWS_OK;
}

int xyws_shard_plan_frames(const xyws_frame* frames, uint64_t n, uint64_t len, uint32_t n_shards,
                           uint64_t* bounds) {
  if (!bounds || !n_shards || (!frames && n)) return XYWS_ERR_INVALID;
  uint64_t last = 0;
  for (uint64_t i = 0; i < n; i++) {  // ascending, inside the batch
    if (frames[i].frame_off < 0) continue;
    const uint64_t x = (uint64_t)frames[i].frame_off;
    if (x < last || x > len) return XYWS_ERR_INVALID;
    last = x;
  }
  bounds[0] = 0;
  bounds[n_shards] = len;
  chooser ch{len, n_shards, 1, bounds};
  for (uint64_t i = 0; i < n; i++)
    if (frames[i].frame_off >= 0 && (uint64_t)frames[i].frame_off < len) ch.offer((uint64_t)frames[i].frame_off);
  ch.offer(len);
  ch.close();
  return XYWS_OK;
}

}  // extern "C"
