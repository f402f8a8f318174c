// ref_harness.cpp — C-ABI harness around the REAL reference headers.
//
// CONTAINER-ONLY TEST INFRASTRUCTURE. It #includes the reference's two hot-path
// headers where they lie (/root/reference/include, passed with -I by
// oracle/Makefile); no reference source is copied into this repository. The
// built library goes to oracle/_ref/ (git-ignored) and travels to the GPU box
// as a prebuilt .so, where bench.py's cpu_baseline leg times it
// (cpu_baseline.kind = "reference"). tests/golden/gen_golden.py uses it to
// produce the golden vectors that pin oracle/xyws_oracle.c.
//
// The headers define non-inline functions (websocket_frame_header.h:136,305),
// so they are included in exactly this one translation unit.
#include <cstdint>
#include <cstring>
#include <span>
#include <thread>
#include <vector>

#include "xynet/http/websocket_frame_header.h"
#include "xynet/http/websocket_frame_mask.h"

#include "xyws.h"  // only for the xyws_frame / xyws_carry layouts

using xynet::websocket_flags;
using xynet::websocket_frame_header;
using xynet::websocket_frame_header_parser;

extern "C" {

// ---- parser object (websocket_frame_header.h:226-303) ----------------------
void* ref_parser_new() { return new websocket_frame_header_parser{}; }
void ref_parser_free(void* p) { delete static_cast<websocket_frame_header_parser*>(p); }
void ref_parser_reset(void* p) { static_cast<websocket_frame_header_parser*>(p)->reset(); }

// parse(span<const byte>) :237-247 (the span<char> overload does not compile)
uint64_t ref_parser_parse(void* p, const uint8_t* data, uint64_t len) {
  auto sp = std::span<const std::byte>{reinterpret_cast<const std::byte*>(data), len};
  return static_cast<websocket_frame_header_parser*>(p)->parse(sp);
}

// result() :264-267 -> (flags, mask_uint32_t(), length()); mask() :269 wire bytes
void ref_parser_result(void* p, uint8_t* flags, uint32_t* mask_u32, uint64_t* length,
                       uint8_t* mask_bytes) {
  auto* q = static_cast<websocket_frame_header_parser*>(p);
  auto [f, m, l] = q->result();
  *flags = static_cast<uint8_t>(f);
  *mask_u32 = m;
  *length = l;
  auto mb = q->mask();
  std::memcpy(mask_bytes, mb.data(), 4);
}

// ---- websocket_mask (websocket_frame_mask.h:6-25) -------------------------
uint64_t ref_mask(uint8_t* data, uint64_t len, uint32_t mask, uint64_t i) {
  auto sp = std::span<std::byte>{reinterpret_cast<std::byte*>(data), len};
  return websocket_mask(sp, mask, i);
}

// ---- builder / header class (websocket_frame_header.h:136-224) ------------
uint64_t ref_header_build(uint8_t* out, uint8_t flags, const uint8_t* mask, uint64_t len) {
  return xynet::detail::websocket_frame_header_builder(
      out, static_cast<websocket_flags>(flags), reinterpret_cast<const char*>(mask), len);
}

uint64_t ref_header_ctor(uint8_t* out, uint8_t flags, uint64_t len) {
  auto h = websocket_frame_header{static_cast<websocket_flags>(flags), len};
  auto sp = h.span();
  std::memcpy(out, sp.data(), sp.size());
  return sp.size();
}

uint64_t ref_header_ctor_masked(uint8_t* out, uint8_t flags, uint32_t mask, uint64_t len) {
  auto h = websocket_frame_header{static_cast<websocket_flags>(flags), mask, len};
  auto sp = h.span();
  std::memcpy(out, sp.data(), sp.size());
  return sp.size();
}

uint64_t ref_calc_frame_header_size(uint8_t flags, uint64_t len) {
  return xynet::detail::calc_frame_header_size(static_cast<websocket_flags>(flags), len);
}

// ---- batch decode composed from the reference primitives -------------------
// The websocket_recv_data shape (example/include/common/websocket.h:110-134)
// applied to a back-to-back batch: fresh parser per frame, parse, result(),
// websocket_mask(payload, mask_uint32_t(), 0), with the carry semantics of
// xyws.h. Frame status bits are not computed here (the reference has none).
uint64_t ref_decode_stream(uint8_t* buf, uint64_t len, const xyws_carry* cin, xyws_carry* cout,
                           xyws_frame* frames, uint64_t cap) {
  xyws_carry c{};
  if (cin) c = *cin;
  uint64_t pos = 0, n = 0;
  if (c.payload_remaining) {
    uint64_t take = c.payload_remaining < len ? c.payload_remaining : len;
    uint32_t k;
    std::memcpy(&k, c.key, 4);
    c.phase = websocket_mask(std::span<std::byte>{reinterpret_cast<std::byte*>(buf), take}, k,
                             c.phase);
    c.payload_remaining -= take;
    pos = take;
    if (!c.payload_remaining) {
      c.phase = 0;
      std::memset(c.key, 0, 4);
    }
  }
  while (pos < len) {
    websocket_frame_header_parser parser{};
    int64_t frame_off = static_cast<int64_t>(pos);
    uint32_t h0 = c.hdr_len;
    if (h0) {
      parser.parse(std::span<const std::byte>{reinterpret_cast<const std::byte*>(c.hdr), h0});
      frame_off -= h0;
    }
    auto r = parser.parse(
        std::span<const std::byte>{reinterpret_cast<const std::byte*>(buf + pos), len - pos});
    if (r == websocket_frame_header_parser::npos) {
      std::memcpy(c.hdr + h0, buf + pos, len - pos);
      c.hdr_len = static_cast<uint8_t>(h0 + (len - pos));
      pos = len;
      break;
    }
    auto [flags, mask, plen] = parser.result();
    xyws_frame f{};
    f.frame_off = frame_off;
    f.payload_off = static_cast<int64_t>(pos + r);
    f.payload_len = plen;
    auto mb = parser.mask();
    std::memcpy(f.key, mb.data(), 4);
    f.flags = static_cast<uint8_t>(flags);
    f.hdr_len = static_cast<uint8_t>(h0 + r);
    c.hdr_len = 0;
    std::memset(c.hdr, 0, sizeof c.hdr);
    uint64_t ps = pos + r, avail = len - ps;
    if (plen <= avail) {
      websocket_mask(std::span<std::byte>{reinterpret_cast<std::byte*>(buf + ps), plen}, mask, 0);
      pos = ps + plen;
    } else {
      c.phase = websocket_mask(std::span<std::byte>{reinterpret_cast<std::byte*>(buf + ps), avail},
                               mask, 0);
      c.payload_remaining = plen - avail;
      std::memcpy(c.key, mb.data(), 4);
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

// CPU baseline on `threads` host threads: one thread walks the headers with
// the reference parser (boundary discovery is serial by nature), then the
// frames' payloads are unmasked with websocket_mask by `threads` workers that
// split the frames into byte-balanced contiguous ranges. Whole frames only:
// a trailing partial frame is ignored (the bench feeds whole-frame samples).
// Returns the frame count.
uint64_t ref_decode_batch_mt(uint8_t* buf, uint64_t len, int threads) {
  struct fr { uint64_t ps, plen; uint32_t mask; };
  std::vector<fr> fs;
  uint64_t pos = 0;
  while (pos < len) {
    websocket_frame_header_parser parser{};
    auto r = parser.parse(
        std::span<const std::byte>{reinterpret_cast<const std::byte*>(buf + pos), len - pos});
    if (r == websocket_frame_header_parser::npos) break;
    auto [flags, mask, plen] = parser.result();
    (void)flags;
    if (plen > len - (pos + r)) break;
    fs.push_back({pos + r, plen, mask});
    pos += r + plen;
  }
  if (threads < 1) threads = 1;
  auto work = [&](size_t a, size_t b) {
    for (size_t i = a; i < b; i++)
      websocket_mask(std::span<std::byte>{reinterpret_cast<std::byte*>(buf + fs[i].ps), fs[i].plen},
                     fs[i].mask, 0);
  };
  if (threads == 1 || fs.size() < 2) {
    work(0, fs.size());
    return fs.size();
  }
  std::vector<std::thread> ts;
  uint64_t total = pos, per = total / threads + 1;
  size_t a = 0;
  for (int t = 0; t < threads && a < fs.size(); t++) {
    size_t b = a;
    uint64_t lim = (uint64_t)(t + 1) * per;
    while (b < fs.size() && (fs[b].ps < lim || b == a)) b++;
    if (t == threads - 1) b = fs.size();
    ts.emplace_back(work, a, b);
    a = b;
  }
  for (auto& t : ts) t.join();
  return fs.size();
}

}  // extern "C"
