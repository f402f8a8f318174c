// xyws/websocket.hpp — header-only C++20 shim over the xyws C-ABI (xyws.h)
// that keeps the names of xynet's WebSocket frame interface, so a
// websocket.h-style caller switches its decode path by include.
//
//   xynet (reference tree)                               here
//   ---------------------------------------------------  ---------------------------------
//   enum class websocket_flags + operators                xyws::websocket_flags (same values)
//     include/xynet/http/websocket_frame_header.h:42-106
//   detail::calc_frame_header_size / calc_frame_size      xyws::detail::calc_frame_header_size
//     :111-131, WS_MAX_FRAME_HEADER_SIZE :134               / calc_frame_size, WS_MAX_FRAME_HEADER_SIZE
//   websocket_mask(R&& data, uint32_t mask, size_t i)     xyws::websocket_mask(ctx, dev span, mask, i)
//     include/xynet/http/websocket_frame_mask.h:6-25        (device memory, in place, returns i+len)
//   websocket_frame_header_parser::result()               xyws::frame::result()
//     :264-267 -> tuple<flags, mask_uint32_t, length>
//   websocket_recv_data: parse -> result -> mask          xyws::frame_decoder::decode
//     example/include/common/websocket.h:110-134            (a whole batch of frames per call)
//
// Nothing here computes on the host: every call goes through libxyws.so to
// HIP kernels for gfx950. Buffers are caller-owned device memory (hipMalloc);
// `stream` is a hipStream_t passed as void*. Errors throw xyws::error.
#pragma once

#include <cstddef>
#include <cstdint>
#include <span>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>

#include "../xyws.h"

namespace xyws {

enum class websocket_flags : unsigned char {
  WS_NONE = 0x0,
  WS_OP_CONTINUE = 0x0,
  WS_OP_TEXT = 0x1,
  WS_OP_BINARY = 0x2,
  WS_OP_CLOSE = 0x8,
  WS_OP_PING = 0x9,
  WS_OP_PONG = 0xA,
  WS_OP_MASK = 0xF,
  WS_FIN = 0x10,
  WS_FINAL_FRAME = 0x10,
  WS_HAS_MASK = 0x20,
};

constexpr websocket_flags operator&(websocket_flags a, websocket_flags b) {
  return websocket_flags(static_cast<unsigned char>(a) & static_cast<unsigned char>(b));
}
constexpr websocket_flags operator|(websocket_flags a, websocket_flags b) {
  return websocket_flags(static_cast<unsigned char>(a) | static_cast<unsigned char>(b));
}
constexpr websocket_flags operator^(websocket_flags a, websocket_flags b) {
  return websocket_flags(static_cast<unsigned char>(a) ^ static_cast<unsigned char>(b));
}
constexpr websocket_flags operator~(websocket_flags a) {
  return websocket_flags(static_cast<unsigned char>(~static_cast<unsigned char>(a)));
}
constexpr websocket_flags& operator&=(websocket_flags& a, websocket_flags b) { return a = a & b; }
constexpr websocket_flags& operator|=(websocket_flags& a, websocket_flags b) { return a = a | b; }
constexpr websocket_flags& operator^=(websocket_flags& a, websocket_flags b) { return a = a ^ b; }
constexpr bool websocket_flags_not_none(websocket_flags f) { return static_cast<unsigned char>(f) != 0; }

namespace detail {
constexpr std::size_t calc_frame_header_size(websocket_flags flags, std::size_t data_len) {
  std::size_t size = 2;
  if (data_len >= 126) size += data_len > 0xFFFF ? 8 : 2;
  if (websocket_flags_not_none(flags & websocket_flags::WS_HAS_MASK)) size += 4;
  return size;
}
constexpr std::size_t calc_frame_size(websocket_flags flags, std::size_t data_len) {
  return data_len + calc_frame_header_size(flags, data_len);
}
}  // namespace detail

inline constexpr std::size_t WS_MAX_FRAME_HEADER_SIZE =
    detail::calc_frame_header_size(websocket_flags::WS_HAS_MASK, 0xFFFFFFFFu);
static_assert(WS_MAX_FRAME_HEADER_SIZE == XYWS_MAX_FRAME_HEADER_SIZE);

class error : public std::runtime_error {
 public:
  error(int code, const char* what)
      : std::runtime_error(std::string(what) + ": " + xyws_strerror(code)), code_(code) {}
  int code() const noexcept { return code_; }

 private:
  int code_;
};

inline void check(int rc, const char* what) {
  if (rc != XYWS_OK) throw error(rc, what);
}

// One context per (thread, device): owns the decoder's device scratch.
class context {
 public:
  explicit context(int device = 0) { check(xyws_ctx_create(device, &h_), "xyws_ctx_create"); }
  ~context() {
    if (h_) xyws_ctx_destroy(h_);
  }
  context(const context&) = delete;
  context& operator=(const context&) = delete;
  context(context&& o) noexcept : h_(std::exchange(o.h_, nullptr)) {}
  context& operator=(context&& o) noexcept {
    if (this != &o) {
      if (h_) xyws_ctx_destroy(h_);
      h_ = std::exchange(o.h_, nullptr);
    }
    return *this;
  }
  // pre-size scratch so later calls allocate nothing (hipGraph capture)
  void reserve(std::uint64_t max_batch_bytes, std::uint64_t max_frames = 0) {
    check(xyws_ctx_reserve(h_, max_batch_bytes, max_frames), "xyws_ctx_reserve");
  }
  std::uint32_t last_device_error() {
    std::uint32_t v = 0;
    check(xyws_ctx_last_device_error(h_, &v), "xyws_ctx_last_device_error");
    return v;
  }
  xyws_ctx* native() const noexcept { return h_; }

 private:
  xyws_ctx* h_ = nullptr;
};

// websocket_mask (websocket_frame_mask.h:6-25) over device bytes: in place,
// data[j] ^= bytes(mask)[(i + j) % 4]; returns i + data.size(). `mask` is
// mask_uint32_t() (the key's wire bytes as a little-endian word).
inline std::size_t websocket_mask(context& ctx, std::span<std::byte> dev_data, std::uint32_t mask,
                                  std::size_t i, void* stream = nullptr) {
  const std::uint8_t key[4] = {std::uint8_t(mask), std::uint8_t(mask >> 8), std::uint8_t(mask >> 16),
                               std::uint8_t(mask >> 24)};
  std::uint64_t out = 0;
  check(xyws_unmask(ctx.native(), dev_data.data(), dev_data.size(), key, i, &out, stream), "xyws_unmask");
  return static_cast<std::size_t>(out);
}

// A decoded frame (device descriptor copied to the host by the caller).
struct frame : xyws_frame {
  websocket_flags flags_() const noexcept { return websocket_flags(xyws_frame::flags); }
  std::uint32_t mask_uint32_t() const noexcept {
    return std::uint32_t(key[0]) | std::uint32_t(key[1]) << 8 | std::uint32_t(key[2]) << 16 |
           std::uint32_t(key[3]) << 24;
  }
  std::size_t length() const noexcept { return static_cast<std::size_t>(payload_len); }
  // websocket_frame_header_parser::result() (:264-267)
  std::tuple<websocket_flags, std::uint32_t, std::size_t> result() const noexcept {
    return {flags_(), mask_uint32_t(), length()};
  }
};
static_assert(sizeof(frame) == sizeof(xyws_frame));

// Batched websocket_recv_data: every frame of each device batch is parsed and
// its payload unmasked in place; a frame or header cut by the batch end
// continues in the next batch through the device-resident carry.
class frame_decoder {
 public:
  // dev_carry: 64 B of caller-owned device memory, zero-filled = fresh stream.
  frame_decoder(context& ctx, xyws_carry* dev_carry, std::uint32_t opts = 0)
      : ctx_(&ctx), carry_(dev_carry), opts_(opts) {}

  // dev_frames (may be empty) receives up to dev_frames.size() descriptors;
  // dev_nframes (nullable device pointer) the frame count.
  void decode(std::span<std::byte> dev_batch, std::span<xyws_frame> dev_frames,
              std::uint64_t* dev_nframes, void* stream = nullptr) {
    check(xyws_decode_stream(ctx_->native(), dev_batch.data(), dev_batch.size(), carry_, carry_,
                             dev_frames.empty() ? nullptr : dev_frames.data(), dev_frames.size(),
                             dev_nframes, opts_, stream),
          "xyws_decode_stream");
  }

  // frames at caller-known offsets (one parser per start, no carry)
  void decode_indexed(std::span<std::byte> dev_batch, const std::uint64_t* dev_starts, std::uint64_t n,
                      xyws_frame* dev_frames, void* stream = nullptr) {
    check(xyws_decode_indexed(ctx_->native(), dev_batch.data(), dev_batch.size(), dev_starts, n, dev_frames,
                              opts_ & XYWS_OPT_PARSE_ONLY, stream),
          "xyws_decode_indexed");
  }

 private:
  context* ctx_;
  xyws_carry* carry_;
  std::uint32_t opts_;
};

}  // namespace xyws
