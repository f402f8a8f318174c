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
//   websocket_mask(R&& data, uint32_t mask, size_t i)     xyws::websocket_mask(data, mask, i): same
//     include/xynet/http/websocket_frame_mask.h:6-25        signature (host or device bytes, done on
//                                                           return); websocket_mask(ctx, dev span,
//                                                           mask, i, stream): asynchronous, device
//   using namespace xynet (websocket.h:17)                namespace xynet = the names below
//   websocket_frame_header_parser::result()               xyws::frame::result()
//     :264-267 -> tuple<flags, mask_uint32_t, length>
//   websocket_recv_data: parse -> result -> mask          xyws::frame_decoder::decode
//     example/include/common/websocket.h:110-134            (a whole batch of frames per call)
//   class websocket_frame_header :179-224                 xyws::websocket_frame_header (same ctors,
//                                                           view(), span(); masked-ctor quirk kept)
//   class websocket_frame_header_parser :226-385          xyws::websocket_frame_header_parser
//     parse / length / flags / mask_uint32_t / result /     (parsed on the device, xyws_parser_*)
//     mask / reset / npos
//   echo_once reply build (websocket_echo.cpp:18-27)      xyws::encode_frames (batched, device)
//   websocket_check_parser_result (websocket.h:81-108)    xyws::classify_frames (device)
//
// Nothing here computes on the host: every call goes through libxyws.so to
// HIP kernels for gfx950. Buffers are caller-owned device memory (hipMalloc);
// `stream` is a hipStream_t passed as void*. Errors throw xyws::error.
#pragma once

#include <array>
#include <concepts>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <ranges>
#include <span>
#include <string_view>
#include <stdexcept>
#include <string>
#include <tuple>
#include <type_traits>
#include <utility>
#include <vector>

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

// The calling thread's context on `device` (what default-constructed parsers
// and the reference-signature websocket_mask use, so `websocket_frame_header_parser{}`
// and `websocket_mask(data_span, mask, 0)` read as in the reference).
inline context& default_context(int device = 0) {
  constexpr int MAXDEV = 64;
  thread_local std::array<context*, MAXDEV> ctxs{};
  if (device < 0 || device >= MAXDEV) device = 0;
  if (!ctxs[device]) {
    thread_local struct owner {
      std::array<context*, MAXDEV>* v;
      ~owner() {
        for (auto* c : *v) delete c;
      }
    } own{&ctxs};
    ctxs[device] = new context(device);
  }
  return *ctxs[device];
}

namespace detail {
// websocket_mask's element types (websocket_frame_mask.h:6-13): anything
// convertible to std::byte, char or unsigned char
template <typename T>
inline constexpr bool mask_element_v = std::is_convertible_v<T, std::byte> || std::is_convertible_v<T, char> ||
                                       std::is_convertible_v<T, unsigned char> || std::is_same_v<T, std::byte>;
// a range the device can XOR where it lies: contiguous bytes
template <typename R>
concept contiguous_bytes = std::ranges::contiguous_range<R> && std::ranges::sized_range<R> &&
                           (sizeof(std::ranges::range_value_t<R>) == 1);
// a range of such pieces behind a view (std::views::join over spans: the
// reference's only multi-piece use, test/playground.cpp:188-189)
template <typename R>
concept joined_pieces = requires(R& r) {
  { r.base() } -> std::ranges::range;
} && contiguous_bytes<std::ranges::range_reference_t<decltype(std::declval<R&>().base())>>;

// one contiguous piece (host or device bytes), on the device of its memory
inline std::size_t mask_piece(void* p, std::size_t n, std::uint32_t mask, std::size_t i) {
  if (n == 0) return i;
  const std::uint8_t key[4] = {std::uint8_t(mask), std::uint8_t(mask >> 8), std::uint8_t(mask >> 16),
                               std::uint8_t(mask >> 24)};
  int dev = -1;
  (void)xyws_pointer_device(p, &dev);
  std::uint64_t out = 0;
  check(xyws_mask_bytes(default_context(dev < 0 ? 0 : dev).native(), p, n, key, i, &out, nullptr),
        "xyws_mask_bytes");
  return static_cast<std::size_t>(out);
}
}  // namespace detail

}  // namespace xyws

// websocket_mask(R&& data, uint32_t mask, size_t i) with the reference's
// signature, scope and contract (websocket_frame_mask.h:6-25, declared in the
// global namespace there too): any range of byte-sized elements, host or
// device memory, unmasked in place when it returns, data[j] ^= bytes(mask)[(i
// + j) % 4]; returns i + the range's length. The XOR runs on the device
// through xyws_mask_bytes (host bytes staged: a compatibility path; batches
// go through xyws::frame_decoder):
//  * a contiguous range: one call where it lies;
//  * a view over contiguous pieces (std::views::join of spans, as
//    test/playground.cpp:188-189 masks two joined spans): one call per piece,
//    the phase carried from piece to piece;
//  * any other range: its elements staged in one host buffer, one call,
//    written back in order.
template <typename R>
  requires std::ranges::range<R> && xyws::detail::mask_element_v<std::ranges::range_value_t<R>>
std::size_t websocket_mask(R&& data, std::uint32_t mask, std::size_t i) {
  using namespace xyws::detail;
  if constexpr (contiguous_bytes<R>) {
    return mask_piece(const_cast<void*>(static_cast<const void*>(std::ranges::data(data))), std::ranges::size(data),
                      mask, i);
  } else if constexpr (joined_pieces<std::remove_reference_t<R>>) {
    for (auto&& piece : data.base())
      i = mask_piece(const_cast<void*>(static_cast<const void*>(std::ranges::data(piece))), std::ranges::size(piece),
                     mask, i);
    return i;
  } else {
    std::vector<unsigned char> stage;
    for (auto&& c : data) stage.push_back(static_cast<unsigned char>(c));
    const std::size_t r = mask_piece(stage.data(), stage.size(), mask, i);
    std::size_t j = 0;
    for (auto it = std::ranges::begin(data); it != std::ranges::end(data); ++it, ++j)
      *it = static_cast<std::ranges::range_value_t<R>>(stage[j]);
    return r;
  }
}

namespace xyws {
// (the same function under the shim's namespace: xyws::websocket_mask(data,
// mask, i) and, through namespace xynet below, the reference's spelling)
using ::websocket_mask;

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

// class websocket_frame_header (websocket_frame_header.h:179-224): a header in
// a 14-byte array. As in the reference, the masked constructors keep the key
// beside the header and build it with the key bytes zero (:183-202); with_key()
// builds the RFC client-role header that carries the key.
class websocket_frame_header {
 public:
  websocket_frame_header(websocket_flags flags, std::size_t data_len) noexcept {
    len_ = static_cast<std::size_t>(
        xyws_header_build(static_cast<std::uint8_t>(flags), nullptr, data_len, hdr_.data()));
  }
  websocket_frame_header(websocket_flags flags, std::span<char, 4> mask, std::size_t data_len) noexcept
      : websocket_frame_header{flags, data_len} {
    std::memcpy(mask_.data(), mask.data(), 4);
  }
  websocket_frame_header(websocket_flags flags, std::uint32_t mask, std::size_t data_len) noexcept
      : websocket_frame_header{flags, data_len} {
    std::memcpy(mask_.data(), &mask, 4);
  }
  static websocket_frame_header with_key(websocket_flags flags, std::uint32_t key, std::size_t data_len) noexcept {
    websocket_frame_header h{flags | websocket_flags::WS_HAS_MASK, data_len};
    std::uint8_t k[4];
    std::memcpy(k, &key, 4);
    h.len_ = static_cast<std::size_t>(xyws_header_build(
        static_cast<std::uint8_t>(flags | websocket_flags::WS_HAS_MASK), k, data_len, h.hdr_.data()));
    std::memcpy(h.mask_.data(), &key, 4);
    return h;
  }
  [[nodiscard]] std::string_view view() const {
    return {reinterpret_cast<const char*>(hdr_.data()), len_};
  }
  [[nodiscard]] std::span<const std::byte> span() const {
    return {reinterpret_cast<const std::byte*>(hdr_.data()), len_};
  }

 private:
  std::array<std::uint8_t, XYWS_MAX_FRAME_HEADER_SIZE> hdr_ = {};
  std::array<char, 4> mask_ = {};
  std::size_t len_ = 0;
};

// class websocket_frame_header_parser (websocket_frame_header.h:226-385). parse()
// takes host or device bytes and returns the bytes consumed in this call up to
// the end of the header, or npos while it is incomplete; after a complete
// header it returns npos until reset(). The parse runs on the device (the
// stream decoder in parse-only mode, device-resident carry); it is synchronous
// on `stream`. Unlike the reference it can throw xyws::error (a HIP failure).
class websocket_frame_header_parser {
 public:
  static constexpr std::size_t npos = static_cast<std::size_t>(-1);

  websocket_frame_header_parser() : websocket_frame_header_parser(default_context()) {}
  explicit websocket_frame_header_parser(context& ctx, void* stream = nullptr) : stream_(stream) {
    check(xyws_parser_create(ctx.native(), &p_), "xyws_parser_create");
  }
  ~websocket_frame_header_parser() {
    if (p_) xyws_parser_destroy(p_);
  }
  websocket_frame_header_parser(const websocket_frame_header_parser&) = delete;
  websocket_frame_header_parser& operator=(const websocket_frame_header_parser&) = delete;
  websocket_frame_header_parser(websocket_frame_header_parser&& o) noexcept
      : p_(std::exchange(o.p_, nullptr)), stream_(o.stream_) {}

  std::size_t parse(std::string_view str) { return parse_bytes(str.data(), str.size()); }
  template <typename T, std::size_t Extent>
  std::size_t parse(std::span<T, Extent> sp) {
    const auto b = std::as_bytes(sp);
    return parse_bytes(b.data(), b.size());
  }

  std::size_t length() const noexcept { return static_cast<std::size_t>(get().payload_len); }
  websocket_flags flags() const noexcept { return websocket_flags(get().flags); }
  std::uint32_t mask_uint32_t() const noexcept {
    const xyws_frame f = get();
    std::uint32_t m;
    std::memcpy(&m, f.key, 4);  // wire bytes reinterpreted as a host int (:259-262)
    return m;
  }
  std::tuple<websocket_flags, std::uint32_t, std::size_t> result() const noexcept {
    return {flags(), mask_uint32_t(), length()};
  }
  std::array<char, 4> mask() const noexcept {
    const xyws_frame f = get();
    std::array<char, 4> m;
    std::memcpy(m.data(), f.key, 4);
    return m;
  }
  void reset() { check(xyws_parser_reset(p_), "xyws_parser_reset"); }

 private:
  std::size_t parse_bytes(const void* data, std::size_t len) {
    std::uint64_t consumed = XYWS_NPOS;
    check(xyws_parser_parse(p_, data, len, &consumed, stream_), "xyws_parser_parse");
    return consumed == XYWS_NPOS ? npos : static_cast<std::size_t>(consumed);
  }
  xyws_frame get() const noexcept {
    xyws_frame f{};
    std::uint64_t len = 0;
    (void)xyws_parser_result(p_, &f.flags, f.key, &len);
    f.payload_len = len;
    return f;
  }

  xyws_parser* p_ = nullptr;
  void* stream_ = nullptr;
};

// Batched echo replies / client-role frames on the device (xyws_encode_frames).
inline void encode_frames(context& ctx, std::span<const std::byte> dev_src, std::span<const xyws_frame> dev_frames,
                          const std::uint64_t* dev_n, websocket_flags flags, std::span<std::byte> dev_out,
                          std::uint64_t* dev_out_len, std::uint32_t enc_opts = 0,
                          const std::uint8_t* dev_keys = nullptr, const xyws_verdict* dev_verdicts = nullptr,
                          std::uint32_t action_mask = 0, std::uint64_t* dev_offsets = nullptr,
                          void* stream = nullptr) {
  check(xyws_encode_frames(ctx.native(), dev_src.data(), dev_src.size(), dev_frames.data(), dev_frames.size(), dev_n,
                           static_cast<std::uint8_t>(flags), enc_opts, dev_keys, dev_verdicts, action_mask,
                           dev_out.data(), dev_out.size(), dev_offsets, dev_out_len, stream),
        "xyws_encode_frames");
}

// websocket_check_parser_result's policy per frame (xyws_classify_frames).
inline void classify_frames(context& ctx, std::span<const std::byte> dev_src, std::span<const xyws_frame> dev_frames,
                            const std::uint64_t* dev_n, std::uint64_t max_payload, std::uint32_t policy,
                            xyws_verdict* dev_verdicts, std::uint64_t* dev_first_close, void* stream = nullptr) {
  check(xyws_classify_frames(ctx.native(), dev_src.data(), dev_src.size(), dev_frames.data(), dev_frames.size(),
                             dev_n, max_payload, policy, dev_verdicts, dev_first_close, stream),
        "xyws_classify_frames");
}

}  // namespace xyws

// The reference's namespace (websocket_frame_header.h, `using namespace xynet`
// at example/include/common/websocket.h:17): its frame names resolve to the
// ones above, so a caller switches by include.
namespace xynet {
using namespace ::xyws;
}
