// test_shim.cpp — C++ callers of include/xyws/websocket.hpp on a real device.
//
// Written for this build (not taken from the reference): it exercises the
// shim the way xynet's own header test does (test/websocket_frame_test.cpp:
// 10-65, the header round trip for 9 flag/length cases; :67-89, the header
// fed in two parts split at every byte) and the way the example's receive loop
// uses the parser (example/include/common/websocket.h:110-134: parse ->
// result -> websocket_mask), with every expected value read from a plain-text
// rendering of tests/golden/frame_header.json (written by the pytest driver,
// tests/test_cpp_shim.py) so this program hard-codes no answers.
//
// usage: test_shim <vectors.txt>; prints one line per failure and "ok <n>".
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "xyws/websocket.hpp"

using namespace xyws;

static int fails = 0, checks = 0;
#define EXPECT(c, ...)                       \
  do {                                       \
    checks++;                                \
    if (!(c)) {                              \
      fails++;                               \
      std::printf("FAIL %s:%d ", __FILE__, __LINE__); \
      std::printf(__VA_ARGS__);              \
      std::printf("\n");                     \
    }                                        \
  } while (0)

static std::string hex(std::span<const std::byte> s) {
  std::string o;
  char b[3];
  for (auto x : s) {
    std::snprintf(b, sizeof b, "%02x", static_cast<unsigned>(x));
    o += b;
  }
  return o;
}

static std::vector<std::uint8_t> unhex(const std::string& h) {
  std::vector<std::uint8_t> v;
  for (std::size_t i = 0; i + 1 < h.size(); i += 2) v.push_back((std::uint8_t)std::stoul(h.substr(i, 2), nullptr, 16));
  return v;
}

// `case <flags> <length> <header hex> <ret> <r_flags> <r_length>`: one header
// round trip through a fresh parser (websocket_frame_test.cpp:59-64)
static void round_trip(std::istringstream& in) {
  unsigned flags;
  unsigned long long length, ret, r_length;
  unsigned r_flags;
  std::string hdr;
  in >> flags >> length >> hdr >> ret >> r_flags >> r_length;
  auto header = websocket_frame_header{websocket_flags(flags), (std::size_t)length};
  EXPECT(hex(header.span()) == hdr, "header %s != %s", hex(header.span()).c_str(), hdr.c_str());
  auto parser = websocket_frame_header_parser{};
  auto got = parser.parse(header.span());
  EXPECT(got == ret && got == header.span().size(), "parse returned %zu, want %llu", got, ret);
  EXPECT((unsigned)parser.flags() == r_flags, "flags %u want %u", (unsigned)parser.flags(), r_flags);
  EXPECT(parser.length() == r_length, "length %zu want %llu", parser.length(), r_length);
  // a completed parser returns npos until reset() (websocket_frame_header.h:378-384)
  EXPECT(parser.parse(header.span()) == websocket_frame_header_parser::npos, "second parse not npos");
  parser.reset();
  EXPECT(parser.parse(header.span()) == ret, "parse after reset");
}

// `split <flags> <length> <split> <ret1> <ret2> <r_flags> <r_length>`
// (websocket_frame_test.cpp:75-89)
static void split(std::istringstream& in) {
  unsigned flags, r_flags;
  unsigned long long length, at, ret1, ret2, r_length;
  in >> flags >> length >> at >> ret1 >> ret2 >> r_flags >> r_length;
  auto header = websocket_frame_header{websocket_flags(flags), (std::size_t)length};
  auto n = header.span().size();
  auto span1 = std::span{header.span().data(), (std::size_t)at};
  auto span2 = std::span{header.span().data() + at, n - at};
  auto parser = websocket_frame_header_parser{};
  auto r1 = parser.parse(span1);
  EXPECT((unsigned long long)r1 == ret1, "split %llu: ret1 %zu want %llu", at, r1, ret1);
  auto r2 = parser.parse(span2);
  EXPECT((unsigned long long)r2 == ret2, "split %llu: ret2 %zu want %llu", at, r2, ret2);
  EXPECT((unsigned)parser.flags() == r_flags, "split %llu: flags", at);
  EXPECT(parser.length() == r_length, "split %llu: length", at);
}

// `build <flags> <length> <key hex> <built_nokey hex> <ctor_masked hex> <built hex>`
// (detail::websocket_frame_header_builder :136-175 and the class's ctors :183-202)
static void build(std::istringstream& in) {
  unsigned flags;
  unsigned long long length;
  std::string key, nokey, masked, built;
  in >> flags >> length >> key >> nokey >> masked >> built;
  auto k = unhex(key);
  std::uint32_t kw;
  std::memcpy(&kw, k.data(), 4);
  auto h1 = websocket_frame_header{websocket_flags(flags), (std::size_t)length};
  EXPECT(hex(h1.span()) == nokey, "build %u %llu: %s != %s", flags, length, hex(h1.span()).c_str(), nokey.c_str());
  auto h2 = websocket_frame_header{websocket_flags(flags), kw, (std::size_t)length};
  EXPECT(hex(h2.span()) == masked, "ctor_masked %u %llu", flags, length);
  if (flags & XYWS_FLAG_HAS_MASK) {
    auto h3 = websocket_frame_header::with_key(websocket_flags(flags), kw, (std::size_t)length);
    EXPECT(hex(h3.span()) == built, "with_key %u %llu: %s != %s", flags, length, hex(h3.span()).c_str(),
           built.c_str());
  }
}

// The example's receive loop (websocket.h:116-133) over DEVICE bytes: the
// frame arrives in two pieces (the header cut after 3 bytes), parse() from the
// device buffer, result(), then websocket_mask on the payload span in place.
static void recv_loop() {
  const char* text = "Hello from the device parser";
  const std::size_t plen = std::strlen(text);
  const std::uint32_t key = 0x3d21fa37u;  // wire bytes 37 fa 21 3d
  auto hdr = websocket_frame_header::with_key(websocket_flags::WS_FIN | websocket_flags::WS_OP_TEXT, key, plen);
  std::vector<std::uint8_t> wire(hdr.span().size() + plen);
  std::memcpy(wire.data(), hdr.span().data(), hdr.span().size());
  for (std::size_t j = 0; j < plen; j++)
    wire[hdr.span().size() + j] = (std::uint8_t)text[j] ^ (std::uint8_t)(key >> (8 * (j % 4)));
  std::byte* dev = nullptr;
  EXPECT(hipMalloc(&dev, 1024) == hipSuccess, "hipMalloc");
  EXPECT(hipMemcpy(dev, wire.data(), wire.size(), hipMemcpyHostToDevice) == hipSuccess, "H2D");
  auto parser = websocket_frame_header_parser{};
  std::size_t recv_bytes = 3, ret = websocket_frame_header_parser::npos, fed = 0;
  while (true) {
    ret = parser.parse(std::span{dev + fed, recv_bytes - fed});
    if (ret != websocket_frame_header_parser::npos) {
      ret += fed;  // bytes of this buffer before the header end
      break;
    }
    fed = recv_bytes;
    recv_bytes = wire.size();
  }
  auto [flags, mask, length] = parser.result();
  EXPECT(ret == hdr.span().size(), "recv loop: header end %zu", ret);
  EXPECT(flags == (websocket_flags::WS_FIN | websocket_flags::WS_OP_TEXT | websocket_flags::WS_HAS_MASK),
         "recv loop: flags %u", (unsigned)flags);
  EXPECT(mask == key, "recv loop: mask %08x", mask);
  EXPECT(length == plen, "recv loop: length");
  auto& ctx = default_context();
  auto next = websocket_mask(ctx, std::span{dev + ret, length}, mask, 0);
  EXPECT(next == length, "websocket_mask returned %zu", next);
  std::vector<char> back(plen);
  EXPECT(hipDeviceSynchronize() == hipSuccess, "sync");
  EXPECT(hipMemcpy(back.data(), dev + ret, plen, hipMemcpyDeviceToHost) == hipSuccess, "D2H");
  EXPECT(std::memcmp(back.data(), text, plen) == 0, "unmasked payload differs");
  EXPECT(default_context().last_device_error() == 0, "device error word");
  (void)hipFree(dev);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s vectors.txt\n", argv[0]);
    return 2;
  }
  std::ifstream f(argv[1]);
  std::string line;
  int n = 0;
  while (std::getline(f, line)) {
    std::istringstream in(line);
    std::string kind;
    in >> kind;
    if (kind == "case") round_trip(in);
    else if (kind == "split") split(in);
    else if (kind == "build") build(in);
    else continue;
    n++;
  }
  recv_loop();
  std::printf("vectors %d checks %d failures %d\n", n, checks, fails);
  if (fails) return 1;
  std::printf("ok %d\n", n);
  return 0;
}
