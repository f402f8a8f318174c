// Loopback echo harness over the xyws C-ABI (SURVEY.md §8(d), config 1's
// optional leg: "the build's own loopback echo harness with <=1000 B frames").
//
// What the reference's server does per frame (example/websocket/websocket_echo.cpp:18-27:
// echo_once = websocket_recv_data + a FIN|TEXT header + send; the close policy of
// example/include/common/websocket.h:81-108: close frame -> 1000, FIN=0 -> 1003,
// unmasked -> 1008, length > MAX_WEBSOCKET_APP_DATA_LEN (1000, :15) -> 1009),
// done here per recv batch on the GPU:
//
//   recv_some into a pinned buffer (as many bytes as the socket holds)
//   -> H2D -> xyws_decode_stream (boundaries, unmask in place, frame table)
//   -> xyws_classify_frames (max_payload 1000, the reference's checks in its
//      order, its bit-3 close test included: XYWS_POL_REFERENCE)
//   -> xyws_encode_frames (one FIN|TEXT reply per data frame, unmasked server
//      frame, as echo_once sends whatever the frame was)
//   -> D2H of the replies -> send, then a close frame with the first close code.
// The reference's test `flags & WS_OP_CLOSE` (websocket.h:87) is bit 3 of the
// opcode, so it answers a ping (0x9), a pong (0xA) or opcodes 0xB-0xF with
// close 1000; that is what this server does by default. `--rfc` departs from
// the reference on purpose: pings get pongs carrying their payload, replies
// keep the frame's own opcode, only a close frame closes 1000.
// A header that announces more than 1000 payload bytes closes 1009 as soon as
// the header is in (the reference checks before it receives the payload),
// even when the frame's payload is still on its way.
//
// A frame cut by the recv boundary is kept (still masked) at the front of the
// host buffer and decoded again with the next bytes, so every batch decodes
// from a frame start (dev_carry_in = NULL). The HTTP upgrade handshake
// (SHA-1/base64, websocket_request_handler.h) is out of scope: the
// client starts sending frames right after connect.
//
// The client (two threads: sender, receiver) builds a stream of masked text
// frames (random ASCII, lengths uniform in [0, max_len]), optional pings and a
// closing frame, sends it in writes of `--chunk` bytes, and checks the whole
// reply stream byte for byte against the replies the reference's echo would
// send. One JSON line on stdout; exit status 0 only when the bytes match.
//
//   echo_loopback [--frames N] [--max-len L] [--chunk B] [--ping-every K]
//                 [--oversize] [--oversize-len L] [--seed S] [--buf BYTES]
//                 [--opts DECODE_OPTS] [--rfc]
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "xyws.h"

namespace {

struct opts_t {
  uint64_t frames = 20000, max_len = 1000, chunk = 64 << 10, ping_every = 0, seed = 0x5EED0001, buf = 4 << 20,
           opts = 0, oversize_len = 1001;
  bool oversize = false, rfc = false;
};

[[noreturn]] void die(const char* what, long rc = 0) {
  std::fprintf(stderr, "echo_loopback: %s (%ld)\n", what, rc);
  std::exit(2);
}
#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) die(#x, (long)e_); } while (0)
#define XYCHK(x) do { int r_ = (x); if (r_ != XYWS_OK) die(#x, (long)r_); } while (0)

void send_all(int fd, const uint8_t* p, size_t n) {
  while (n) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k <= 0) die("send", (long)k);
    p += k;
    n -= (size_t)k;
  }
}

void append_frame(std::vector<uint8_t>& out, uint8_t flags, const uint8_t* key, const uint8_t* payload,
                  uint64_t len) {
  uint8_t h[XYWS_MAX_FRAME_HEADER_SIZE];
  uint64_t hl = xyws_header_build(flags, key, len, h);
  out.insert(out.end(), h, h + hl);
  size_t at = out.size();
  out.insert(out.end(), payload, payload + len);
  if (key)
    for (uint64_t i = 0; i < len; ++i) out[at + i] ^= key[i & 3];  // websocket_mask, phase 0
}

// The client's stream and the reply stream the reference's echo would send
// (or, with --rfc, an RFC 6455 server: pongs for pings).
void build_streams(const opts_t& o, std::vector<uint8_t>& wire, std::vector<uint8_t>& expect, uint64_t& payload,
                   uint64_t& echoes, uint16_t& code) {
  std::mt19937_64 rng(o.seed);
  std::vector<uint8_t> p;
  payload = 0;
  echoes = 0;
  code = 0;
  for (uint64_t i = 0; i < o.frames; ++i) {
    bool ping = o.ping_every && (i % o.ping_every) == o.ping_every - 1;
    uint64_t len = rng() % ((ping ? std::min<uint64_t>(o.max_len, 125) : o.max_len) + 1);
    if (o.oversize && i == o.frames - 1) len = o.oversize_len;
    p.resize(len);
    for (auto& b : p) b = (uint8_t)(0x20 + rng() % 95);
    uint8_t key[4];
    uint32_t k = (uint32_t)rng();
    std::memcpy(key, &k, 4);
    uint8_t op = ping ? XYWS_FLAG_OP_PING : XYWS_FLAG_OP_TEXT;
    append_frame(wire, op | XYWS_FLAG_FIN | XYWS_FLAG_HAS_MASK, key, p.data(), len);
    if (ping && !o.rfc && !code) code = 1000;  // the reference closes on a ping (websocket.h:87)
    if (len > 1000 && !code) code = 1009;      // the server closes with 1009 here
    if (code) break;                           // (the server has closed: the client stops here)
    append_frame(expect, (ping ? XYWS_FLAG_OP_PONG : XYWS_FLAG_OP_TEXT) | XYWS_FLAG_FIN, nullptr, p.data(), len);
    payload += len;
    echoes++;
  }
  if (!code) {
    code = 1000;
    uint8_t key[4] = {0x11, 0x22, 0x33, 0x44}, be[2] = {0x03, 0xE8};
    append_frame(wire, XYWS_FLAG_OP_CLOSE | XYWS_FLAG_FIN | XYWS_FLAG_HAS_MASK, key, be, 2);
  }
  uint8_t be[2] = {(uint8_t)(code >> 8), (uint8_t)code};
  append_frame(expect, XYWS_FLAG_OP_CLOSE | XYWS_FLAG_FIN, nullptr, be, 2);  // websocket_send_close (:67-76)
}

struct server_stats {
  uint64_t batches = 0, frames = 0, max_batch = 0, early_close = 0;
  uint16_t close_code = 0;
};

// One connection, the GPU pipeline per recv batch.
void serve(int fd, uint64_t B, uint32_t opts, bool rfc, server_stats& st) {
  xyws_ctx* ctx = nullptr;
  XYCHK(xyws_ctx_create(0, &ctx));
  const uint64_t cap = B / 6 + 2;  // a masked frame is >= 6 bytes
  XYCHK(xyws_ctx_reserve(ctx, B, cap));
  hipStream_t s;
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint8_t *hin, *hout, *din, *dout;
  HIPCHK(hipHostMalloc((void**)&hin, B));
  HIPCHK(hipHostMalloc((void**)&hout, B + 16));
  HIPCHK(hipMalloc((void**)&din, B));
  HIPCHK(hipMalloc((void**)&dout, B + 16));
  xyws_frame* dframes;
  xyws_verdict* dverd;
  xyws_carry* dcarry;
  uint64_t* dsc;  // [0] nframes, [1] first_close, [2] out_len
  uint64_t *doffs, *hoffs;  // reply offsets (cap + 1)
  HIPCHK(hipMalloc((void**)&dframes, cap * sizeof(xyws_frame)));
  HIPCHK(hipMalloc((void**)&dverd, cap * sizeof(xyws_verdict)));
  HIPCHK(hipMalloc((void**)&dcarry, sizeof(xyws_carry)));
  HIPCHK(hipMalloc((void**)&dsc, 4 * sizeof(uint64_t)));
  HIPCHK(hipMalloc((void**)&doffs, (cap + 1) * sizeof(uint64_t)));
  HIPCHK(hipHostMalloc((void**)&hoffs, (cap + 1) * sizeof(uint64_t)));
  struct small_t { uint64_t sc[4]; xyws_carry carry; xyws_frame last; xyws_verdict v; } *hs;
  HIPCHK(hipHostMalloc((void**)&hs, sizeof(small_t)));

  uint64_t filled = 0;
  for (;;) {
    ssize_t k = ::recv(fd, hin + filled, B - filled, 0);
    if (k <= 0) break;  // peer closed
    filled += (uint64_t)k;
    while (filled < B) {  // take what else the socket already holds
      k = ::recv(fd, hin + filled, B - filled, MSG_DONTWAIT);
      if (k <= 0) break;
      filled += (uint64_t)k;
    }
    HIPCHK(hipMemcpyAsync(din, hin, filled, hipMemcpyHostToDevice, s));
    XYCHK(xyws_decode_stream(ctx, din, filled, nullptr, dcarry, dframes, cap, dsc, opts, s));
    HIPCHK(hipMemcpyAsync(hs->sc, dsc, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&hs->carry, dcarry, sizeof(xyws_carry), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    uint64_t nfr = hs->sc[0];
    if (nfr > cap) die("frame table overflow", (long)nfr);
    uint64_t complete = nfr;
    const bool cut = hs->carry.payload_remaining != 0;  // the last frame's payload continues past the batch
    if (cut) {
      complete = nfr - 1;
      HIPCHK(hipMemcpyAsync(&hs->last, dframes + complete, sizeof(xyws_frame), hipMemcpyDeviceToHost, s));
      if (!complete) HIPCHK(hipStreamSynchronize(s));  // (else read after the batch's next sync)
    }
    bool closing = false;
    // frames with a complete header: every complete frame, and the cut one
    // (its header alone decides a close: the reference checks the header
    // before it receives the payload, websocket.h:117-128)
    const uint64_t nchk = nfr;
    if (nchk) {
      // one more round trip for the batch: classify, encode every complete
      // frame (offsets per reply), copy back the replies (a server reply is
      // never longer than the client frame it answers: <= filled bytes), the
      // offsets and the first close index; the replies up to that index go out
      st.batches++;
      st.frames += complete;
      if (complete > st.max_batch) st.max_batch = complete;
      const uint32_t policy = rfc ? 0u : XYWS_POL_REFERENCE;
      XYCHK(xyws_classify_frames(ctx, din, filled, dframes, nchk, nullptr, 1000, policy, dverd, dsc + 1, s));
      if (complete) {
        const uint8_t flags = rfc ? 0 : (XYWS_FLAG_FIN | XYWS_FLAG_OP_TEXT);
        const uint32_t acts = rfc ? (1u << XYWS_ACT_DATA) | (1u << XYWS_ACT_PING) : (1u << XYWS_ACT_DATA);
        XYCHK(xyws_encode_frames(ctx, din, filled, dframes, complete, nullptr, flags, rfc ? XYWS_ENC_FRAME_OPCODE : 0,
                                 nullptr, dverd, acts, dout, B + 16, doffs, dsc + 2, s));
        HIPCHK(hipMemcpyAsync(hoffs, doffs, (complete + 1) * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(hout, dout, filled, hipMemcpyDeviceToHost, s));
      } else {
        HIPCHK(hipMemsetAsync(dsc + 2, 0, 8, s));
      }
      HIPCHK(hipMemcpyAsync(&hs->sc[1], dsc + 1, 16, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      const uint64_t first_close = hs->sc[1], out_len = hs->sc[2];
      if (out_len > filled) die("reply longer than the batch", (long)out_len);
      const uint64_t reply_len = first_close < complete ? hoffs[first_close] : out_len;
      if (reply_len) send_all(fd, hout, reply_len);
      if (first_close < nchk) {
        if (first_close == complete) st.early_close = 1;  // (closed on the cut frame's header)
        HIPCHK(hipMemcpyAsync(&hs->v, dverd + first_close, sizeof(xyws_verdict), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        st.close_code = hs->v.close_code;
        uint8_t c[4] = {XYWS_FLAG_OP_CLOSE | 0x80, 2, (uint8_t)(st.close_code >> 8), (uint8_t)st.close_code};
        send_all(fd, c, 4);
        closing = true;
      }
    }
    if (closing) break;
    const uint64_t tail = cut ? (uint64_t)hs->last.frame_off : filled - hs->carry.hdr_len;
    std::memmove(hin, hin + tail, filled - tail);
    filled -= tail;
    if (filled == B) die("a frame larger than the receive buffer");
  }
  uint32_t derr = 0;
  xyws_ctx_last_device_error(ctx, &derr);
  if (derr) die("device error word", (long)derr);
  ::shutdown(fd, SHUT_WR);
  (void)hipHostFree(hin); (void)hipHostFree(hout); (void)hipHostFree(hs); (void)hipHostFree(hoffs);
  (void)hipFree(doffs); (void)hipFree(din); (void)hipFree(dout); (void)hipFree(dframes); (void)hipFree(dverd);
  (void)hipFree(dcarry); (void)hipFree(dsc);
  (void)hipStreamDestroy(s);
  xyws_ctx_destroy(ctx);
}

}  // namespace

int main(int argc, char** argv) {
  opts_t o;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto num = [&]() -> uint64_t { if (i + 1 >= argc) die("missing value"); return std::strtoull(argv[++i], nullptr, 0); };
    if (a == "--frames") o.frames = num();
    else if (a == "--max-len") o.max_len = num();
    else if (a == "--chunk") o.chunk = num();
    else if (a == "--ping-every") o.ping_every = num();
    else if (a == "--seed") o.seed = num();
    else if (a == "--buf") o.buf = num();
    else if (a == "--opts") o.opts = num();  // xyws_decode_stream opts (experiments)
    else if (a == "--oversize") o.oversize = true;
    else if (a == "--oversize-len") o.oversize_len = num();
    else if (a == "--rfc") o.rfc = true;
    else die(("unknown option " + a).c_str());
  }
  if (o.max_len > 1000 || o.frames == 0 || o.chunk == 0 || o.buf < 4096 || o.oversize_len <= 1000 ||
      o.oversize_len > (32u << 20))
    die("bad options");

  std::vector<uint8_t> wire, expect;
  uint64_t payload = 0, want_echoes = 0;
  uint16_t want_code = 0;
  build_streams(o, wire, expect, payload, want_echoes, want_code);

  int ls = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  addr.sin_port = 0;
  if (ls < 0 || ::bind(ls, (sockaddr*)&addr, sizeof addr) || ::listen(ls, 1)) die("listen");
  socklen_t al = sizeof addr;
  ::getsockname(ls, (sockaddr*)&addr, &al);

  // the device context first (one-time init is not part of the timed run)
  { xyws_ctx* c = nullptr; XYCHK(xyws_ctx_create(0, &c)); xyws_ctx_destroy(c); }

  int cs = ::socket(AF_INET, SOCK_STREAM, 0);
  int one = 1, big = 4 << 20;
  for (int fd : {cs, ls}) {
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    ::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof big);
    ::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
  }
  if (::connect(cs, (sockaddr*)&addr, sizeof addr)) die("connect");
  int ss = ::accept(ls, nullptr, nullptr);
  if (ss < 0) die("accept");

  server_stats st;
  std::vector<uint8_t> got;
  got.reserve(expect.size() + 65536);
  auto t0 = std::chrono::steady_clock::now();
  std::thread server([&] { serve(ss, o.buf, (uint32_t)o.opts, o.rfc, st); });
  std::thread receiver([&] {
    std::vector<uint8_t> b(1 << 20);
    for (;;) {
      ssize_t k = ::recv(cs, b.data(), b.size(), 0);
      if (k <= 0) break;
      got.insert(got.end(), b.data(), b.data() + k);
    }
  });
  for (uint64_t off = 0; off < wire.size(); off += o.chunk)
    send_all(cs, wire.data() + off, std::min<uint64_t>(o.chunk, wire.size() - off));
  server.join();
  receiver.join();
  double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  ::close(cs); ::close(ss); ::close(ls);

  // (a close on a complete frame counts that frame in st.frames; one on a cut
  // frame's header does not)
  uint64_t echoed = st.frames - ((st.close_code && !st.early_close) ? 1 : 0);
  bool ok = got == expect && st.close_code == want_code && echoed == want_echoes;
  std::printf("{\"harness\": \"echo_loopback\", \"ok\": %s, \"frames\": %lu, \"payload_bytes\": %lu, "
              "\"wire_bytes_in\": %zu, \"reply_bytes\": %zu, \"close_code\": %u, \"seconds\": %.6f, "
              "\"frames_per_s\": %.1f, \"payload_MBps\": %.2f, \"wire_in_MBps\": %.2f, \"batches\": %lu, "
              "\"frames_per_batch_avg\": %.1f, \"frames_per_batch_max\": %lu, \"chunk\": %lu, \"max_len\": %lu, "
              "\"mode\": \"%s\", \"closed_on_header\": %s}\n",
              ok ? "true" : "false", (unsigned long)echoed, (unsigned long)payload, wire.size(), got.size(),
              st.close_code, sec, echoed / sec, payload / sec / 1e6, wire.size() / sec / 1e6,
              (unsigned long)st.batches, st.batches ? (double)st.frames / st.batches : 0.0,
              (unsigned long)st.max_batch, (unsigned long)o.chunk, (unsigned long)o.max_len,
              o.rfc ? "rfc" : "reference", st.early_close ? "true" : "false");
  if (!ok) {
    size_t i = 0;
    while (i < got.size() && i < expect.size() && got[i] == expect[i]) ++i;
    std::fprintf(stderr, "echo_loopback: reply stream differs at byte %zu (got %zu bytes, expected %zu)\n", i,
                 got.size(), expect.size());
  }
  return ok ? 0 : 1;
}
