// xyws_frames.hip — gfx950 kernels over a decoded frame table (the callers
// on either side of the decode path) and their C-ABI entry points:
//
//   xyws_encode_frames    batched detail::websocket_frame_header_builder
//                         (include/xynet/http/websocket_frame_header.h:136-175)
//                         + payload copy: echo_once's reply
//                         (example/websocket/websocket_echo.cpp:18-27), or
//                         client-role masked frames
//   xyws_classify_frames  websocket_check_parser_result's close policy
//                         (example/include/common/websocket.h:81-108)
//   xyws_reassemble       FIN=0 chains gathered into messages + UTF-8 check
//
// All three are byte/integer work bound by HBM (the gathers) or by launch
// latency (the per-frame passes): per-frame passes are one lane per frame;
// frame-order offsets come from a three-kernel scan (block partials, one block
// over the partials, fix-up); the gathers write 16 KiB output tiles per
// workgroup, each lane four 16-byte chunks, with the items touching the tile
// staged in LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xyws.h"
#include "xyws_device.h"
#include "xyws_ctx.h"

using namespace xyws_internal;

namespace {

constexpr uint32_t FT = 256;           // threads per block, frame-list kernels
constexpr uint32_t SB = 4 * FT;        // items per scan block (4 per lane)
constexpr uint32_t GTILE = 16384;      // gather tile (bytes of output)
constexpr uint32_t GLDS = 512;         // items staged per tile
constexpr uint64_t U64MAX = ~0ull;

// ---------------------------------------------------------------- header build
// detail::websocket_frame_header_builder (:136-175) into four little-endian
// words (byte i = w[i/4] >> 8*(i%4)); returns H. The key word kw (wire bytes,
// little-endian) is written only when has_key, as the builder copies the
// key only for a non-null mask (:168-173). Register-only (no byte array).
__host__ __device__ inline uint32_t build_header(uint32_t flags, uint64_t len, bool has_key, uint32_t kw,
                                                 uint32_t w[4]) {
  const uint32_t b0 = ((flags & XYWS_FLAG_FIN) ? 0x80u : 0u) | (flags & XYWS_FLAG_OP_MASK);
  uint32_t b1 = (flags & XYWS_FLAG_HAS_MASK) ? 0x80u : 0u;
  const bool masked = (flags & XYWS_FLAG_HAS_MASK) != 0;
  const uint32_t k = has_key ? kw : 0u;
  w[0] = w[1] = w[2] = w[3] = 0;
  uint32_t h;
  if (len < 126u) {
    b1 |= (uint32_t)len;
    w[0] = b0 | (b1 << 8);
    if (masked) { w[0] |= k << 16; w[1] = k >> 16; }
    h = 2;
  } else if (len <= 0xFFFFu) {
    b1 |= 126u;
    w[0] = b0 | (b1 << 8) | ((uint32_t)(len >> 8) << 16) | ((uint32_t)(len & 0xFFu) << 24);
    if (masked) w[1] = k;
    h = 4;
  } else {
    b1 |= 127u;
    // bytes 2..9: the length big-endian = the little-endian bytes of bswap64(len)
    uint64_t be = 0;
    for (int i = 0; i < 8; i++) be |= ((len >> (8 * i)) & 0xFFull) << (56 - 8 * i);
    w[0] = b0 | (b1 << 8) | ((uint32_t)(be & 0xFFFFu) << 16);
    w[1] = (uint32_t)(be >> 16);
    w[2] = (uint32_t)(be >> 48);
    if (masked) { w[2] |= k << 16; w[3] = k >> 16; }
    h = 10;
  }
  return masked ? h + 4 : h;
}

XYWS_DEV uint64_t n_eff(uint64_t n, const uint64_t* dev_n) {
  if (!dev_n) return n;
  const uint64_t m = *dev_n;
  return m < n ? m : n;
}

// ---------------------------------------------------------------- scans
// Inclusive/exclusive scans of n u64 values in three kernels: block partials,
// one block over the partials, fix-up. Rev scans from the end (index n-1-i).
struct op_sum {
  static XYWS_DEV uint64_t id() { return 0; }
  static XYWS_DEV uint64_t f(uint64_t a, uint64_t b) { return a + b; }
};
struct op_max {
  static XYWS_DEV uint64_t id() { return 0; }
  static XYWS_DEV uint64_t f(uint64_t a, uint64_t b) { return a > b ? a : b; }
};
struct op_min {
  static XYWS_DEV uint64_t id() { return U64MAX; }
  static XYWS_DEV uint64_t f(uint64_t a, uint64_t b) { return a < b ? a : b; }
};

// Block-wide scan of one value per lane (FT lanes): *exc / return = the
// lane's exclusive / inclusive prefix, *tot the block total.
template <class Op>
XYWS_DEV uint64_t block_scan(uint64_t v, uint64_t* sh, uint64_t* exc, uint64_t* tot) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint64_t x = v;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o, 64);
    if (lane >= o) x = Op::f(y, x);
  }
  uint64_t xe = __shfl_up(x, 1, 64);
  if (lane == 63) sh[wave] = x;
  __syncthreads();
  uint64_t pre = Op::id(), all = Op::id();
  for (uint32_t w = 0; w < FT / 64; w++) {
    if (w < wave) pre = Op::f(pre, sh[w]);
    all = Op::f(all, sh[w]);
  }
  __syncthreads();
  *tot = all;
  *exc = lane ? Op::f(pre, xe) : pre;
  return Op::f(pre, x);
}

template <class Op, bool Rev>
XYWS_DEV uint64_t at(uint64_t n, uint64_t i) { return Rev ? n - 1 - i : i; }

// The values a scan starts from: x[] itself, or (a generator) computed from
// the frame table in the scan's first pass, so that the per-frame pass that
// produced them is not a launch of its own. val<K>(x, j): scan K's value at
// index j.
struct gen_load {
  template <int K>
  XYWS_DEV uint64_t val(const uint64_t* x, uint64_t j) const { return x[j]; }
};

// pass 1: x[idx] <- the block-local scan (exclusive if Excl) of the values
// g gives; part[b] <- total
template <class Op, bool Rev, bool Excl, int K = 0, class Gen = gen_load>
XYWS_DEV void scan_local(uint64_t* x, uint64_t n, uint64_t* part, uint64_t* sh, const Gen& g = Gen()) {
  const uint64_t i0 = (uint64_t)blockIdx.x * SB + 4ull * threadIdx.x;
  uint64_t v[4], acc = Op::id();
#pragma unroll
  for (int k = 0; k < 4; k++) {
    v[k] = i0 + k < n ? g.template val<K>(x, at<Op, Rev>(n, i0 + k)) : Op::id();
    acc = Op::f(acc, v[k]);
  }
  uint64_t run, tot;
  (void)block_scan<Op>(acc, sh, &run, &tot);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint64_t out = Excl ? run : Op::f(run, v[k]);
    run = Op::f(run, v[k]);
    if (i0 + k < n) x[at<Op, Rev>(n, i0 + k)] = out;
  }
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}
template <class Op, bool Rev, bool Excl, class Gen>
__global__ void __launch_bounds__(FT) k_scan_local(uint64_t* x, uint64_t n, uint64_t* part, Gen g) {
  __shared__ uint64_t sh[FT / 64];
  scan_local<Op, Rev, Excl, 0, Gen>(x, n, part, sh, g);
}

// pass 2: one block scans the nb partials exclusively in place; *total <- all
template <class Op>
XYWS_DEV void scan_parts(uint64_t* part, uint64_t nb, uint64_t* total, uint64_t* sh, uint64_t* total2 = nullptr) {
  uint64_t carry = Op::id();
  for (uint64_t c = 0; c < nb; c += FT) {
    const uint64_t i = c + threadIdx.x;
    const uint64_t v = i < nb ? part[i] : Op::id();
    uint64_t ex, tot;
    (void)block_scan<Op>(v, sh, &ex, &tot);
    if (i < nb) part[i] = Op::f(carry, ex);
    carry = Op::f(carry, tot);
  }
  if (threadIdx.x == 0 && total) *total = carry;
  if (threadIdx.x == 0 && total2) *total2 = carry;
}
template <class Op>
__global__ void __launch_bounds__(FT) k_scan_parts(uint64_t* part, uint64_t nb, uint64_t* total, uint64_t* total2) {
  __shared__ uint64_t sh[FT / 64];
  scan_parts<Op>(part, nb, total, sh, total2);
}

// pass 3: x[idx] <- part[block] (op) x[idx]; exclusive scans also x[n] <- total
template <class Op, bool Rev, bool Excl>
XYWS_DEV void scan_fix(uint64_t* x, uint64_t n, const uint64_t* part, const uint64_t* total, uint64_t i) {
  if (Excl && i == 0 && total) x[n] = *total;
  if (i >= n) return;
  const uint64_t p = part[i / SB];
  const uint64_t j = at<Op, Rev>(n, i);
  x[j] = Op::f(p, x[j]);
}
template <class Op, bool Rev, bool Excl>
__global__ void __launch_bounds__(FT) k_scan_fix(uint64_t* x, uint64_t n, const uint64_t* part,
                                                  const uint64_t* total) {
  scan_fix<Op, Rev, Excl>(x, n, part, total, (uint64_t)blockIdx.x * FT + threadIdx.x);
}

// Three independent scans of n values in the same three kernels (the
// reassembly's scans come in two groups of three: one launch per pass instead
// of three). S = scan3_spec<Op, Rev, Excl>; part: 3 * nb words.
template <class O, bool R, bool E>
struct scan3_spec {
  using Op = O;
  static constexpr bool Rev = R, Excl = E;
};
struct scan3_args {
  uint64_t* x[3];
  uint64_t* total[3];
};
template <class S0, class S1, class S2, class Gen>
__global__ void __launch_bounds__(FT) k_scan3_local(scan3_args A, uint64_t n, uint64_t* part, uint64_t nb, Gen g) {
  __shared__ uint64_t sh[FT / 64];
  scan_local<typename S0::Op, S0::Rev, S0::Excl, 0, Gen>(A.x[0], n, part, sh, g);
  scan_local<typename S1::Op, S1::Rev, S1::Excl, 1, Gen>(A.x[1], n, part + nb, sh, g);
  scan_local<typename S2::Op, S2::Rev, S2::Excl, 2, Gen>(A.x[2], n, part + 2 * nb, sh, g);
}
template <class S0, class S1, class S2>
__global__ void __launch_bounds__(FT) k_scan3_parts(scan3_args A, uint64_t* part, uint64_t nb) {
  __shared__ uint64_t sh[FT / 64];
  scan_parts<typename S0::Op>(part, nb, A.total[0], sh);
  scan_parts<typename S1::Op>(part + nb, nb, A.total[1], sh);
  scan_parts<typename S2::Op>(part + 2 * nb, nb, A.total[2], sh);
}
template <class S0, class S1, class S2>
__global__ void __launch_bounds__(FT) k_scan3_fix(scan3_args A, uint64_t n, const uint64_t* part, uint64_t nb) {
  const uint64_t i = (uint64_t)blockIdx.x * FT + threadIdx.x;
  scan_fix<typename S0::Op, S0::Rev, S0::Excl>(A.x[0], n, part, A.total[0], i);
  scan_fix<typename S1::Op, S1::Rev, S1::Excl>(A.x[1], n, part + nb, A.total[1], i);
  scan_fix<typename S2::Op, S2::Rev, S2::Excl>(A.x[2], n, part + 2 * nb, A.total[2], i);
}
template <class S0, class S1, class S2, class Gen>
int scan3(const scan3_args& A, uint64_t n, uint64_t* part, const Gen& g, hipStream_t s) {
  const uint64_t nb = (n + SB - 1) / SB;
  if (nb) hipLaunchKernelGGL((k_scan3_local<S0, S1, S2, Gen>), dim3(nb), dim3(FT), 0, s, A, n, part, nb, g);
  hipLaunchKernelGGL((k_scan3_parts<S0, S1, S2>), dim3(1), dim3(FT), 0, s, A, part, nb);
  hipLaunchKernelGGL((k_scan3_fix<S0, S1, S2>), dim3(nb ? (n + FT - 1) / FT : 1), dim3(FT), 0, s, A, n,
                     (const uint64_t*)part, nb);
  return hip_err(hipGetLastError());
}

// Scan n values (from g) in place (device memory x, n+1 words when Excl &&
// total), part: (n / SB + 1) words of scratch, total / total2: device words
// (nullable) for the total.
template <class Op, bool Rev, bool Excl, class Gen>
int scan(uint64_t* x, uint64_t n, uint64_t* part, uint64_t* total, uint64_t* total2, const Gen& g, hipStream_t s) {
  const uint64_t nb = (n + SB - 1) / SB;
  if (nb == 0) {
    if (Excl && total) {
      hipLaunchKernelGGL((k_scan_parts<Op>), dim3(1), dim3(FT), 0, s, part, 0ull, total, total2);
      hipLaunchKernelGGL((k_scan_fix<Op, Rev, Excl>), dim3(1), dim3(FT), 0, s, x, 0ull, part, total);
    }
    return hip_err(hipGetLastError());
  }
  hipLaunchKernelGGL((k_scan_local<Op, Rev, Excl, Gen>), dim3(nb), dim3(FT), 0, s, x, n, part, g);
  hipLaunchKernelGGL((k_scan_parts<Op>), dim3(1), dim3(FT), 0, s, part, nb, total, total2);
  hipLaunchKernelGGL((k_scan_fix<Op, Rev, Excl>), dim3((n + FT - 1) / FT), dim3(FT), 0, s, x, n,
                     (const uint64_t*)part, (const uint64_t*)total);
  return hip_err(hipGetLastError());
}

// ---------------------------------------------------------------- gather
// One item of a gather: output [dst, dst + H + len) = header bytes hw (H of
// them) then src[soff .. soff + len) XOR the key (payload index from 0).
struct gitem {
  uint64_t dst, soff, len;
  uint32_t hw[4];
  uint32_t h, key;
};

enum { G_ENC = 0, G_REASM = 1 };

struct gparams {
  const uint8_t* src;  // 16-byte aligned base; the frame table's offset p is src[src_lo + p]
  uint64_t src_lo, src_len;
  const xyws_frame* frames;
  const uint64_t* off;  // n_eff + 1 exclusive offsets of the items' outputs
  uint64_t n;
  const uint64_t* dev_n;
  uint32_t mode, flags, enc_opts;
  const uint8_t* keys;
  uint8_t* out;  // 16-byte aligned base; output byte q lives at out[out_lo + q]
  uint64_t out_lo, out_cap;
  uint32_t* err;
};

XYWS_DEV uint32_t reply_flags(const gparams& G, uint32_t fflags) {
  if (!(G.enc_opts & XYWS_ENC_FRAME_OPCODE)) return G.flags;
  uint32_t op = fflags & XYWS_FLAG_OP_MASK;
  if (op == XYWS_FLAG_OP_PING) op = XYWS_FLAG_OP_PONG;
  return op | (fflags & XYWS_FLAG_FIN) | (G.flags & XYWS_FLAG_HAS_MASK);
}

XYWS_DEV gitem item_of(const gparams& G, uint64_t i) {
  gitem it;
  const xyws_frame f = G.frames[i];
  it.dst = G.off[i];
  const uint64_t size = G.off[i + 1] - it.dst;
  it.soff = (uint64_t)f.payload_off;
  it.hw[0] = it.hw[1] = it.hw[2] = it.hw[3] = 0;
  it.h = 0;
  it.key = 0;
  if (G.mode == G_ENC && size) {
    const uint32_t fl = reply_flags(G, f.flags);
    uint32_t kw = 0;
    const bool have = G.keys && (fl & XYWS_FLAG_HAS_MASK);
    if (have)
      kw = (uint32_t)G.keys[4 * i] | ((uint32_t)G.keys[4 * i + 1] << 8) | ((uint32_t)G.keys[4 * i + 2] << 16) |
           ((uint32_t)G.keys[4 * i + 3] << 24);
    it.h = build_header(fl, f.payload_len, have, kw, it.hw);
    it.key = kw;
  }
  it.len = size - it.h;
  return it;
}

XYWS_DEV uint8_t src_byte(const gparams& G, uint64_t p) {
  if (p < G.src_len) return G.src[G.src_lo + p];
  atomicOr(G.err, 0x100u);
  return 0;
}

// Byte q (output coordinate) of item `it`.
XYWS_DEV uint8_t item_byte(const gparams& G, const gitem& it, uint64_t q) {
  const uint64_t r = q - it.dst;
  if (r < it.h) {
    // (shifts, not an index into hw[]: the compiler keeps it in registers)
    const uint32_t q = (uint32_t)r;
    const uint64_t lo = (uint64_t)it.hw[0] | ((uint64_t)it.hw[1] << 32);
    const uint64_t hi = (uint64_t)it.hw[2] | ((uint64_t)it.hw[3] << 32);
    return (uint8_t)((q < 8 ? lo >> (8u * q) : hi >> (8u * (q - 8))) & 0xFFu);
  }
  const uint64_t j = r - it.h;
  return src_byte(G, it.soff + j) ^ (uint8_t)(it.key >> (8u * (j & 3u)));
}

// The last item whose output starts at or before q, among items [a, b) whose
// starts (off) are ascending; from LDS (ls != null) or memory.
XYWS_DEV uint64_t find_item(const uint64_t* ls, const uint64_t* off, uint64_t a, uint64_t b, uint64_t base,
                            uint64_t q) {
  // invariant: start(a) <= q, answer in [a, b)
  uint64_t lo = a, hi = b;
  while (hi - lo > 1) {
    const uint64_t m = (lo + hi) >> 1;
    const uint64_t v = ls ? ls[m - base] : off[m];
    if (v <= q) lo = m; else hi = m;
  }
  return lo;
}

// Tile map: map[t] = the item whose output holds the first byte of gather
// tile t (tile t covers out[] bytes [t*GTILE, (t+1)*GTILE), its first output
// byte is q = max(t*GTILE - out_lo, 0)). One lane per item writes the tiles
// whose first byte it holds (a 1 MiB reply spans 64 of them), so a tile finds
// its items with one load instead of a binary search of the offsets.
__global__ void __launch_bounds__(FT) k_tile_map(gparams G, uint64_t* map, uint64_t ntiles) {
  const uint64_t i = (uint64_t)blockIdx.x * FT + threadIdx.x;
  const uint64_t ne = n_eff(G.n, G.dev_n);
  if (i >= ne) return;
  const uint64_t total = G.off[ne];
  const uint64_t lim = total < G.out_cap ? total : G.out_cap;
  const uint64_t qs = G.off[i], qe0 = G.off[i + 1], qe = qe0 < lim ? qe0 : lim;
  if (qs >= qe) return;
  if (qs == 0) map[0] = i;
  uint64_t t = (qs + G.out_lo + GTILE - 1) / GTILE;
  if (t == 0) t = 1;
  const uint64_t t1 = (qe + G.out_lo + GTILE - 1) / GTILE;
  for (; t < t1 && t < ntiles; t++) map[t] = i;
}

// A chunk-relative position clamped to [-16, 32] (only [0, 16) matters).
XYWS_DEV int32_t rel16(int64_t x) { return x < -16 ? -16 : x > 32 ? 32 : (int32_t)x; }

// Bytes [e, e + 16) of the 16-byte little-endian vector h0..h3 placed at
// offset 0 of an otherwise zero byte line (e in [-15, 15]): a 128-bit shift
// on two 64-bit halves.
XYWS_DEV u32x4 window16s(uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3, int32_t e) {
  const uint64_t lo = (uint64_t)h0 | ((uint64_t)h1 << 32), hi = (uint64_t)h2 | ((uint64_t)h3 << 32);
  const uint32_t s = 8u * (uint32_t)(e < 0 ? -e : e), s7 = s & 63u;  // s in [0, 120]
  uint64_t rl, rh;
  if (e >= 0) {  // (lo, hi) >> s
    const uint64_t x = s7 ? hi << (64u - s7) : 0ull;
    rl = s >= 64 ? hi >> s7 : (lo >> s7) | x;
    rh = s >= 64 ? 0ull : hi >> s7;
  } else {  // (lo, hi) << s
    const uint64_t x = s7 ? lo >> (64u - s7) : 0ull;
    rh = s >= 64 ? lo << s7 : (hi << s7) | x;
    rl = s >= 64 ? 0ull : lo << s7;
  }
  return u32x4{(uint32_t)rl, (uint32_t)(rl >> 32), (uint32_t)rh, (uint32_t)(rh >> 32)};
}

// Byte-select mask (0xFF per byte) of the chunk bytes t in [lo, hi), lo and
// hi chunk-relative (rel16): bytes [0, hi) and not bytes [0, lo), each as
// two 64-bit halves.
XYWS_DEV void low16(int32_t n, uint64_t& m0, uint64_t& m1) {
  const uint32_t c = (uint32_t)(n < 0 ? 0 : n > 16 ? 16 : n);
  const uint64_t a = ~(~0ull << (8u * (c & 7u)));  // bytes [0, c mod 8)
  m0 = c >= 8 ? ~0ull : a;
  m1 = c >= 16 ? ~0ull : c >= 8 ? a : 0ull;
}
XYWS_DEV u32x4 span16(int32_t lo, int32_t hi) {
  uint64_t h0, h1, l0, l1;
  low16(hi, h0, h1);
  low16(lo, l0, l1);
  const uint64_t m0 = h0 & ~l0, m1 = h1 & ~l1;
  return u32x4{(uint32_t)m0, (uint32_t)(m0 >> 32), (uint32_t)m1, (uint32_t)(m1 >> 32)};
}

// Bytes [sh, sh + 16) of the 32 bytes x | y (sh in [0, 16)): a half-select
// (sh >= 8) and two 64-bit funnel shifts.
XYWS_DEV u32x4 funnel16(const u32x4& x, const u32x4& y, uint32_t sh) {
  const uint64_t x0 = (uint64_t)x.x | ((uint64_t)x.y << 32), x1 = (uint64_t)x.z | ((uint64_t)x.w << 32);
  const uint64_t y0 = (uint64_t)y.x | ((uint64_t)y.y << 32), y1 = (uint64_t)y.z | ((uint64_t)y.w << 32);
  const bool h = sh >= 8;
  const uint64_t A = h ? x1 : x0, B = h ? y0 : x1, C = h ? y1 : y0;
  const uint32_t s = 8u * (sh & 7u);
  const uint64_t r0 = s ? (A >> s) | (B << (64u - s)) : A;
  const uint64_t r1 = s ? (B >> s) | (C << (64u - s)) : B;
  return u32x4{(uint32_t)r0, (uint32_t)(r0 >> 32), (uint32_t)r1, (uint32_t)(r1 >> 32)};
}

// Position of the n-th (from 0) set bit of m (n < popcount(m)).
XYWS_DEV uint32_t nth_bit(uint64_t m, uint32_t n) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t w = 32; w; w >>= 1) {
    const uint32_t c = (uint32_t)__builtin_popcountll((m >> pos) & ((1ull << w) - 1ull));
    if (n >= c) { n -= c; pos += w; }
  }
  return pos;
}

// 16 source bytes at src offset p (signed, may start before 0 or run past the
// end): the two aligned 16-byte lines around it, lines outside the source
// [0, round16(src_lo + src_len)) read as zero.
XYWS_DEV u32x4 src16(const gparams& G, int64_t p) {
  const int64_t A = (int64_t)G.src_lo + p;
  const int64_t a = A & ~(int64_t)15;
  const int64_t top = (int64_t)((G.src_lo + G.src_len + 15) & ~15ull);
  const u32x4 z = {0u, 0u, 0u, 0u};
  const u32x4 x = (a >= 0 && a < top) ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(G.src + a)) : z;
  const uint32_t sh = (uint32_t)(A & 15);
  if (!sh) return x;
  const u32x4 y = (a + 16 >= 0 && a + 16 < top) ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(G.src + a + 16)) : z;
  return funnel16(x, y, sh);
}

XYWS_DEV u32x4 shfl_down16(const u32x4& x) {
  return u32x4{(uint32_t)__shfl_down((int)x.x, 1, 64), (uint32_t)__shfl_down((int)x.y, 1, 64),
               (uint32_t)__shfl_down((int)x.z, 1, 64), (uint32_t)__shfl_down((int)x.w, 1, 64)};
}

// Items staged per tile (struct of arrays in LDS).
struct gstage {
  uint64_t dst[GLDS + 1];  // output start (q coordinate); dst[k] of the item after the last: its start
  uint64_t soff[GLDS];
  uint32_t hw[GLDS][4];
  uint32_t h[GLDS], key[GLDS];
  uint16_t cmap[GTILE / 16];  // tiles of many items: chunk -> staged item holding its first byte
};

// Tiles of more items than this map their chunks to items while staging
// (one LDS read per chunk instead of a binary search over the items).
constexpr uint32_t GMAP_ITEMS = 8;

// The first chunk c in [0, GTILE/16] of a tile whose first output byte
// max(base + 16c, 0) lies at or past q = d (base: q of the tile's byte 0).
XYWS_DEV uint32_t chunk_at(int64_t d, int64_t base) {
  if (d <= 0 || d <= base) return 0;
  const int64_t c = (d - base + 15) >> 4;
  return c > (int64_t)(GTILE / 16) ? GTILE / 16 : (uint32_t)c;
}

// The gather (encode replies / message payloads): output tiles of GTILE bytes,
// each lane four 16-byte chunks. The items touching a tile (from the tile map)
// are staged in LDS once; a chunk finds its first item by a binary search in
// LDS (tiles of more than GMAP_ITEMS items: the chunk map written while
// staging). Chunks inside one item's payload (all of them for large frames)
// take a fast path: two chunks per lane per round, and the second line a
// misaligned chunk needs is the next lane's first (a lane shuffle), so every
// source line is read once. The rest (item boundaries, headers) are compacted
// per wave and composed from at most a few items: header bytes from the
// staged header words, payload bytes from two aligned 16-byte source loads and
// a funnel shift, XORed with the rotated key word, each selected by its byte
// mask. One 16-byte store per chunk (byte stores only at the output's ends).
// Tiles with more items than fit in LDS take the per-byte path.
__global__ void __launch_bounds__(FT) k_gather(gparams G, const uint64_t* __restrict__ map, uint64_t ntiles) {
  __shared__ gstage S;
  __shared__ uint64_t s_f0, s_f1;
  const uint64_t ne = n_eff(G.n, G.dev_n);
  const uint64_t total = G.off[ne];
  const uint64_t lim = total < G.out_cap ? total : G.out_cap;  // bytes written
  if (!lim || !ne) return;
  // output chunks are 16-byte aligned in the out[] coordinate: q in [0, lim)
  // sits at out_lo + q
  const uint64_t o0 = G.out_lo, o1 = G.out_lo + lim;
  const uint64_t nt = (o1 + GTILE - 1) / GTILE;
  for (uint64_t tile = blockIdx.x; tile < nt && tile < ntiles; tile += gridDim.x) {
    const uint64_t t0 = tile * GTILE;
    if (threadIdx.x == 0) {
      s_f0 = map[tile];
      s_f1 = tile + 1 < nt ? map[tile + 1] + 1 : ne;
      if (s_f1 > ne) s_f1 = ne;
    }
    __syncthreads();
    const uint64_t f0 = s_f0, f1 = s_f1;
    const bool in_lds = f1 - f0 <= GLDS;
    const bool use_map = in_lds && f1 - f0 > GMAP_ITEMS;
    if (in_lds) {
      const int64_t base = (int64_t)t0 - (int64_t)o0;
      for (uint64_t k = threadIdx.x; k < f1 - f0; k += FT) {
        const gitem it = item_of(G, f0 + k);
        S.dst[k] = it.dst;
        S.soff[k] = it.soff;
        S.hw[k][0] = it.hw[0]; S.hw[k][1] = it.hw[1]; S.hw[k][2] = it.hw[2]; S.hw[k][3] = it.hw[3];
        S.h[k] = it.h;
        S.key[k] = it.key;
        if (use_map) {
          // the chunks whose first byte this item holds: [dst, dst + size)
          const uint32_t c1 = chunk_at((int64_t)(it.dst + it.h + it.len), base);
          for (uint32_t c = chunk_at((int64_t)it.dst, base); c < c1; c++) S.cmap[c] = (uint16_t)k;
        }
      }
      if (threadIdx.x == 0) S.dst[f1 - f0] = G.off[f1];
    }
    __syncthreads();
    constexpr uint32_t GC = GTILE / 16 / FT;
    uint32_t fastm = 0;  // chunks done by the fast path
    if (in_lds) {
      const uint32_t n = (uint32_t)(f1 - f0), lane = __lane_id();
      // two chunks per round (registers: the per-chunk loop below runs in the
      // same kernel at the occupancy this path leaves)
      constexpr uint32_t GH = 2;
#pragma unroll 1
      for (uint32_t c0 = 0; c0 < GC; c0 += GH) {
      u32x4 x[GH], y[GH];
      uint32_t sh[GH], kw[GH], nbm = 0;
#pragma unroll
      for (uint32_t j = 0; j < GH; j++) {
        const uint32_t c = c0 + j;
        const uint64_t a = t0 + (uint64_t)(c * FT + threadIdx.x) * 16;
        const int64_t ca = (int64_t)a - (int64_t)o0;
        const uint64_t qa = a > o0 ? a - o0 : 0;
        uint32_t g = 0;
        if (use_map) {
          g = S.cmap[c * FT + threadIdx.x];
          if (g >= n) g = n - 1;  // (a guard: every chunk in the output is mapped)
        } else {
          uint32_t hi = n;
          while (hi - g > 1) {
            const uint32_t m = (g + hi) >> 1;
            if (S.dst[m] <= qa) g = m; else hi = m;
          }
        }
        const int64_t ds = (int64_t)S.dst[g], de = (int64_t)S.dst[g + 1], ps = ds + S.h[g];
        const int64_t sp = (int64_t)S.soff[g] + (ca - ps);  // source payload index of chunk byte 0
        const bool simple = a >= o0 && a + 16 <= o1 && ps <= ca && de >= ca + 16 && sp + 16 <= (int64_t)G.src_len;
        x[j] = y[j] = u32x4{0u, 0u, 0u, 0u};
        sh[j] = 0;
        kw[j] = 0;
        if (simple) {
          const uint64_t A = G.src_lo + (uint64_t)sp, la = A & ~15ull;
          sh[j] = (uint32_t)(A & 15u);
          kw[j] = rotr8(S.key[g], (uint32_t)(ca - ps));
          x[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(G.src + la));
          fastm |= 1u << c;
          // the second line: the next lane's first when its chunk is the same
          // item's next 16 bytes (its line la + 16), else loaded here
          const bool nb = lane < 63 && de >= ca + 32 && a + 32 <= o1 && sp + 32 <= (int64_t)G.src_len;
          if (sh[j] && !nb) y[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(G.src + la + 16));
          if (nb) nbm |= 1u << j;
        }
      }
#pragma unroll
      for (uint32_t j = 0; j < GH; j++) {
        const uint32_t c = c0 + j;
        const u32x4 yn = shfl_down16(x[j]);
        if (((fastm >> c) & 1u) && sh[j]) {
          x[j] = funnel16(x[j], ((nbm >> j) & 1u) ? yn : y[j], sh[j]);
        }
        if ((fastm >> c) & 1u) {
          const uint64_t a = t0 + (uint64_t)(c * FT + threadIdx.x) * 16;
          __builtin_nontemporal_store(x[j] ^ u32x4{kw[j], kw[j], kw[j], kw[j]}, reinterpret_cast<u32x4*>(G.out + a));
        }
      }
      }
    }
    // The chunks the fast path left (item boundaries, headers, the output's
    // ends), compacted across the wave's rounds: with small items nearly every
    // round of every wave holds a few, and the composition below is the
    // kernel's VALU cost — one pass over the wave's list instead of one per
    // round. Lane i takes the i-th chunk in (round, lane) order.
    uint32_t need = 0;
#pragma unroll
    for (uint32_t c = 0; c < GC; c++) {
      const uint64_t a = t0 + (uint64_t)(c * FT + threadIdx.x) * 16;
      if (!(a + 16 <= o0 || a >= o1 || ((fastm >> c) & 1u))) need |= 1u << c;
    }
    uint64_t bm[GC];
    uint32_t pre[GC + 1];
    pre[0] = 0;
#pragma unroll
    for (uint32_t r = 0; r < GC; r++) {
      bm[r] = __ballot((need >> r) & 1u);
      pre[r + 1] = pre[r] + (uint32_t)__builtin_popcountll(bm[r]);
    }
    const uint32_t wl = __lane_id();
#pragma unroll 1
    for (uint32_t kb = 0; kb < pre[GC]; kb += 64) {
      const uint32_t kk = kb + wl;
      if (kk >= pre[GC]) break;
      uint32_t r = 0, nn = kk;
      uint64_t bmr = bm[0];
#pragma unroll
      for (uint32_t j = 1; j < GC; j++)
        if (kk >= pre[j]) { r = j; bmr = bm[j]; nn = kk - pre[j]; }
      const uint32_t ci = r * FT + (threadIdx.x & ~63u) + nth_bit(bmr, nn);  // the chunk, tile-relative
      const uint64_t a = t0 + (uint64_t)ci * 16;  // aligned out[] position
      const uint64_t qa = a > o0 ? a - o0 : 0;  // first output byte of the chunk
      if (!in_lds) {
        // many tiny items: byte by byte from memory
        uint64_t gi = find_item(nullptr, G.off, f0, f1, f0, qa);
        gitem it = item_of(G, gi);
        uint64_t nxt = gi + 1 < ne ? G.off[gi + 1] : U64MAX;
        for (uint32_t t = 0; t < 16; t++) {
          const uint64_t p = a + t;
          if (p < o0 || p >= o1) continue;
          const uint64_t q = p - o0;
          while (q >= nxt) {
            gi++;
            it = item_of(G, gi);
            nxt = gi + 1 < ne ? G.off[gi + 1] : U64MAX;
          }
          G.out[p] = item_byte(G, it, q);
        }
        continue;
      }
      const uint32_t n = (uint32_t)(f1 - f0);
      uint32_t g = 0;
      if (use_map) {
        g = S.cmap[ci];
        if (g >= n) g = n - 1;  // (every processed chunk is mapped: a guard)
      } else {
        uint32_t hi = n;
        while (hi - g > 1) {
          const uint32_t m = (g + hi) >> 1;
          if (S.dst[m] <= qa) g = m; else hi = m;
        }
      }
      const int64_t ca = (int64_t)a - (int64_t)o0;  // q of chunk byte 0 (may be < 0 in the first chunk)
      u32x4 w = {0u, 0u, 0u, 0u};
      bool oob = false;
      // (positions relative to the chunk, clamped to [-16, 32] in 32 bits:
      // only [0, 16) matters, and the masks below are 64-bit pairs, so that
      // the wave's instruction count per chunk stays small — with many items
      // per tile every wave takes these branches)
      for (uint32_t k = g; k < n; k++) {
        const int64_t ds64 = (int64_t)S.dst[k] - ca;
        if (ds64 >= 16) break;
        const uint32_t hk = S.h[k];
        const int64_t ps64 = ds64 + hk;
        const int32_t ds = rel16(ds64), ps = rel16(ps64), de = rel16((int64_t)S.dst[k + 1] - ca);
        if (hk && ps > 0) {  // header bytes (the item starts before the chunk's end)
          const u32x4 v = window16s(S.hw[k][0], S.hw[k][1], S.hw[k][2], S.hw[k][3], -ds);
          w |= v & span16(ds, ps);
        }
        if (de > ps && ps < 16 && de > 0) {  // payload bytes
          const int64_t d = -ps64;  // payload index of chunk byte 0
          const int64_t sp = (int64_t)S.soff[k] + d;
          u32x4 v = src16(G, sp);
          const uint32_t kw = rotr8(S.key[k], (uint32_t)d);
          const u32x4 m = span16(ps, de);
          // bytes past the source read as zero (and are reported)
          const int64_t past = (int64_t)G.src_len - sp;  // chunk bytes t >= past lie past src_len
          if (past < 16) {
            const u32x4 vm = span16(rel16(past), 16);
            v &= ~vm;
            const u32x4 pm = vm & m;
            if (pm.x | pm.y | pm.z | pm.w) oob = true;
          }
          w |= (v ^ kw) & m;
        }
      }
      if (oob) atomicOr(G.err, 0x100u);
      if (a >= o0 && a + 16 <= o1) {
        __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(G.out + a));
      } else {
        for (uint32_t t = 0; t < 16; t++) {
          const uint64_t p = a + t;
          const uint32_t wt = t < 4 ? w.x : t < 8 ? w.y : t < 12 ? w.z : w.w;  // (no dynamic index: no scratch)
          if (p >= o0 && p < o1) G.out[p] = (uint8_t)(wt >> (8u * (t & 3u)));
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- encode
// sizes: header + payload of every selected frame (0 for the others), made
// in the offsets scan's first pass
struct gen_enc {
  gparams G;
  const xyws_verdict* verd;
  uint32_t amask;
  template <int K>
  XYWS_DEV uint64_t val(const uint64_t*, uint64_t i) const {
    const uint64_t ne = n_eff(G.n, G.dev_n);
    if (i >= ne || (verd && !((amask >> verd[i].action) & 1u))) return 0;
    const xyws_frame f = G.frames[i];
    uint32_t w[4];
    return build_header(reply_flags(G, f.flags), f.payload_len, false, 0, w) + f.payload_len;
  }
};

// ---------------------------------------------------------------- classify
__global__ void __launch_bounds__(FT) k_classify(const uint8_t* src, uint64_t src_len, const xyws_frame* frames,
                                                 uint64_t n, const uint64_t* dev_n, uint64_t max_payload,
                                                 uint32_t policy, xyws_verdict* out, uint64_t* first) {
  const uint64_t i = (uint64_t)blockIdx.x * FT + threadIdx.x;
  const uint64_t ne = n_eff(n, dev_n);
  if (i >= ne) return;
  const xyws_frame f = frames[i];
  const uint32_t op = f.flags & XYWS_FLAG_OP_MASK;
  xyws_verdict v;
  v.close_code = 0;
  v.peer_code = 0;
  v.action = op == XYWS_FLAG_OP_PING ? XYWS_ACT_PING : op == XYWS_FLAG_OP_PONG ? XYWS_ACT_PONG : XYWS_ACT_DATA;
  v.reserved[0] = v.reserved[1] = v.reserved[2] = 0;
  const bool proto = (f.status & (XYWS_ST_RSV | XYWS_ST_RESERVED_OPCODE | XYWS_ST_BAD_CONTROL)) != 0;
  uint16_t code = 0;
  if ((policy & XYWS_POL_STRICT) && proto) code = 1002;
  else if (op == XYWS_FLAG_OP_CLOSE || ((policy & XYWS_POL_REFERENCE) && (op & 8u)))
    code = 1000;  // (websocket.h:87-90: the opcode compared exactly, or its bit 3 as the reference tests it)
  else if (!(f.flags & XYWS_FLAG_FIN) && !(policy & XYWS_POL_FRAGMENTS)) code = 1003;
  else if (!(f.flags & XYWS_FLAG_HAS_MASK) && !(policy & XYWS_POL_UNMASKED)) code = 1008;
  else if (f.payload_len > max_payload) code = 1009;
  if (op == XYWS_FLAG_OP_CLOSE) {
    v.action = XYWS_ACT_CLOSE;
    const uint64_t p = (uint64_t)f.payload_off;
    v.peer_code = 1005;  // (RFC 6455 7.4.1: no status code present)
    if (f.payload_len >= 2 && p + 2 <= src_len) v.peer_code = (uint16_t)((src[p] << 8) | src[p + 1]);
  }
  if (code) {
    v.close_code = code;
    v.action = XYWS_ACT_CLOSE;
    if (first) atomicMin(reinterpret_cast<unsigned long long*>(first), (unsigned long long)i);
  }
  out[i] = v;
}

// ---------------------------------------------------------------- reassembly
// The first scan group's values (made in its first pass): a[i] = 1 + i for a
// text/binary frame (a message start), else 0 (max-scanned: 1 + the last
// start <= i); b[i] = i for a data frame with FIN, else UINT64_MAX
// (min-scanned from the end: the next FIN >= i); st[i] = 1 for a start
// (exclusive sum: message ranks).
struct gen_marks {
  const xyws_frame* frames;
  uint64_t n;
  const uint64_t* dev_n;
  template <int K>
  XYWS_DEV uint64_t val(const uint64_t*, uint64_t i) const {
    if (i >= n_eff(n, dev_n)) return K == 1 ? U64MAX : 0;
    const uint32_t fl = frames[i].flags, op = fl & XYWS_FLAG_OP_MASK;
    const bool start = op == XYWS_FLAG_OP_TEXT || op == XYWS_FLAG_OP_BINARY;
    if (K == 0) return start ? i + 1 : 0;
    if (K == 1) return (op <= XYWS_FLAG_OP_BINARY && (fl & XYWS_FLAG_FIN)) ? i : U64MAX;
    return start ? 1 : 0;
  }
};

// After the scans: a[i] = 1 + the last start <= i (0: none), b[i] = the next
// data frame with FIN >= i. Frame i belongs to the message of s = a[i] - 1
// when it is a data frame and i <= b[s]. sz[i] = its payload bytes, cnt[i] =
// 1 for members; orphan continuations raise orph[the next start's rank].
__global__ void __launch_bounds__(FT) k_rs_sizes(const xyws_frame* frames, uint64_t n, const uint64_t* dev_n,
                                                 const uint64_t* a, const uint64_t* b, uint64_t* sz,
                                                 uint64_t* cnt, uint64_t* orphan_flag, const uint64_t* rank,
                                                 uint64_t* starts) {
  const uint64_t i = (uint64_t)blockIdx.x * FT + threadIdx.x;
  if (i >= n) return;
  const uint64_t ne = n_eff(n, dev_n);
  uint64_t s = 0, c = 0, o = 0;
  if (i < ne) {
    const xyws_frame f = frames[i];
    const uint32_t op = f.flags & XYWS_FLAG_OP_MASK;
    if (op <= XYWS_FLAG_OP_BINARY) {
      const uint64_t st = a[i];
      if (st && i <= b[st - 1]) {
        s = f.payload_len;
        c = 1;
      } else {
        o = 1;  // (a continuation outside a message: dropped)
      }
    }
  }
  // starts[m] = the first frame of message m for EVERY message (also past
  // msg_cap: a record's length and frame count end at the next message's
  // start), by rank (st[] exclusive-scanned: frame i starts a message when
  // the rank steps after it)
  if (i < ne) {
    const uint64_t r = rank[i];
    if (rank[i + 1] != r) starts[r] = i;
  }
  sz[i] = s;
  cnt[i] = c;
  orphan_flag[i] = o;
}

constexpr uint32_t UT = 65536;  // UTF-8 tile: bytes of out[] (k_utf8)

// each record from the offsets of its start and the next start (starts[]:
// every message's first frame, k_rs_sizes); continuations after the last
// message's FIN with no message after them set bit 0x200 of the device error
// word. With umap, also the UTF-8 tile map: umap[t] = the message holding
// the first byte of UTF-8 tile t (UT bytes of out[]), written by the lanes of
// the messages whose bytes start a tile (a 1 MiB message spans 16), so that a
// tile finds its messages with two loads and skips at once when none of them
// is a text message.
__global__ void __launch_bounds__(FT) k_rs_msgs(const xyws_frame* frames, const uint64_t* dev_n, uint64_t n,
                                                const uint64_t* nmsg_p,
                                                const uint64_t* off, const uint64_t* cntoff, const uint64_t* b,
                                                const uint64_t* starts, const uint64_t* orph_rank,
                                                uint64_t out_cap, xyws_message* msgs, uint64_t msg_cap,
                                                uint64_t* dev_nmsgs, uint32_t* err, uint64_t* umap,
                                                uint64_t utiles, uint64_t out_lo) {
  const uint64_t m = (uint64_t)blockIdx.x * FT + threadIdx.x;
  const uint64_t ne = n_eff(n, dev_n), nm = *nmsg_p;
  if (m == 0) {
    if (dev_nmsgs) *dev_nmsgs = nm;
    const uint64_t before = nm ? orph_rank[starts[nm - 1]] : 0;
    if (orph_rank[ne] > before) atomicOr(err, 0x200u);
  }
  if (m >= nm || m >= msg_cap) return;
  const uint64_t s = starts[m];
  const uint64_t ns = m + 1 < nm ? starts[m + 1] : ne;
  const uint64_t op = frames[s].flags & XYWS_FLAG_OP_MASK;
  uint32_t st = 0;
  if (b[s] < ns) st |= XYWS_MSG_COMPLETE;
  else if (m + 1 < nm) st |= XYWS_MSG_INTERRUPTED;
  if (off[ns] > out_cap) st |= XYWS_MSG_TRUNCATED;
  // orphans between the previous start (or the batch start) and this one:
  // orph_rank = orphan flags prefix-summed; orphans before s minus those
  // before the previous start
  const uint64_t ps = m ? starts[m - 1] : 0;
  if (orph_rank[s] - (m ? orph_rank[ps] : 0) > 0) st |= XYWS_MSG_ORPHANS;
  // the whole 40-byte record in five 8-byte stores (status, opcode and the
  // reserved bytes as one little-endian word)
  static_assert(sizeof(xyws_message) == 40 && offsetof(xyws_message, status) == 32, "xyws_message layout");
  uint64_t* r = reinterpret_cast<uint64_t*>(msgs + m);
  r[0] = s;
  r[1] = cntoff[ns] - cntoff[s];
  r[2] = off[s];
  r[3] = off[ns] - off[s];
  r[4] = (uint64_t)st | (op << 32);
  if (umap) {
    const uint64_t qs = off[s], qe = off[ns] < out_cap ? off[ns] : out_cap;
    if (qs < qe) {
      if (qs == 0) umap[0] = m;
      uint64_t t = (qs + out_lo + UT - 1) / UT;
      if (t == 0) t = 1;
      const uint64_t t1 = (qe + out_lo + UT - 1) / UT;
      for (; t < t1 && t < utiles; t++) umap[t] = m;
    }
  }
}

// UTF-8 (RFC 3629) over every text message's bytes in out[out_lo + ...]; one
// lane per 16-byte chunk, neighbours read for sequences crossing chunks.
XYWS_DEV uint32_t lead_len(uint32_t c) { return c >= 0xF0u ? 4u : c >= 0xE0u ? 3u : c >= 0xC0u ? 2u : 0u; }

// True when the bytes at out[] positions q in [q0, q1) of message [mo, me)
// (out coordinates q = position - out_lo, total written) hold an invalid
// UTF-8 sequence: k_utf8's per-byte rules (a continuation byte must be
// claimed by a lead at most 3 bytes before it in the message; C0, C1 and
// F5..FF never appear; a lead's continuations, overlongs, surrogates and
// code points above U+10FFFF; a sequence cut by the message end is invalid
// only in a complete, untruncated message). For the probe pass (the first
// bytes of each message), not the streaming pass.
XYWS_DEV bool utf8_span_bad(const uint8_t* out, uint64_t out_lo, uint64_t total, uint64_t q0, uint64_t q1,
                            uint64_t mo, uint64_t me, uint32_t ty) {
  // (q1 - q0 <= 16: the bytes [q0 - 3, q0 + 19) the rules look at come from
  // three aligned 16-byte lines loaded at once — one memory round trip, not
  // one per byte; lines at or past the bytes written read as zero, and the
  // rules never look past them)
  const uint64_t A = (out_lo + (q0 >= 3 ? q0 - 3 : 0)) & ~15ull, lim = out_lo + total;
  u32x4 L0 = {0u, 0u, 0u, 0u}, L1 = L0, L2 = L0;
  if (A < lim) L0 = *reinterpret_cast<const u32x4*>(out + A);
  if (A + 16 < lim) L1 = *reinterpret_cast<const u32x4*>(out + A + 16);
  if (A + 32 < lim) L2 = *reinterpret_cast<const u32x4*>(out + A + 32);
  auto pick = [](const u32x4& v, uint32_t k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; };
  auto at = [&](uint64_t q) -> uint32_t {
    const uint32_t i = (uint32_t)(out_lo + q - A), k = (i >> 2) & 3u;
    const uint32_t d0 = pick(L0, k), d1 = pick(L1, k), d2 = pick(L2, k);
    const uint32_t d = i < 16 ? d0 : i < 32 ? d1 : d2;  // (selects: no private array)
    return (d >> (8u * (i & 3u))) & 0xFFu;
  };
  for (uint64_t q = q0; q < q1 && q < me && q < total; q++) {
    const uint32_t ch = at(q);
    if (ch < 0x80u) continue;
    if (ch < 0xC0u) {
      bool claimed = false;
      for (uint32_t d = 1; d <= 3 && !claimed; d++) {
        if (q < mo + d) break;
        if (lead_len(at(q - d)) > d) claimed = true;
      }
      if (!claimed) return true;
    } else if (ch == 0xC0u || ch == 0xC1u || ch >= 0xF5u) {
      return true;
    } else {
      const uint32_t L = lead_len(ch);
      if (q + L > me || q + L > total) return (ty & XYWS_MSG_COMPLETE) && !(ty & XYWS_MSG_TRUNCATED);
      uint32_t c1 = 0;
      for (uint32_t d = 1; d < L; d++) {
        const uint32_t cb = at(q + d);
        if ((cb & 0xC0u) != 0x80u) return true;
        if (d == 1) c1 = cb;
      }
      if ((ch == 0xE0u && c1 < 0xA0u) || (ch == 0xEDu && c1 > 0x9Fu) || (ch == 0xF0u && c1 < 0x90u) ||
          (ch == 0xF4u && c1 > 0x8Fu))
        return true;
    }
  }
  return false;
}

// The tile's messages (up to UMS) are staged in LDS with a bad flag each; a
// lane marks its message's flag, and the flags reach the records once per tile
// (one atomic per bad message per tile, not one per byte or chunk).
constexpr uint32_t UMS = 512;
struct ustage {
  uint64_t mo[UMS], me[UMS];
  uint32_t ty[UMS];  // status bits | text (bit 31)
  uint32_t bad[UMS];
};
constexpr uint32_t UTEXT = 1u << 31;
constexpr uint32_t UPROBE = 16;  // bytes of each message the probe pass checks

__global__ void __launch_bounds__(FT) k_utf8(const uint8_t* out, uint64_t out_lo, uint64_t out_cap,
                                             const uint64_t* nmsg_p, xyws_message* msgs, uint64_t msg_cap,
                                             const uint64_t* map, uint64_t ntiles) {
  __shared__ ustage U;
  __shared__ uint32_t s_text;
  __shared__ uint64_t s_m0, s_m1;
  const uint64_t nm0 = *nmsg_p, nm = nm0 < msg_cap ? nm0 : msg_cap;
  if (!nm) return;
  const uint64_t total0 = msgs[nm - 1].out_off + msgs[nm - 1].length;
  const uint64_t total = total0 < out_cap ? total0 : out_cap;
  if (!total) return;
  const uint64_t nt = (out_lo + total + UT - 1) / UT;
  for (uint64_t tile = blockIdx.x; tile < nt && tile < ntiles; tile += gridDim.x) {
    if (threadIdx.x == 0) {
      s_m0 = map[tile];
      s_m1 = tile + 1 < nt ? map[tile + 1] : nm - 1;  // (inclusive)
      s_text = 0;
    }
    __syncthreads();
    const uint64_t m0 = s_m0, m1 = s_m1 < nm ? s_m1 : nm - 1;
    const bool inl = m1 - m0 < UMS;  // the tile's messages staged in LDS
    for (uint64_t m = m0 + threadIdx.x; m <= m1; m += FT) {
      const xyws_message r = msgs[m];
      const bool text = r.opcode == XYWS_FLAG_OP_TEXT && r.length;
      if (text) s_text = 1;
      if (inl) {
        const uint32_t k = (uint32_t)(m - m0);
        U.mo[k] = r.out_off;
        U.me[k] = r.out_off + r.length;
        U.ty[k] = r.status | (r.opcode == XYWS_FLAG_OP_TEXT ? UTEXT : 0u);
        U.bad[k] = 0;
      }
    }
    __syncthreads();
    // message m's fields, from LDS or the records
    auto mo_of = [&](uint64_t m) -> uint64_t { return inl ? U.mo[m - m0] : msgs[m].out_off; };
    auto me_of = [&](uint64_t m) -> uint64_t { return inl ? U.me[m - m0] : msgs[m].out_off + msgs[m].length; };
    auto ty_of = [&](uint64_t m) -> uint32_t {
      return inl ? U.ty[m - m0] | (U.bad[m - m0] ? XYWS_MSG_UTF8_BAD : 0u)
                 : msgs[m].status | (msgs[m].opcode == XYWS_FLAG_OP_TEXT ? UTEXT : 0u);
    };
    auto mark = [&](uint64_t m, uint32_t ty) {
      if (ty & XYWS_MSG_UTF8_BAD) return;
      if (inl) U.bad[m - m0] = 1;
      else atomicOr(&msgs[m].status, XYWS_MSG_UTF8_BAD);
    };
    if (s_text) {
      // Probe pass: the first UPROBE bytes of each text message starting in
      // the tile, one lane per message; a message found bad there is skipped
      // by the streaming pass below before its loads (random "text", c1:
      // every message is bad within its first bytes, so the tile's rows are
      // never loaded — 64 lanes each checking their own chunk of a message's
      // first row was 64 checks where one suffices)
      {
        const uint64_t tq0 = tile * UT > out_lo ? tile * UT - out_lo : 0;
        for (uint64_t m = m0 + threadIdx.x; m <= m1; m += FT) {
          const uint32_t ty = ty_of(m);
          if (!(ty & UTEXT) || (ty & XYWS_MSG_UTF8_BAD)) continue;
          const uint64_t mo = mo_of(m), me = me_of(m);
          if (mo < tq0) continue;  // (its first bytes are an earlier tile's probe)
          if (utf8_span_bad(out, out_lo, total, mo, mo + UPROBE, mo, me, ty)) mark(m, ty);
        }
        __syncthreads();
      }
      // the tile's 16-byte chunks in out[] coordinates q = position - out_lo
      const uint64_t t0 = tile * UT;
      // each wave walks its own UT/4 bytes row by row (a row: 64 chunks, one
      // per lane), so a lane's next chunk usually lies in the message of its
      // last one: once that message is known bad (random "text": in its
      // first row) the lane skips the rest of it, loads included
      constexpr uint32_t UROWS = UT / 16 / FT;
      const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
      uint64_t sk0 = 1, sk1 = 0;  // q range of a message this lane needs not check
      for (uint32_t kr = 0; kr < UROWS; kr++) {
        const uint32_t c = (wv * UROWS + kr) * 64u + ln;
        const uint64_t a = t0 + (uint64_t)c * 16;  // out[] byte position
        if (a + 16 <= out_lo) continue;
        const uint64_t q0 = a > out_lo ? a - out_lo : 0;
        if (q0 >= total) break;
        if (q0 >= sk0 && a + 16 - out_lo <= sk1) continue;
        {
          // (a chunk inside a message the probe found bad: no load)
          uint64_t lo = m0, hi = m1 + 1;
          while (hi - lo > 1) {
            const uint64_t md = (lo + hi) >> 1;
            if (mo_of(md) <= q0) lo = md; else hi = md;
          }
          const uint64_t q1 = a + 16 - out_lo;
          if ((ty_of(lo) & XYWS_MSG_UTF8_BAD) && q1 <= me_of(lo)) {
            sk0 = mo_of(lo);
            sk1 = me_of(lo);
            continue;
          }
        }
        // the chunk's bytes: one 16-byte load when it lies inside the written
        // range, else byte loads of the bytes that do (the rest read as 0)
        uint32_t w[4];
        if (a >= out_lo && a + 16 <= out_lo + total && !((uintptr_t)out & 15u)) {
          const u32x4 v = *reinterpret_cast<const u32x4*>(out + a);
          w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        } else {
          w[0] = w[1] = w[2] = w[3] = 0;
          for (uint32_t t = 0; t < 16; t++)
            if (a + t >= out_lo && a + t < out_lo + total) w[t >> 2] |= (uint32_t)out[a + t] << (8u * (t & 3u));
        }
        // ASCII bytes are valid anywhere, and a lead byte before the chunk
        // checks its own continuations: an all-ASCII chunk has nothing to do
        if (!((w[0] | w[1] | w[2] | w[3]) & 0x80808080u)) continue;
        // the last message starting at or before q0, among [m0, m1]
        uint64_t lo = m0, hi = m1 + 1;
        while (hi - lo > 1) {
          const uint64_t md = (lo + hi) >> 1;
          if (mo_of(md) <= q0) lo = md; else hi = md;
        }
        uint64_t m = lo;
        uint64_t mo = mo_of(m), me = me_of(m);
        uint64_t nx = m + 1 <= m1 ? mo_of(m + 1) : ~0ull;
        uint32_t ty = ty_of(m);
        bool bad = false;  // for message m, reported once when m changes
        for (uint32_t t = 0; t < 16; t++) {
          const uint64_t pq = a + t;
          if (pq < out_lo) continue;
          const uint64_t q = pq - out_lo;
          if (q >= total) break;
          if (nx <= q) {
            if (bad) mark(m, ty);
            bad = false;
            while (m + 1 <= m1 && mo_of(m + 1) <= q) m++;
            mo = mo_of(m);
            me = me_of(m);
            nx = m + 1 <= m1 ? mo_of(m + 1) : ~0ull;
            ty = ty_of(m);
          }
          if (!(ty & UTEXT) || q < mo || q >= me || bad || (ty & XYWS_MSG_UTF8_BAD)) continue;
          const uint32_t ch = (w[t >> 2] >> (8u * (t & 3u))) & 0xFFu;
          if (ch < 0x80u) {
          } else if (ch < 0xC0u) {
            // a continuation byte: a lead within 3 bytes before must claim it
            bool claimed = false;
            for (uint32_t d = 1; d <= 3 && !claimed; d++) {
              if (q < mo + d) break;
              const uint32_t pb = t >= d ? (w[(t - d) >> 2] >> (8u * ((t - d) & 3u))) & 0xFFu
                                         : out[out_lo + q - d];
              if (lead_len(pb) > d) claimed = true;
            }
            bad = !claimed;
          } else if (ch == 0xC0u || ch == 0xC1u || ch >= 0xF5u) {
            bad = true;
          } else {
            const uint32_t L = lead_len(ch);
            if (q + L > me || q + L > total) {
              // cut by the end: invalid only in a complete message whose bytes
              // all fit (an incomplete message continues in a later batch)
              bad = (ty & XYWS_MSG_COMPLETE) && !(ty & XYWS_MSG_TRUNCATED);
            } else {
              uint32_t c1 = 0;
              for (uint32_t d = 1; d < L; d++) {
                const uint32_t cb = t + d < 16 ? (w[(t + d) >> 2] >> (8u * ((t + d) & 3u))) & 0xFFu
                                               : out[out_lo + q + d];
                if ((cb & 0xC0u) != 0x80u) bad = true;
                if (d == 1) c1 = cb;
              }
              if (ch == 0xE0u && c1 < 0xA0u) bad = true;  // overlong
              if (ch == 0xEDu && c1 > 0x9Fu) bad = true;  // surrogates
              if (ch == 0xF0u && c1 < 0x90u) bad = true;  // overlong
              if (ch == 0xF4u && c1 > 0x8Fu) bad = true;  // above U+10FFFF
            }
          }
        }
        if (bad) mark(m, ty);
        // (the chunk's last message: nothing left to check in it)
        if (bad || (ty & XYWS_MSG_UTF8_BAD) || !(ty & UTEXT)) {
          sk0 = mo;
          sk1 = me;
        }
      }
    }
    __syncthreads();
    if (inl)
      for (uint64_t m = m0 + threadIdx.x; m <= m1; m += FT)
        if (U.bad[m - m0] && !(U.ty[m - m0] & XYWS_MSG_UTF8_BAD)) atomicOr(&msgs[m].status, XYWS_MSG_UTF8_BAD);
    __syncthreads();
  }
}

__global__ void k_put(uint64_t* p, uint64_t v) { *p = v; }

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

uint64_t xyws_header_build(uint8_t flags, const uint8_t* key, uint64_t len, uint8_t out[14]) {
  uint32_t w[4];
  const uint32_t kw = key ? ((uint32_t)key[0] | ((uint32_t)key[1] << 8) | ((uint32_t)key[2] << 16) |
                             ((uint32_t)key[3] << 24))
                          : 0u;
  const uint32_t h = build_header(flags, len, key != nullptr, kw, w);
  if (out)
    for (uint32_t i = 0; i < h; i++) out[i] = (uint8_t)(w[i >> 2] >> (8u * (i & 3u)));
  return h;
}

int xyws_encode_frames(xyws_ctx* ctx, const void* dev_src, uint64_t src_len, const xyws_frame* dev_frames,
                       uint64_t n, const uint64_t* dev_n, uint8_t flags, uint32_t enc_opts,
                       const uint8_t* dev_keys, const xyws_verdict* dev_verdicts, uint32_t action_mask,
                       void* dev_out, uint64_t out_cap, uint64_t* dev_offsets, uint64_t* dev_out_len,
                       void* stream) {
  if (!ctx || (!dev_frames && n) || (!dev_src && src_len) || (!dev_out && out_cap)) return XYWS_ERR_INVALID;
  std::lock_guard<std::mutex> lk(ctx->mu);
  device_guard gd(ctx->device);
  if (!gd.ok) return XYWS_ERR_HIP;
  hipStream_t s = (hipStream_t)stream;
  const bool capt = capturing(s);
  scratch_slot* sl = nullptr;
  int rc = acquire_slot(ctx, s, capt, &sl);
  if (rc) return rc;
  // scratch: offsets (n + 1, unless the caller's), block partials, total
  const uint64_t nb = (n + SB - 1) / SB + 1;
  const uint64_t oa0 = reinterpret_cast<uintptr_t>(dev_out) & 15;
  const uint64_t ntiles = (oa0 + out_cap + GTILE - 1) / GTILE + 1;
  if ((rc = ensure_aux(sl, 8 * ((dev_offsets ? 0 : n + 1) + nb + 2 + ntiles), capt))) return rc;
  uint64_t* aux = static_cast<uint64_t*>(sl->aux_mem);
  uint64_t* off = dev_offsets ? dev_offsets : aux;
  uint64_t* part = dev_offsets ? aux : aux + n + 1;
  uint64_t* total = part + nb;
  uint64_t* tmap = total + 2;
  const uintptr_t oa = reinterpret_cast<uintptr_t>(dev_out);
  const uintptr_t sa = reinterpret_cast<uintptr_t>(dev_src);
  gparams G;
  G.src = reinterpret_cast<const uint8_t*>(sa & ~(uintptr_t)15);
  G.src_lo = sa & 15;
  G.src_len = src_len;
  G.frames = dev_frames;
  G.off = off;
  G.n = n;
  G.dev_n = dev_n;
  G.mode = G_ENC;
  G.flags = flags;
  G.enc_opts = enc_opts;
  G.keys = dev_keys;
  G.out = reinterpret_cast<uint8_t*>(oa & ~(uintptr_t)15);
  G.out_lo = oa & 15;
  G.out_cap = out_cap;
  G.err = ctx->err;
  // (the sizes made in the scan's first pass; the total also into dev_out_len)
  if ((rc = scan<op_sum, false, true>(off, n, part, total, dev_out_len, gen_enc{G, dev_verdicts, action_mask}, s)))
    return rc;
  if (n && out_cap) {
    const uint64_t tiles = (G.out_lo + out_cap + GTILE - 1) / GTILE;
    hipLaunchKernelGGL(k_tile_map, dim3((n + FT - 1) / FT), dim3(FT), 0, s, G, tmap, ntiles);
    hipLaunchKernelGGL(k_gather, dim3(grid_for(tiles, 1, 8192)), dim3(FT), 0, s, G, (const uint64_t*)tmap, ntiles);
    if ((rc = hip_err(hipGetLastError()))) return rc;
  }
  return XYWS_OK;
}

int xyws_classify_frames(xyws_ctx* ctx, const void* dev_src, uint64_t src_len, const xyws_frame* dev_frames,
                         uint64_t n, const uint64_t* dev_n, uint64_t max_payload, uint32_t policy,
                         xyws_verdict* dev_verdicts, uint64_t* dev_first_close, void* stream) {
  if (!ctx || (!dev_frames && n) || (!dev_verdicts && n)) return XYWS_ERR_INVALID;
  device_guard gd(ctx->device);
  if (!gd.ok) return XYWS_ERR_HIP;
  hipStream_t s = (hipStream_t)stream;
  if (dev_first_close) {
    hipLaunchKernelGGL(k_put, dim3(1), dim3(1), 0, s, dev_first_close, U64MAX);
  }
  if (n) {
    hipLaunchKernelGGL(k_classify, dim3((n + FT - 1) / FT), dim3(FT), 0, s,
                       static_cast<const uint8_t*>(dev_src), src_len, dev_frames, n, dev_n, max_payload, policy,
                       dev_verdicts, dev_first_close);
  }
  return hip_err(hipGetLastError());
}

int xyws_reassemble(xyws_ctx* ctx, const void* dev_src, uint64_t src_len, const xyws_frame* dev_frames,
                    uint64_t n, const uint64_t* dev_n, uint32_t opts, void* dev_out, uint64_t out_cap,
                    xyws_message* dev_msgs, uint64_t msg_cap, uint64_t* dev_nmsgs, void* stream) {
  if (!ctx || (!dev_frames && n) || (!dev_src && src_len) || (!dev_out && out_cap) || (!dev_msgs && msg_cap))
    return XYWS_ERR_INVALID;
  std::lock_guard<std::mutex> lk(ctx->mu);
  device_guard gd(ctx->device);
  if (!gd.ok) return XYWS_ERR_HIP;
  hipStream_t s = (hipStream_t)stream;
  const bool capt = capturing(s);
  scratch_slot* sl = nullptr;
  int rc = acquire_slot(ctx, s, capt, &sl);
  if (rc) return rc;
  // scratch: a, b, st/rank, sz/off, cnt/cntoff, orphan flags/prefix (n + 1
  // each), block partials, totals
  const uint64_t w = n + 1, nb = (n + SB - 1) / SB + 1;
  const uint64_t ntiles = ((reinterpret_cast<uintptr_t>(dev_out) & 15) + out_cap + GTILE - 1) / GTILE + 1;
  const uint64_t utiles = ((reinterpret_cast<uintptr_t>(dev_out) & 15) + out_cap + UT - 1) / UT + 1;
  if ((rc = ensure_aux(sl, 8 * (7 * w + 3 * nb + 4 + ntiles + utiles), capt))) return rc;
  uint64_t* A = static_cast<uint64_t*>(sl->aux_mem);
  uint64_t *a = A, *b = A + w, *st = A + 2 * w, *off = A + 3 * w, *cnt = A + 4 * w, *orph = A + 5 * w;
  uint64_t* starts = A + 6 * w;   // every message's first frame
  uint64_t* part = A + 7 * w;     // 3 * nb: one slice per scan of a group
  uint64_t* tot = part + 3 * nb;  // tot[0]: bytes, tot[1]: messages, tot[2], tot[3]: scratch totals
  uint64_t* tmap = tot + 4;       // gather tile map
  uint64_t* umap = tmap + ntiles; // UTF-8 tile map
  const bool utf8 = (opts & XYWS_REASM_UTF8) && out_cap && msg_cap;
  const dim3 gn((uint32_t)((n + FT - 1) / FT > 0 ? (n + FT - 1) / FT : 1));
  // the last start at or before each frame, the next FIN at or after it, and
  // the message ranks of the starts (the marks made in the first pass)
  if ((rc = scan3<scan3_spec<op_max, false, false>, scan3_spec<op_min, true, false>, scan3_spec<op_sum, false, true>>(
           scan3_args{{a, b, st}, {tot + 2, tot + 3, tot + 1}}, n, part, gen_marks{dev_frames, n, dev_n}, s)))
    return rc;
  // (the sizes in a kernel of their own: made inside the scan, each of its
  // three values repeated the frame's random loads, c2 0.238 -> 0.307 ms)
  if (n) {
    hipLaunchKernelGGL(k_rs_sizes, gn, dim3(FT), 0, s, dev_frames, n, dev_n, (const uint64_t*)a,
                       (const uint64_t*)b, off, cnt, orph, (const uint64_t*)st, starts);
    if ((rc = hip_err(hipGetLastError()))) return rc;
  }
  // output offsets, frame counts and orphan ranks
  if ((rc = scan3<scan3_spec<op_sum, false, true>, scan3_spec<op_sum, false, true>, scan3_spec<op_sum, false, true>>(
           scan3_args{{off, cnt, orph}, {tot + 0, tot + 2, tot + 3}}, n, part, gen_load{}, s)))
    return rc;
  hipLaunchKernelGGL(k_rs_msgs, gn, dim3(FT), 0, s, dev_frames, dev_n, n, (const uint64_t*)(tot + 1),
                     (const uint64_t*)off,
                     (const uint64_t*)cnt, (const uint64_t*)b, (const uint64_t*)starts, (const uint64_t*)orph,
                     out_cap, dev_msgs, msg_cap, dev_nmsgs, ctx->err, utf8 ? umap : nullptr, utiles,
                     (uint64_t)(reinterpret_cast<uintptr_t>(dev_out) & 15));
  if ((rc = hip_err(hipGetLastError()))) return rc;
  const uintptr_t oa = reinterpret_cast<uintptr_t>(dev_out);
  const uintptr_t sa = reinterpret_cast<uintptr_t>(dev_src);
  gparams G;
  G.src = reinterpret_cast<const uint8_t*>(sa & ~(uintptr_t)15);
  G.src_lo = sa & 15;
  G.src_len = src_len;
  G.frames = dev_frames;
  G.off = off;
  G.n = n;
  G.dev_n = dev_n;
  G.mode = G_REASM;
  G.flags = 0;
  G.enc_opts = 0;
  G.keys = nullptr;
  G.out = reinterpret_cast<uint8_t*>(oa & ~(uintptr_t)15);
  G.out_lo = oa & 15;
  G.out_cap = out_cap;
  G.err = ctx->err;
  if (n && out_cap) {
    const uint64_t tiles = (G.out_lo + out_cap + GTILE - 1) / GTILE;
    hipLaunchKernelGGL(k_tile_map, dim3((n + FT - 1) / FT), dim3(FT), 0, s, G, tmap, ntiles);
    hipLaunchKernelGGL(k_gather, dim3(grid_for(tiles, 1, 8192)), dim3(FT), 0, s, G, (const uint64_t*)tmap, ntiles);
    if ((rc = hip_err(hipGetLastError()))) return rc;
  }
  if (utf8) {
    // (the UTF-8 tile map: k_rs_msgs)
    hipLaunchKernelGGL(k_utf8, dim3(grid_for(utiles, 1, 4096)), dim3(FT), 0, s, (const uint8_t*)G.out, G.out_lo,
                       out_cap, (const uint64_t*)(tot + 1), dev_msgs, msg_cap, (const uint64_t*)umap, utiles);
    if ((rc = hip_err(hipGetLastError()))) return rc;
  }
  return XYWS_OK;
}

}  // extern "C"
