// xyws.hip — gfx950 WebSocket frame decode: kernels + the C-ABI of include/xyws.h.
//
// Hot path of xuanyi-fu/xynet re-designed for MI355X (paths relative to the
// reference tree):
//   websocket_mask            include/xynet/http/websocket_frame_mask.h:6-25
//   header parse              include/xynet/http/websocket_frame_header.h:305-385
//   per-frame driver          example/include/common/websocket.h:110-134
//
// Kernels in this file
//   k_unmask_range   xyws_unmask: in-place XOR of one contiguous range, 16 B/lane.
//   k_parse_indexed  xyws_decode_indexed, step 1: one lane per caller-given start.
//   k_stream_serial  xyws_decode_stream with XYWS_OPT_SERIAL_SCAN: one-lane
//                    boundary chase (exact, latency bound; debug/reference shape).
//   k_unmask_tiles   step 2 of both: byte tiles of 16 KiB per workgroup, each
//                    lane XORs 4 x 16 B with the covering frames' rotated keys.
//   k_stream_runs    (xyws_stream.hip) the default stream decoder: one
//                    workgroup per contiguous run, exact chase inside a run,
//                    speculative run entries checked by the predecessor.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <mutex>

#include "xyws.h"
#include "xyws_device.h"
#include "xyws_stream.h"
#include "xyws_ctx.h"

#ifndef XYWS_HAVE_FUSED
#define XYWS_HAVE_FUSED 1
#endif

#define UNMASK_TILE 16384u
#define UNMASK_THREADS 256u
#define UNMASK_LDS_FRAMES 512u

// ---------------------------------------------------------------------------
// k_unmask_range: dev[j] ^= K[(ph + j) % 4] over positions [lo, hi), the
// device analogue of websocket_mask (websocket_frame_mask.h:14-24).
// kw = aligned_key(K, lo, ph). Persistent workgroups (UNMASK_WPC per CU) claim
// tiles of UNMASK_NT x UNMASK_U chunks of 16 bytes from one counter, one claim
// ahead, and keep the next tile's nontemporal loads in flight while the
// current tile is XORed and stored (a register double buffer): every CU
// streams to the end of the range instead of a fixed share of it. The stores
// are sc1|nt (written through past the XCD's L2, as the lattice decoder's).
// Geometry and store policy from scripts/bw_probe11 on the c3 batch, R+W
// (profiles/r06_unmask_ab.txt): one 1024-thread workgroup per CU on 64 KiB
// tiles with sc1|nt stores 6.75 TB/s; two per CU 6.31 (nt stores 6.22, the
// round-3..5 form); 80 KiB tiles 6.65, 96 KiB 6.56, 128 KiB 6.49; 48 KiB
// tiles two per CU 6.15. (Round 3: the fixed 2048-block grid-stride form
// 5.34 TB/s, scripts/bw_probe7.) The two edge chunks store only their
// in-range bytes. The last workgroup out resets the counter. ctr == nullptr (a launch
// captured into a graph, or no scratch slot free for the stream): the same
// loop over static tiles (workgroup b: tiles b, b + grid, ...), no state
// outside the launch, so a replay may run on any stream, concurrently too.
#define UNMASK_NT 1024u
#define UNMASK_U 4u
#define UNMASK_WPC 1u
#define UNMASK_AUX_ST 18  // sc1 | nt
__global__ void __launch_bounds__(UNMASK_NT) k_unmask_range(uint8_t* __restrict__ base, uint64_t lo, uint64_t hi,
                                                            uint32_t kw, uint32_t* __restrict__ ctr) {
  constexpr uint32_t TILE = UNMASK_NT * UNMASK_U;  // chunks per tile
  const uint64_t c0 = lo >> 4, c1 = (hi + 15) >> 4;
  const uint64_t ntiles = (c1 - c0 + TILE - 1) / TILE;
  const uint32_t t = threadIdx.x;
  __shared__ uint64_t s_tile;
  uint64_t ahead = ~0ull;  // thread 0: the tile claimed one tile ahead
  if (t == 0) {
    const uint64_t a = ctr ? atomicAdd(ctr, 1u) : blockIdx.x;
    s_tile = a < ntiles ? a : ~0ull;
    if (a < ntiles) {
      const uint64_t b = ctr ? atomicAdd(ctr, 1u) : (uint64_t)blockIdx.x + gridDim.x;
      ahead = b < ntiles ? b : ~0ull;
    }
  }
  __syncthreads();
  uint64_t cur = s_tile;
  // chunk range [c0, c1) as buffer offsets from base + 16*c0; loads past it read
  // zero, stores past it are dropped
  const uint64_t nbytes = (c1 - c0) * 16;
  auto rsrc = [&](uint64_t tile) {
    const uint64_t off = tile * TILE * 16;
    const uint64_t room = nbytes - off;
    return __builtin_amdgcn_make_buffer_rsrc(base + c0 * 16 + off, 0,
                                             room < TILE * 16 ? (uint32_t)room : TILE * 16, 0x00020000);
  };
  u32x4 e[UNMASK_U];
  if (cur != ~0ull) {
    const auto r = rsrc(cur);
#pragma unroll
    for (uint32_t u = 0; u < UNMASK_U; u++)
      e[u] = __builtin_amdgcn_raw_buffer_load_b128(r, t * 16u, u * UNMASK_NT * 16u, 2);
  }
  while (cur != ~0ull) {
    __syncthreads();  // (s_tile is rewritten below)
    if (t == 0) {
      s_tile = ahead;
      if (ahead != ~0ull) {
        const uint64_t b = ctr ? atomicAdd(ctr, 1u) : ahead + gridDim.x;
        ahead = b < ntiles ? b : ~0ull;
      }
    }
    __syncthreads();
    const uint64_t nx = s_tile;
    u32x4 d[UNMASK_U];
#pragma unroll
    for (uint32_t u = 0; u < UNMASK_U; u++) d[u] = e[u] ^ kw;
    if (nx != ~0ull) {
      const auto r = rsrc(nx);
#pragma unroll
      for (uint32_t u = 0; u < UNMASK_U; u++)
        e[u] = __builtin_amdgcn_raw_buffer_load_b128(r, t * 16u, u * UNMASK_NT * 16u, 2);
    }
    const auto w = rsrc(cur);
    // (a tile away from both ends stores every chunk whole: a uniform branch)
    const uint64_t tc = c0 + cur * TILE;  // the tile's first chunk
    if (tc << 4 >= lo && (tc + TILE) << 4 <= hi) {
#pragma unroll
      for (uint32_t u = 0; u < UNMASK_U; u++) {
        __builtin_amdgcn_raw_buffer_store_b128(d[u], w, t * 16u, u * UNMASK_NT * 16u, UNMASK_AUX_ST);
        // (the store's data registers stay live past the next store)
        asm volatile("" ::"v"(d[u].x), "v"(d[u].y), "v"(d[u].z), "v"(d[u].w));
      }
    } else {
#pragma unroll
      for (uint32_t u = 0; u < UNMASK_U; u++) {
        const uint64_t c = tc + u * UNMASK_NT + t;  // absolute chunk
        const uint64_t a = c << 4;
        const bool whole = a >= lo && a + 16 <= hi;
        __builtin_amdgcn_raw_buffer_store_b128(d[u], w, whole ? t * 16u : 0x80000000u, u * UNMASK_NT * 16u,
                                               UNMASK_AUX_ST);
        asm volatile("" ::"v"(d[u].x), "v"(d[u].y), "v"(d[u].z), "v"(d[u].w));
        if (!whole && c < c1) {  // an edge chunk: its in-range bytes
          for (uint32_t b = 0; b < 16; b++) {
            const uint64_t q = a + b;
            const uint32_t wd = b < 4 ? d[u].x : b < 8 ? d[u].y : b < 12 ? d[u].z : d[u].w;
            if (q >= lo && q < hi) base[q] = (uint8_t)(wd >> (8u * (b & 3u)));
          }
        }
      }
    }
    asm volatile("s_nop 1" ::: "memory");
    cur = nx;
  }
  __syncthreads();
  if (t == 0 && ctr) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const uint32_t n = atomicAdd(ctr + 1, 1u);
    if (n + 1 == gridDim.x) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------------------
// k_parse_indexed: one lane per frame start (ascending, caller supplied).
__global__ void __launch_bounds__(256) k_parse_indexed(const uint8_t* __restrict__ base, uint64_t lo,
                                                       uint64_t hi, const uint64_t* __restrict__ starts,
                                                       uint64_t n, frame_table tab,
                                                       xyws_frame* __restrict__ frames) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t len = hi - lo;
  const uint64_t s_rel = starts[i];
  const uint64_t s = lo + (s_rel < len ? s_rel : len);
  uint8_t hb[XYWS_MAX_FRAME_HEADER_SIZE];
  uint32_t avail = 0;
  for (; avail < XYWS_MAX_FRAME_HEADER_SIZE && s + avail < hi; avail++) hb[avail] = base[s + avail];
  hdr_info h = parse_header_bytes(hb, avail);
  xyws_frame f;
  f.frame_off = (int64_t)s_rel;
  f.payload_off = (int64_t)s_rel;
  f.payload_len = 0;
  f.flags = 0; f.hdr_len = 0; f.status = 0; f.reserved = 0;
  f.key[0] = f.key[1] = f.key[2] = f.key[3] = 0;
  uint64_t ps = s, pe = s;
  if (h.hlen && s_rel < len) {
    ps = s + h.hlen;
    uint64_t end = sat_add(ps, h.plen);
    pe = end < hi ? end : hi;
    uint8_t st = h.status;
    if (end > hi) st |= XYWS_ST_PAYLOAD_INCOMPLETE;
    if (i + 1 < n) {  // clip at the next caller start (relative coordinates: no overflow)
      const uint64_t nx_rel = starts[i + 1];
      if (end - lo > nx_rel) st |= XYWS_ST_OVERLAP;
      if (nx_rel < len && pe > lo + nx_rel) pe = lo + nx_rel;
    }
    if (pe < ps) pe = ps;
    f.payload_off = (int64_t)(s_rel + h.hlen);
    f.payload_len = h.plen;
    f.key[0] = (uint8_t)h.key; f.key[1] = (uint8_t)(h.key >> 8);
    f.key[2] = (uint8_t)(h.key >> 16); f.key[3] = (uint8_t)(h.key >> 24);
    f.flags = h.flags;
    f.hdr_len = (uint8_t)h.hlen;
    f.status = st;
  }
  tab.start[i] = s;
  tab.ps[i] = ps;
  tab.pe[i] = pe;
  tab.kw[i] = aligned_key(h.key, ps, 0);
  if (i == 0) *tab.count = n;
  if (frames) frames[i] = f;
}

// ---------------------------------------------------------------------------
// k_stream_serial: exact one-lane chase (XYWS_OPT_SERIAL_SCAN). Writes the
// frame table, descriptors, count and carry. Latency bound by design: it is
// the simplest statement of the stream semantics on the device.
__global__ void k_stream_serial(const uint8_t* __restrict__ base, uint64_t lo, uint64_t hi,
                                const xyws_carry* __restrict__ cin, xyws_carry* __restrict__ cout,
                                frame_table tab, uint64_t tab_cap, xyws_frame* __restrict__ frames,
                                uint64_t cap, uint64_t* __restrict__ nframes,
                                uint32_t* __restrict__ err) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  xyws_carry c;
  if (cin) c = *cin; else memset(&c, 0, sizeof c);
  uint64_t pos = lo, nt = 0, nf = 0;
  if (c.payload_remaining) {
    uint64_t take = c.payload_remaining < hi - lo ? c.payload_remaining : hi - lo;
    uint32_t k = (uint32_t)c.key[0] | ((uint32_t)c.key[1] << 8) | ((uint32_t)c.key[2] << 16) |
                 ((uint32_t)c.key[3] << 24);
    tab.start[nt] = lo; tab.ps[nt] = lo; tab.pe[nt] = lo + take;
    tab.kw[nt] = aligned_key(k, lo, c.phase);
    nt++;
    c.phase += take;
    c.payload_remaining -= take;
    pos = lo + take;
    if (!c.payload_remaining) { c.phase = 0; c.key[0] = c.key[1] = c.key[2] = c.key[3] = 0; }
  }
  while (pos < hi) {
    uint8_t hb[XYWS_MAX_FRAME_HEADER_SIZE];
    uint32_t h0 = c.hdr_len, avail = h0;
    for (uint32_t i = 0; i < h0; i++) hb[i] = c.hdr[i];
    for (; avail < XYWS_MAX_FRAME_HEADER_SIZE && pos + (avail - h0) < hi; avail++)
      hb[avail] = base[pos + (avail - h0)];
    hdr_info h = parse_header_bytes(hb, avail);
    if (!h.hlen) {  // incomplete header: carry its bytes
      for (uint32_t i = h0; i < avail; i++) c.hdr[i] = hb[i];
      c.hdr_len = (uint8_t)avail;
      pos = hi;
      break;
    }
    const uint64_t ps = pos + (h.hlen - h0);
    const uint64_t end = sat_add(ps, h.plen);
    uint8_t st = h.status;
    uint64_t pe = end;
    if (end > hi) {
      pe = hi;
      st |= XYWS_ST_PAYLOAD_INCOMPLETE;
      c.payload_remaining = h.plen - (hi - ps);
      c.phase = hi - ps;
      c.key[0] = (uint8_t)h.key; c.key[1] = (uint8_t)(h.key >> 8);
      c.key[2] = (uint8_t)(h.key >> 16); c.key[3] = (uint8_t)(h.key >> 24);
    }
    if (nt >= tab_cap) { atomicOr(err, 1u); break; }
    tab.start[nt] = pos; tab.ps[nt] = ps; tab.pe[nt] = pe; tab.kw[nt] = aligned_key(h.key, ps, 0);
    nt++;
    if (frames && nf < cap) {
      xyws_frame f;
      f.frame_off = (int64_t)(pos - lo) - (int64_t)h0;
      f.payload_off = (int64_t)(ps - lo);
      f.payload_len = h.plen;
      f.key[0] = (uint8_t)h.key; f.key[1] = (uint8_t)(h.key >> 8);
      f.key[2] = (uint8_t)(h.key >> 16); f.key[3] = (uint8_t)(h.key >> 24);
      f.flags = h.flags; f.hdr_len = (uint8_t)h.hlen; f.status = st; f.reserved = 0;
      frames[nf] = f;
    }
    nf++;
    c.hdr_len = 0;
    for (int i = 0; i < 14; i++) c.hdr[i] = 0;
    pos = pe;
  }
  c.frames_total += nf;
  *tab.count = nt;
  if (nframes) *nframes = nf;
  if (cout) *cout = c;
}

// ---------------------------------------------------------------------------
// k_unmask_tiles: 16 KiB byte tiles over [lo, hi). Each workgroup stages the
// frame-table slice that touches its tile in LDS; each lane handles four
// 16-byte chunks (coalesced: chunk = tile*1024 + k*256 + lane).
__global__ void __launch_bounds__(UNMASK_THREADS) k_unmask_tiles(uint8_t* __restrict__ base, uint64_t lo,
                                                                 uint64_t hi, frame_table tab) {
  __shared__ uint64_t s_ps[UNMASK_LDS_FRAMES], s_pe[UNMASK_LDS_FRAMES];
  __shared__ uint32_t s_kw[UNMASK_LDS_FRAMES];
  __shared__ uint64_t s_f0, s_f1;
  const uint64_t n = *tab.count;
  const uint64_t t0 = lo & ~(uint64_t)(UNMASK_TILE - 1);
  const uint64_t ntiles = (hi - t0 + UNMASK_TILE - 1) / UNMASK_TILE;
  u32x4* __restrict__ p = reinterpret_cast<u32x4*>(base);
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t ts = t0 + tile * UNMASK_TILE, te = ts + UNMASK_TILE;
    if (threadIdx.x == 0) {
      // f0: first frame with pe > ts; f1: first frame with ps >= te (pe, ps non-decreasing)
      uint64_t a = 0, b = n;
      while (a < b) { uint64_t m = (a + b) >> 1; if (tab.pe[m] > ts) b = m; else a = m + 1; }
      s_f0 = a;
      b = n;
      while (a < b) { uint64_t m = (a + b) >> 1; if (tab.ps[m] >= te) b = m; else a = m + 1; }
      s_f1 = a;
    }
    __syncthreads();
    const uint64_t f0 = s_f0, f1 = s_f1, nf = f1 - f0;
    const bool in_lds = nf <= UNMASK_LDS_FRAMES;
    if (in_lds) {
      for (uint64_t i = threadIdx.x; i < nf; i += blockDim.x) {
        s_ps[i] = tab.ps[f0 + i]; s_pe[i] = tab.pe[f0 + i]; s_kw[i] = tab.kw[f0 + i];
      }
    }
    __syncthreads();
    if (nf) {
#pragma unroll
      for (uint32_t k = 0; k < UNMASK_TILE / (16u * UNMASK_THREADS); k++) {
        const uint64_t a = ts + ((uint64_t)k * UNMASK_THREADS + threadIdx.x) * 16u;
        if (a + 16 <= lo || a >= hi) continue;
        // first frame with pe > a
        uint64_t g;
        {
          uint64_t x = 0, y = nf;
          while (x < y) {
            uint64_t m = (x + y) >> 1;
            uint64_t pem = in_lds ? s_pe[m] : tab.pe[f0 + m];
            if (pem > a) y = m; else x = m + 1;
          }
          g = x;
        }
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        for (; g < nf; g++) {
          const uint64_t ps = in_lds ? s_ps[g] : tab.ps[f0 + g];
          if (ps >= a + 16) break;
          const uint64_t pe = in_lds ? s_pe[g] : tab.pe[f0 + g];
          const uint32_t kw = in_lds ? s_kw[g] : tab.kw[f0 + g];
#pragma unroll
          for (uint32_t d = 0; d < 4; d++) w[d] |= kw & range_mask(a + 4 * d, ps, pe);
        }
        if ((w[0] | w[1] | w[2] | w[3]) == 0u) continue;
        if (a >= lo && a + 16 <= hi) {
          u32x4 v = p[a >> 4];
          v.x ^= w[0]; v.y ^= w[1]; v.z ^= w[2]; v.w ^= w[3];
          p[a >> 4] = v;
        } else {
          for (uint32_t t = 0; t < 16; t++) {
            uint64_t q = a + t;
            uint8_t x = (uint8_t)(w[t >> 2] >> (8u * (t & 3u)));
            if (q >= lo && q < hi && x) base[q] ^= x;
          }
        }
      }
    }
    __syncthreads();
  }
}

// ===========================================================================
// C-ABI
// ===========================================================================
using namespace xyws_internal;

extern "C" {

int xyws_abi_version(void) { return XYWS_ABI_VERSION; }

const char* xyws_strerror(int code) {
  switch (code) {
    case XYWS_OK: return "ok";
    case XYWS_ERR_INVALID: return "invalid argument";
    case XYWS_ERR_HIP: return "HIP runtime error";
    case XYWS_ERR_NOMEM: return "device allocation failed";
    case XYWS_ERR_CAPACITY: return "scratch capacity exceeded";
    case XYWS_ERR_DEVICE: return "device-side error";
    case XYWS_ERR_AGAIN: return "not complete yet";
    default: return "unknown error";
  }
}

int xyws_ctx_create(int device, xyws_ctx** out) {
  if (!out) return XYWS_ERR_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return XYWS_ERR_HIP;
  if (device < 0 || device >= ndev) return XYWS_ERR_INVALID;
  device_guard g(device);
  if (!g.ok) return XYWS_ERR_HIP;
  xyws_ctx* c = new xyws_ctx();
  c->device = device;
  c->err = nullptr;
  c->reserve_bytes = 0;
  c->reserve_frames = 0;
  c->reserve_iov = 0;
  c->stage = nullptr;
  c->stage_cap = 0;
  for (auto& st : c->arena_stream) st = nullptr;
  c->arena_rr = 0;
  for (auto& sl : c->slot) {
    sl.bound = false;
    sl.stream = nullptr;
    sl.tab_mem = nullptr;
    sl.aux_mem = nullptr;
    sl.aux_cap = 0;
    sl.iov_mem = nullptr;
    sl.iov_cap = 0;
    sl.tab_cap = 0;
    stream_scratch_init(&sl.ss, device);
  }
  if (hipMalloc(&c->err, 64) != hipSuccess) {
    delete c;
    return XYWS_ERR_NOMEM;
  }
  if (zero_now(c->err, 64) != hipSuccess) {
    (void)hipFree(c->err);
    delete c;
    return XYWS_ERR_HIP;
  }
  *out = c;
  return XYWS_OK;
}

int xyws_ctx_destroy(xyws_ctx* ctx) {
  if (!ctx) return XYWS_ERR_INVALID;
  {
    device_guard g(ctx->device);
    (void)hipDeviceSynchronize();
    for (auto& sl : ctx->slot) {
      if (sl.tab_mem) (void)hipFree(sl.tab_mem);
      if (sl.aux_mem) (void)hipFree(sl.aux_mem);
      if (sl.iov_mem) (void)hipFree(sl.iov_mem);
      stream_scratch_free(&sl.ss);
    }
    if (ctx->err) (void)hipFree(ctx->err);
    if (ctx->stage) (void)hipFree(ctx->stage);
    for (auto st : ctx->arena_stream)
      if (st) (void)hipStreamDestroy(st);
  }
  delete ctx;
  return XYWS_OK;
}

int xyws_ctx_reserve(xyws_ctx* ctx, uint64_t max_batch_bytes, uint64_t max_frames) {
  if (!ctx) return XYWS_ERR_INVALID;
  std::lock_guard<std::mutex> lk(ctx->mu);
  device_guard g(ctx->device);
  if (!g.ok) return XYWS_ERR_HIP;
  if (max_batch_bytes > ctx->reserve_bytes) ctx->reserve_bytes = max_batch_bytes;
  if (max_frames > ctx->reserve_frames) ctx->reserve_frames = max_frames;
  bool spare = true;  // the first unbound slot: the one the next new stream binds (acquire_slot)
  for (auto& sl : ctx->slot) {
    // the stream decoder's scratch (small: ~160 B per 128 KiB segment) in
    // every slot; the per-frame tables in the slots bound to a stream now and
    // in one spare, so that a stream first used inside graph capture finds
    // them (the others get them when a stream binds them: acquire_slot)
    int rc = stream_scratch_reserve(&sl.ss, ctx->reserve_bytes);
    if (rc) return rc;
    const bool take = sl.bound || spare;
    if (!sl.bound) spare = false;
    if (ctx->reserve_frames && take) {
      if ((rc = ensure_table(&sl, ctx->reserve_frames, false))) return rc;
      if ((rc = stream_scratch_reserve_frames(&sl.ss, ctx->reserve_bytes, ctx->reserve_frames))) return rc;
    }
  }
  return XYWS_OK;
}

int xyws_ctx_reserve_iov(xyws_ctx* ctx, uint64_t max_total_bytes) {
  if (!ctx) return XYWS_ERR_INVALID;
  std::lock_guard<std::mutex> lk(ctx->mu);
  device_guard g(ctx->device);
  if (!g.ok) return XYWS_ERR_HIP;
  const uint64_t bytes = max_total_bytes + 16;  // (xyws_decode_stream_iov's staging: total + 16)
  if (bytes > ctx->reserve_iov) ctx->reserve_iov = bytes;
  // the slots bound to a stream now and one spare (the one the next new
  // stream binds), as xyws_ctx_reserve's per-frame tables; the others get
  // theirs when a stream binds them (acquire_slot)
  bool spare = true;
  for (auto& sl : ctx->slot) {
    const bool take = sl.bound || spare;
    if (!sl.bound) spare = false;
    if (take)
      if (const int rc = ensure_iov(&sl, ctx->reserve_iov, false)) return rc;
  }
  return XYWS_OK;
}

int xyws_ctx_last_device_error(xyws_ctx* ctx, uint32_t* out) {
  if (!ctx || !out) return XYWS_ERR_INVALID;
  std::lock_guard<std::mutex> lk(ctx->mu);
  device_guard g(ctx->device);
  if (hipDeviceSynchronize() != hipSuccess) return XYWS_ERR_HIP;
  uint32_t v = 0;
  if (hipMemcpy(&v, ctx->err, 4, hipMemcpyDeviceToHost) != hipSuccess) return XYWS_ERR_HIP;
  if (v && zero_now(ctx->err, 4) != hipSuccess) return XYWS_ERR_HIP;
  for (auto& sl : ctx->slot) v |= stream_scratch_error(&sl.ss, true);
  *out = v;
  return v ? XYWS_ERR_DEVICE : XYWS_OK;
}

// Internal (not part of include/xyws.h): resolution counters of the last fused
// stream decode run with XYWS_OPT_STATS (0x100) on `stream`. Synchronizes the
// device. out: XYWS_NSTATS words.
int xyws_debug_stats(xyws_ctx* ctx, void* stream, uint64_t* out) {
  if (!ctx || !out) return XYWS_ERR_INVALID;
  std::lock_guard<std::mutex> lk(ctx->mu);
  device_guard g(ctx->device);
  for (auto& sl : ctx->slot)
    if (sl.bound && sl.stream == (hipStream_t)stream) return stream_scratch_stats(&sl.ss, out);
  return XYWS_ERR_INVALID;
}

// Internal: the run records of the last fused stream decode on `stream`, at
// most max_runs of them; returns the count copied or a negative error.
// Synchronizes the device.
int64_t xyws_debug_records(xyws_ctx* ctx, void* stream, uint64_t* out, uint64_t max_runs) {
  if (!ctx || !out) return XYWS_ERR_INVALID;
  std::lock_guard<std::mutex> lk(ctx->mu);
  device_guard g(ctx->device);
  for (auto& sl : ctx->slot)
    if (sl.bound && sl.stream == (hipStream_t)stream) return stream_scratch_records(&sl.ss, out, max_runs);
  return XYWS_ERR_INVALID;
}

// Internal: the lattice decoder's device-side choice on `stream`: {the device
// policy word (bit 63 a call finished, bits 48..55 its decoder, bits 0..47
// the size all its frames had or 0), lattice calls handed whole to the run
// decoder on that word, ... by the prologue's checks (first frame, lattice
// points 1-2), lattice calls whose segment loops ran in 75 KiB segments, ...
// in 120 KiB segments} (counts per stream slot, cumulative). Synchronizes the
// device. out: 5 words.
int xyws_debug_lattice(xyws_ctx* ctx, void* stream, uint64_t* out) {
  if (!ctx || !out) return XYWS_ERR_INVALID;
  std::lock_guard<std::mutex> lk(ctx->mu);
  device_guard g(ctx->device);
  for (auto& sl : ctx->slot)
    if (sl.bound && sl.stream == (hipStream_t)stream) return stream_scratch_lattice(&sl.ss, out);
  return XYWS_ERR_INVALID;
}

// Internal: the decoder-choice words the last fused stream decode on `stream`
// published ({epoch, batch bytes, smallest, largest last-frame size, decoder:
// 0 or 2 the run decoder (2: 512-thread workgroups), 3 the lattice
// decoder}). Synchronizes the device.
int xyws_debug_policy(xyws_ctx* ctx, void* stream, uint64_t* out) {
  if (!ctx || !out) return XYWS_ERR_INVALID;
  std::lock_guard<std::mutex> lk(ctx->mu);
  device_guard g(ctx->device);
  if (hipDeviceSynchronize() != hipSuccess) return XYWS_ERR_HIP;
  for (auto& sl : ctx->slot)
    if (sl.bound && sl.stream == (hipStream_t)stream) {
      if (!sl.ss.pol_h) return XYWS_ERR_INVALID;
      for (int i = 0; i < 5; i++) out[i] = sl.ss.pol_h[i];
      return XYWS_OK;
    }
  return XYWS_ERR_INVALID;
}

// xyws_unmask with ctx->mu held: the claim counter is the stream's scratch
// slot's when the stream has one bound or a free slot to bind (eager launches
// only); a captured launch, or a stream finding every slot bound to others,
// takes the static-tile form (ctr == nullptr: no state outside the launch, no
// eviction, no device synchronization).
static int unmask_locked(xyws_ctx* ctx, void* dev, uint64_t len, const uint8_t key[4], uint64_t phase,
                         hipStream_t s) {
  uint32_t* ctr = nullptr;
  uint32_t ncu = 256;
  if (!capturing(s)) {
    scratch_slot* sl = nullptr;
    bool avail = false;
    for (auto& x : ctx->slot) avail = avail || !x.bound || x.stream == s;
    if (avail) {
      if (const int rc = acquire_slot(ctx, s, false, &sl)) return rc;
      if (const int rc = stream_scratch_unmask_counter(&sl->ss, false, &ctr)) return rc;
      ncu = (uint32_t)sl->ss.ncu;
    } else {
      ncu = (uint32_t)ctx->slot[0].ss.ncu;
    }
  } else {
    ncu = (uint32_t)ctx->slot[0].ss.ncu;
  }
  const uintptr_t addr = reinterpret_cast<uintptr_t>(dev);
  uint8_t* base = reinterpret_cast<uint8_t*>(addr & ~(uintptr_t)15);
  const uint64_t lo = addr & 15, hi = lo + len;
  const uint32_t k = (uint32_t)key[0] | ((uint32_t)key[1] << 8) | ((uint32_t)key[2] << 16) |
                     ((uint32_t)key[3] << 24);
  // aligned_key(k, lo, phase) on the host: rotation by (phase - lo) mod 4
  const uint32_t c = (uint32_t)(phase - lo) & 3u;
  const uint32_t kw = c ? ((k >> (8u * c)) | (k << (32u - 8u * c))) : k;
  const uint64_t chunks = ((hi + 15) >> 4) - (lo >> 4);
  const uint32_t grid = grid_for(chunks, UNMASK_NT * UNMASK_U, ncu * UNMASK_WPC);
  hipLaunchKernelGGL(k_unmask_range, dim3(grid), dim3(UNMASK_NT), 0, s, base, lo, hi, kw, ctr);
  return hip_err(hipGetLastError());
}

int xyws_unmask(xyws_ctx* ctx, void* dev, uint64_t len, const uint8_t key[4], uint64_t phase,
                uint64_t* phase_out, void* stream) {
  if (!ctx || !key || (!dev && len)) return XYWS_ERR_INVALID;
  if (phase_out) *phase_out = phase + len;
  if (!len) return XYWS_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  device_guard g(ctx->device);
  if (!g.ok) return XYWS_ERR_HIP;
  return unmask_locked(ctx, dev, len, key, phase, (hipStream_t)stream);
}

int xyws_pointer_device(const void* p, int* device) {
  if (!device) return XYWS_ERR_INVALID;
  *device = -1;
  if (!p) return XYWS_OK;
  hipPointerAttribute_t attr;
  const bool on_dev = hipPointerGetAttributes(&attr, p) == hipSuccess && attr.type == hipMemoryTypeDevice;
  (void)hipGetLastError();  // (an unregistered host pointer leaves an error behind)
  if (on_dev) *device = attr.device;
  return XYWS_OK;
}

// websocket_mask with the reference's contract (websocket_frame_mask.h:14,
// called at example/include/common/websocket.h:131): host or device bytes,
// done when it returns. Device bytes are unmasked in place; host bytes go
// through the context's device stage (copy in, k_unmask_range, copy out).
int xyws_mask_bytes(xyws_ctx* ctx, void* data, uint64_t len, const uint8_t key[4], uint64_t phase,
                    uint64_t* phase_out, void* stream) {
  if (!ctx || !key || (!data && len)) return XYWS_ERR_INVALID;
  if (phase_out) *phase_out = phase + len;
  if (!len) return XYWS_OK;
  device_guard g(ctx->device);
  if (!g.ok) return XYWS_ERR_HIP;
  hipStream_t s = (hipStream_t)stream;
  if (capturing(s)) return XYWS_ERR_CAPACITY;  // (synchronous by contract)
  int pdev = -1;
  if (const int rc = xyws_pointer_device(data, &pdev)) return rc;
  if (pdev >= 0) {
    if (pdev != ctx->device) return XYWS_ERR_INVALID;  // (another device's memory: its own context)
    if (const int rc = xyws_unmask(ctx, data, len, key, phase, nullptr, stream)) return rc;
    return hip_err(hipStreamSynchronize(s));
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (ctx->stage_cap < len) {
    if (ctx->stage) {
      (void)hipStreamSynchronize(s);
      (void)hipFree(ctx->stage);
      ctx->stage = nullptr;
      ctx->stage_cap = 0;
    }
    const uint64_t cap = len < 4096 ? 4096 : len;
    if (hipMalloc(&ctx->stage, cap) != hipSuccess) return XYWS_ERR_NOMEM;
    ctx->stage_cap = cap;
  }
  // the stage keeps the bytes' 16-byte phase, so the kernel sees the same lanes
  if (hipMemcpyAsync(ctx->stage, data, len, hipMemcpyHostToDevice, s) != hipSuccess) return XYWS_ERR_HIP;
  if (const int rc = unmask_locked(ctx, ctx->stage, len, key, phase, s)) return rc;
  if (hipMemcpyAsync(data, ctx->stage, len, hipMemcpyDeviceToHost, s) != hipSuccess) return XYWS_ERR_HIP;
  return hip_err(hipStreamSynchronize(s));
}

int xyws_decode_indexed(xyws_ctx* ctx, void* dev_buf, uint64_t len, const uint64_t* dev_starts,
                        uint64_t n, xyws_frame* dev_frames, uint32_t opts, void* stream) {
  if (!ctx || (!dev_buf && len) || (!dev_starts && n)) return XYWS_ERR_INVALID;
  if (!n) return XYWS_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  device_guard g(ctx->device);
  if (!g.ok) return XYWS_ERR_HIP;
  hipStream_t s = (hipStream_t)stream;
  const bool cap = capturing(s);
  scratch_slot* sl = nullptr;
  int rc = acquire_slot(ctx, s, cap, &sl);
  if (rc) return rc;
  if ((rc = ensure_table(sl, n, cap))) return rc;
  const uintptr_t addr = reinterpret_cast<uintptr_t>(dev_buf);
  uint8_t* base = reinterpret_cast<uint8_t*>(addr & ~(uintptr_t)15);
  const uint64_t lo = addr & 15, hi = lo + len;
  frame_table t = table_of(sl);
  hipLaunchKernelGGL(k_parse_indexed, dim3(grid_for(n, 256, 1u << 30)), dim3(256), 0, s, base, lo, hi,
                     dev_starts, n, t, dev_frames);
  if ((rc = hip_err(hipGetLastError()))) return rc;
  if (!(opts & XYWS_OPT_PARSE_ONLY) && len) {
    const uint64_t tiles = (hi - (lo & ~(uint64_t)(UNMASK_TILE - 1)) + UNMASK_TILE - 1) / UNMASK_TILE;
    hipLaunchKernelGGL(k_unmask_tiles, dim3(grid_for(tiles, 1, 4096)), dim3(UNMASK_THREADS), 0, s,
                       base, lo, hi, t);
    if ((rc = hip_err(hipGetLastError()))) return rc;
  }
  return XYWS_OK;
}

int xyws_decode_stream(xyws_ctx* ctx, void* dev_buf, uint64_t len, const xyws_carry* dev_carry_in,
                       xyws_carry* dev_carry_out, xyws_frame* dev_frames, uint64_t cap,
                       uint64_t* dev_nframes, uint32_t opts, void* stream) {
  if (!ctx || (!dev_buf && len)) return XYWS_ERR_INVALID;
  if (len >= (1ull << 46) - 64) return XYWS_ERR_INVALID;  // (entry granules hold 46-bit positions)
  std::lock_guard<std::mutex> lk(ctx->mu);
  device_guard g(ctx->device);
  if (!g.ok) return XYWS_ERR_HIP;
  const uintptr_t addr = reinterpret_cast<uintptr_t>(dev_buf);
  uint8_t* base = reinterpret_cast<uint8_t*>(addr & ~(uintptr_t)15);
  const uint64_t lo = addr & 15, hi = lo + len;
  hipStream_t s = (hipStream_t)stream;
  const bool capt = capturing(s);
  scratch_slot* sl = nullptr;
  int rc = acquire_slot(ctx, s, capt, &sl);
  if (rc) return rc;
  if ((opts & XYWS_OPT_SERIAL_SCAN) || !XYWS_HAVE_FUSED) {
    // worst case is a 2-byte unmasked frame every 2 bytes; the debug path caps
    // its table at 2^24 frames and flags the device error word beyond that.
    uint64_t want = len / 2 + 2;
    if (want > (1ull << 24)) want = 1ull << 24;
    if ((rc = ensure_table(sl, want, capt))) return rc;
    frame_table t = table_of(sl);
    hipLaunchKernelGGL(k_stream_serial, dim3(1), dim3(64), 0, s, base, lo, hi, dev_carry_in,
                       dev_carry_out, t, sl->tab_cap, dev_frames, cap, dev_nframes, ctx->err);
    if ((rc = hip_err(hipGetLastError()))) return rc;
    if (!(opts & XYWS_OPT_PARSE_ONLY) && len) {
      const uint64_t tiles = (hi - (lo & ~(uint64_t)(UNMASK_TILE - 1)) + UNMASK_TILE - 1) / UNMASK_TILE;
      hipLaunchKernelGGL(k_unmask_tiles, dim3(grid_for(tiles, 1, 4096)), dim3(UNMASK_THREADS), 0, s,
                         base, lo, hi, t);
      if ((rc = hip_err(hipGetLastError()))) return rc;
    }
    return XYWS_OK;
  }
  return stream_decode_fused(&sl->ss, base, lo, hi, dev_carry_in, dev_carry_out, dev_frames, cap,
                             dev_nframes, opts, s);
}

// ---------------------------------------------------------------------------
// xyws_decode_stream_iov: a recv's buffer sequence (buffer.h:94-110, filled by
// recv_all.h:99-121) decoded as one stream — the pieces gathered into the
// slot's staging buffer by one launch, one fused decode there, the bytes
// scattered back by one launch: three launches whatever the piece count (one
// decode per piece would cost a decode's fixed latency each). The piece
// table travels in the kernel arguments.
struct iov_args {
  uint8_t* base[XYWS_IOV_MAX];
  uint64_t len[XYWS_IOV_MAX];
  uint64_t off[XYWS_IOV_MAX];  // the piece's start in the staging buffer
};
// One piece per blockIdx.y; lane i of the grid moves the i-th 16-byte line of
// the destination: its source bytes are the two aligned source lines around
// them and a funnel shift (lines holding no byte of the piece are not
// loaded), whatever the two alignments; the lines at the piece's two ends
// are stored bytewise. to_stage: pieces -> stage, else back.
XYWS_DEV u32x4 iov_funnel(const u32x4& x, const u32x4& y, uint32_t sh) {
  const uint64_t x0 = (uint64_t)x.x | ((uint64_t)x.y << 32), x1 = (uint64_t)x.z | ((uint64_t)x.w << 32);
  const uint64_t y0 = (uint64_t)y.x | ((uint64_t)y.y << 32);
  const uint64_t y1 = (uint64_t)y.z | ((uint64_t)y.w << 32);
  const bool h = sh >= 8;
  const uint64_t a = h ? x1 : x0, b = h ? y0 : x1, c = h ? y1 : y0;
  const uint32_t s8 = 8u * (sh & 7u);
  const uint64_t r0 = s8 ? (a >> s8) | (b << (64u - s8)) : a, r1 = s8 ? (b >> s8) | (c << (64u - s8)) : b;
  return u32x4{(uint32_t)r0, (uint32_t)(r0 >> 32), (uint32_t)r1, (uint32_t)(r1 >> 32)};
}
__global__ void __launch_bounds__(256) k_iov_copy(iov_args A, uint8_t* __restrict__ stage, int to_stage) {
  const uint32_t k = blockIdx.y;
  const uint64_t n = A.len[k];
  if (!n) return;
  uint8_t* sp = stage + A.off[k];
  const uint8_t* src = to_stage ? A.base[k] : sp;
  uint8_t* dst = to_stage ? sp : A.base[k];
  const uint64_t d0 = reinterpret_cast<uintptr_t>(dst), d1 = d0 + n;
  const uint64_t s0 = reinterpret_cast<uintptr_t>(src), s1 = s0 + n;
  const uint64_t c0 = d0 & ~15ull, nch = (d1 - c0 + 15) / 16;
  const u32x4 z = {0u, 0u, 0u, 0u};
  for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < nch; c += (uint64_t)gridDim.x * 256) {
    const uint64_t D = c0 + 16 * c, S = D - d0 + s0;  // (S: the source of byte D; wraps below s0 in line 0)
    const uint64_t Sa = S & ~15ull;
    const uint32_t sh = (uint32_t)(S & 15u);
    const u32x4 x = Sa + 16 > s0 && Sa < s1 ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(Sa)) : z;
    const u32x4 y = sh && Sa + 32 > s0 && Sa + 16 < s1
                        ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(Sa + 16)) : z;
    const u32x4 v = sh ? iov_funnel(x, y, sh) : x;
    if (D >= d0 && D + 16 <= d1) {
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(D));
    } else {
      for (uint32_t t = 0; t < 16; t++) {
        const uint32_t w = t < 4 ? v.x : t < 8 ? v.y : t < 12 ? v.z : v.w;  // (no dynamic index: no scratch)
        if (D + t >= d0 && D + t < d1) *reinterpret_cast<uint8_t*>(D + t) = (uint8_t)(w >> (8u * (t & 3u)));
      }
    }
  }
}

// The buffer-sequence decode in pieces (xyws_decode_stream_iov): out ==
// nullptr: *cnt = the stream's frame count before the call (0 for a fresh
// stream); else *out = c's count minus it (the frames of the call).
__global__ void k_iov_count(const xyws_carry* c, uint64_t* cnt, uint64_t* out) {
  if (threadIdx.x) return;
  const uint64_t v = c ? c->frames_total : 0;
  if (out) *out = v - *cnt;
  else *cnt = v;
}
// Pieces at least this long (empty ones not counted) are decoded in place one
// by one when no descriptors are asked for (see xyws_decode_stream_iov): a
// piece costs one decode's fixed cost instead of two more passes over its
// bytes (~0.8 us per MiB). That cost follows the frames: ~20 us after a
// call of equal frames (the lattice decoder), up to ~200 us after mixed
// ones (the run decoder's entry scans). Measured (profiles/r06_iov_rate.jsonl,
// gather/decode/scatter vs in place): c3 in 4 pieces 2.67 vs 0.72 ms, in 16
// (128 MiB) 2.47 vs 0.97; c1 in 16 (16 MiB) 0.33 vs 0.42; c4 in 8 (128 MiB)
// 1.46 vs 1.73.
constexpr uint64_t IOV_PIECE_MIN_EQUAL = 64ull << 20, IOV_PIECE_MIN_MIXED = 256ull << 20;

int xyws_decode_stream_iov(xyws_ctx* ctx, const xyws_iov* iov, uint32_t niov, const xyws_carry* dev_carry_in,
                           xyws_carry* dev_carry_out, xyws_frame* dev_frames, uint64_t cap,
                           uint64_t* dev_nframes, uint32_t opts, void* stream) {
  if (!ctx || (!iov && niov) || niov > XYWS_IOV_MAX) return XYWS_ERR_INVALID;
  if ((opts & XYWS_OPT_SERIAL_SCAN) || !XYWS_HAVE_FUSED) return XYWS_ERR_INVALID;  // (the fused path only)
  iov_args A;
  uint64_t total = 0, longest = 0;
  constexpr uint64_t LIMIT = (1ull << 46) - 64;
  for (uint32_t k = 0; k < niov; k++) {
    if (!iov[k].base && iov[k].len) return XYWS_ERR_INVALID;
    if (iov[k].len >= LIMIT - total) return XYWS_ERR_INVALID;  // (checked before the add: no wrap)
    A.base[k] = static_cast<uint8_t*>(iov[k].base);
    A.len[k] = iov[k].len;
    A.off[k] = total;
    total += iov[k].len;
    if (iov[k].len > longest) longest = iov[k].len;
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  device_guard g(ctx->device);
  if (!g.ok) return XYWS_ERR_HIP;
  hipStream_t s = (hipStream_t)stream;
  const bool capt = capturing(s);
  scratch_slot* sl = nullptr;
  int rc = acquire_slot(ctx, s, capt, &sl);
  if (rc) return rc;
  // Pieces in place: each piece decoded where it lies as the next batch of the
  // stream, the carry chained from piece to piece on the device (a frame or
  // header cut by a piece's end continues in the next, as across any two
  // batches: the decode of a stream cut at any byte is the decode of the
  // whole), so the bytes move once instead of three times (gather, decode,
  // scatter). One decode per piece: for sequences of few large pieces
  // without descriptors (the frame ordinals and offsets of later pieces
  // would need the earlier pieces' counts on the host). Measured in DESIGN
  // §4.4 (profiles/r06_iov_rate.jsonl).
  uint32_t nz = 0;
  uint64_t minlen = UINT64_MAX;
  for (uint32_t k = 0; k < niov; k++)
    if (iov[k].len) {
      nz++;
      if (iov[k].len < minlen) minlen = iov[k].len;
    }
  const bool desc = dev_frames && cap;
  if (nz == 1 && !(opts & XYWS_OPT_IOV_STAGE)) {
    // one non-empty piece: the decode of that buffer (offsets from its start,
    // which is the sequence's: every piece before it is empty)
    for (uint32_t k = 0; k < niov; k++)
      if (iov[k].len) {
        const uintptr_t addr = reinterpret_cast<uintptr_t>(iov[k].base);
        return stream_decode_fused(&sl->ss, reinterpret_cast<uint8_t*>(addr & ~(uintptr_t)15), addr & 15,
                                   (addr & 15) + iov[k].len, dev_carry_in, dev_carry_out, dev_frames, cap,
                                   dev_nframes, opts, s);
      }
  }
  const volatile uint64_t* pol = sl->ss.pol_h;  // (the stream's previous call: equal frames?)
  const bool equal = pol && pol[3] && pol[2] == pol[3];
  const uint64_t pmin = equal ? IOV_PIECE_MIN_EQUAL : IOV_PIECE_MIN_MIXED;
  const bool pieces = nz > 1 && !desc && !(opts & XYWS_OPT_IOV_STAGE) &&
                      ((opts & XYWS_OPT_IOV_PIECES) || minlen >= pmin);
  if (pieces) {
    // scratch: [0, 64) the carry between pieces, [64, 72) the frame count of
    // the stream before the call (the count is the difference at the end)
    if ((rc = ensure_iov(sl, 128, capt))) return rc;
    xyws_carry* mid = static_cast<xyws_carry*>(sl->iov_mem);
    uint64_t* base_cnt = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(sl->iov_mem) + 64);
    xyws_carry* last_out = dev_carry_out ? dev_carry_out : mid;
    if (dev_nframes) {
      hipLaunchKernelGGL(k_iov_count, dim3(1), dim3(64), 0, s, dev_carry_in, base_cnt, (uint64_t*)nullptr);
      if ((rc = hip_err(hipGetLastError()))) return rc;
    }
    uint32_t j = 0;
    const xyws_carry* cin = dev_carry_in;
    for (uint32_t k = 0; k < niov; k++) {
      if (!iov[k].len) continue;
      const bool lastp = ++j == nz;
      xyws_carry* cout = lastp ? last_out : mid;
      const uintptr_t addr = reinterpret_cast<uintptr_t>(iov[k].base);
      uint8_t* b = reinterpret_cast<uint8_t*>(addr & ~(uintptr_t)15);
      const uint64_t lo = addr & 15;
      if ((rc = stream_decode_fused(&sl->ss, b, lo, lo + iov[k].len, cin, cout, nullptr, 0, nullptr, opts, s)))
        return rc;
      cin = cout;
    }
    if (dev_nframes) {
      hipLaunchKernelGGL(k_iov_count, dim3(1), dim3(64), 0, s, last_out, base_cnt, dev_nframes);
      if ((rc = hip_err(hipGetLastError()))) return rc;
    }
    return XYWS_OK;
  }
  if ((rc = ensure_iov(sl, total + 16, capt))) return rc;
  uint8_t* stage = static_cast<uint8_t*>(sl->iov_mem);
  const dim3 grid((uint32_t)grid_for(longest / 16 + 2, 256, 1024), niov ? niov : 1);
  if (niov && total) {
    hipLaunchKernelGGL(k_iov_copy, grid, dim3(256), 0, s, A, stage, 1);
    if ((rc = hip_err(hipGetLastError()))) return rc;
  }
  if ((rc = stream_decode_fused(&sl->ss, stage, 0, total, dev_carry_in, dev_carry_out, dev_frames, cap,
                                dev_nframes, opts, s)))
    return rc;
  if (niov && total && !(opts & XYWS_OPT_PARSE_ONLY)) {
    hipLaunchKernelGGL(k_iov_copy, grid, dim3(256), 0, s, A, stage, 0);
    if ((rc = hip_err(hipGetLastError()))) return rc;
  }
  return XYWS_OK;
}

// ---------------------------------------------------------------------------
// websocket_frame_header_parser (websocket_frame_header.h:226-385) through the
// device: each parse() hands the bytes that can still belong to the header
// (at most 14 minus those already fed) to the stream decoder in parse-only
// mode with the parser's device-resident carry, then reads back whether a
// header completed. While no header has completed every byte fed so far is a
// header byte, so the bytes consumed in the completing call are its hdr_len
// minus the bytes fed before it (:342, :362, :375); once complete, parse()
// returns npos until reset() (:378-384).
// While a header is incomplete, result() reports what the reference's state
// machine has parsed so far (:305-385): flags from the first byte (FIN, opcode),
// HAS_MASK and the 7-bit length from the second (0 for the 126/127 forms), the
// extended length accumulated big-endian over the bytes received, the mask
// bytes received so far; k_parser_partial computes that on the device from the
// header bytes the decoder's carry holds (at most 13).
struct xyws_parser {
  xyws_ctx* ctx;
  uint8_t* dev;       // device: carry (64 B) | frame (32 B) | count (8 B) | staging (32 B)
  uint8_t* host;      // pinned: frame (32 B) | count (8 B)
  uint64_t fed;       // header bytes fed since reset()
  bool finished;
  xyws_frame res;
};

// The parser's result() after an incomplete header, on the device from the
// decoder's carry (the header bytes fed since reset(), hdr_len <= 13), as the
// reference's state machine leaves it mid-header (websocket_frame_header.h:
// 305-385: flags after byte 0, HAS_MASK and the 7-bit length after byte 1,
// the 16/64-bit length accumulated byte by byte, the mask bytes so far).
// Runs only when the decode completed no header (*count == 0).
__global__ void k_parser_partial(const xyws_carry* __restrict__ carry, const uint64_t* __restrict__ count,
                                 xyws_frame* __restrict__ r) {
  if (threadIdx.x != 0 || *count != 0) return;
  const uint8_t* hb = carry->hdr;
  const unsigned k = carry->hdr_len;
  xyws_frame f = {};  // reset(): no flags, zero mask, zero length
  if (k >= 1) f.flags = (uint8_t)((hb[0] & 0x0Fu) | ((hb[0] & 0x80u) ? XYWS_FLAG_FIN : 0u));
  if (k >= 2) {
    uint64_t len = hb[1] & 0x7Fu;
    if (hb[1] & 0x80u) f.flags |= XYWS_FLAG_HAS_MASK;
    const unsigned ext = len == 127 ? 8 : len == 126 ? 2 : 0;
    if (ext) {
      len = 0;
      for (unsigned i = 2; i < 2 + ext && i < k; i++) len = (len << 8) | hb[i];
    }
    f.payload_len = len;
    if (f.flags & XYWS_FLAG_HAS_MASK)
      for (unsigned i = 2 + ext; i < k && i < 2 + ext + 4; i++) f.key[i - 2 - ext] = hb[i];
  }
  *r = f;
}

int xyws_parser_create(xyws_ctx* ctx, xyws_parser** out) {
  if (!ctx || !out) return XYWS_ERR_INVALID;
  *out = nullptr;
  device_guard g(ctx->device);
  if (!g.ok) return XYWS_ERR_HIP;
  xyws_parser* p = new xyws_parser();
  p->ctx = ctx;
  p->dev = nullptr;
  p->host = nullptr;
  if (hipMalloc(&p->dev, 256) != hipSuccess) {
    delete p;
    return XYWS_ERR_NOMEM;
  }
  if (hipHostMalloc(&p->host, 64, hipHostMallocDefault) != hipSuccess) {
    (void)hipFree(p->dev);
    delete p;
    return XYWS_ERR_NOMEM;
  }
  *out = p;
  return xyws_parser_reset(p);
}

int xyws_parser_destroy(xyws_parser* p) {
  if (!p) return XYWS_ERR_INVALID;
  device_guard g(p->ctx->device);
  (void)hipDeviceSynchronize();
  (void)hipFree(p->dev);
  (void)hipHostFree(p->host);
  delete p;
  return XYWS_OK;
}

int xyws_parser_reset(xyws_parser* p) {
  if (!p) return XYWS_ERR_INVALID;
  device_guard g(p->ctx->device);
  if (!g.ok) return XYWS_ERR_HIP;
  p->fed = 0;
  p->finished = false;
  memset(&p->res, 0, sizeof p->res);
  return hip_err(zero_now(p->dev, 64));  // a zero carry: a fresh parser (s_start)
}

int xyws_parser_parse(xyws_parser* p, const void* data, uint64_t len, uint64_t* consumed, void* stream) {
  if (!p || !consumed || (!data && len)) return XYWS_ERR_INVALID;
  *consumed = XYWS_NPOS;
  if (p->finished || !len) return XYWS_OK;
  device_guard g(p->ctx->device);
  if (!g.ok) return XYWS_ERR_HIP;
  hipStream_t s = (hipStream_t)stream;
  const uint64_t room = XYWS_MAX_FRAME_HEADER_SIZE - p->fed;
  const uint64_t n = len < room ? len : room;
  xyws_carry* carry = reinterpret_cast<xyws_carry*>(p->dev);
  xyws_frame* frame = reinterpret_cast<xyws_frame*>(p->dev + 64);
  uint64_t* count = reinterpret_cast<uint64_t*>(p->dev + 96);
  uint8_t* stage = p->dev + 128;
  // device memory is parsed where it lies; host bytes are staged
  const void* src = data;
  hipPointerAttribute_t attr;
  const bool on_dev = hipPointerGetAttributes(&attr, data) == hipSuccess && attr.type == hipMemoryTypeDevice;
  (void)hipGetLastError();  // (an unregistered host pointer leaves an error behind)
  if (!on_dev) {
    if (hipMemcpyAsync(stage, data, n, hipMemcpyHostToDevice, s) != hipSuccess) return XYWS_ERR_HIP;
    src = stage;
  }
  int rc = xyws_decode_stream(p->ctx, const_cast<void*>(src), n, carry, carry, frame, 1, count,
                              XYWS_OPT_PARSE_ONLY, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_parser_partial, dim3(1), dim3(64), 0, s, carry, count, frame);
  if (hipGetLastError() != hipSuccess) return XYWS_ERR_HIP;
  if (hipMemcpyAsync(p->host, frame, 40, hipMemcpyDeviceToHost, s) != hipSuccess) return XYWS_ERR_HIP;
  if (hipStreamSynchronize(s) != hipSuccess) return XYWS_ERR_HIP;
  uint64_t nf;
  memcpy(&nf, p->host + 32, 8);
  memcpy(&p->res, p->host, sizeof p->res);  // the header, or the partial state (k_parser_partial)
  if (nf == 0) {
    p->fed += n;
    return XYWS_OK;
  }
  p->finished = true;
  *consumed = p->res.hdr_len - p->fed;
  return XYWS_OK;
}

int xyws_parser_result(const xyws_parser* p, uint8_t* flags, uint8_t key[4], uint64_t* length) {
  if (!p) return XYWS_ERR_INVALID;
  if (flags) *flags = p->res.flags;
  if (key) memcpy(key, p->res.key, 4);
  if (length) *length = p->res.payload_len;
  return XYWS_OK;
}

}  // extern "C"

