// xyws_ctx.h — internal: the C-ABI context (per-stream device scratch slots)
// shared by the entry points in xyws.hip and xyws_frames.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <mutex>

#include "xyws.h"
#include "xyws_stream.h"

// ---------------------------------------------------------------------------
// Frame table (device scratch, SoA) consumed by k_unmask_tiles. Entries are
// sorted by position and non-overlapping; [ps, pe) is the payload range to
// unmask (already clipped), kw the key word for 4-byte-aligned positions.
struct frame_table {
  uint64_t* start;
  uint64_t* ps;
  uint64_t* pe;
  uint32_t* kw;
  uint64_t* count;  // number of valid entries (device)
};

// Device scratch is kept per (context, stream): a decode's run records, flags
// and frame table belong to the stream it was enqueued on, so calls on one
// context from several streams (an io_uring service overlapping batches) run
// concurrently without sharing scratch. XYWS_SLOTS streams get a slot each;
// when a further stream arrives while every slot is bound, the device is
// synchronized (every slot idle) and the bindings start over.
#define XYWS_SLOTS 16

struct scratch_slot {
  bool bound;
  hipStream_t stream;
  // frame table scratch (indexed + serial modes)
  void* tab_mem;
  uint64_t tab_cap;
  stream_scratch ss;  // fused stream decoder scratch (xyws_stream.hip)
  // frame-list kernels' scratch (xyws_frames.hip): block sums, message tables
  void* aux_mem;
  uint64_t aux_cap;
  // xyws_decode_stream_iov: the pieces of one buffer sequence, gathered
  void* iov_mem;
  uint64_t iov_cap;
};

struct xyws_ctx {
  int device;
  std::mutex mu;
  uint32_t* err;  // device error word (serial / indexed modes)
  uint64_t reserve_bytes, reserve_frames;  // applied to every slot
  uint64_t reserve_iov;                     // xyws_ctx_reserve_iov: the iov staging buffer of bound slots
  void* stage;          // xyws_mask_bytes: device copy of host bytes (under mu)
  uint64_t stage_cap;
  scratch_slot slot[XYWS_SLOTS];
  // recv arenas share a few streams of the context (arena k: stream k mod
  // XYWS_ARENA_STREAMS), so that any number of connections bind at most that
  // many scratch slots (created on first use, destroyed with the context)
  hipStream_t arena_stream[8];
  uint32_t arena_rr;
};
#define XYWS_ARENA_STREAMS 8

namespace xyws_internal {

struct device_guard {
  int prev = -1;
  bool ok = false;
  explicit device_guard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = hipSetDevice(dev) == hipSuccess;
  }
  ~device_guard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

inline int hip_err(hipError_t e) { return e == hipSuccess ? XYWS_OK : XYWS_ERR_HIP; }

// Zero device memory and wait until it is zero: hipMemset on device memory may
// return before the memset ran (it goes to the null stream, which does not
// order the caller's non-blocking streams); a kernel on such a stream would
// otherwise read the allocation's old contents (scratch tickets, epochs).
inline hipError_t zero_now(void* p, size_t n) {
  hipError_t e = hipMemset(p, 0, n);
  if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
  return e;
}

inline bool capturing(hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(s, &cs);
  return cs != hipStreamCaptureStatusNone;
}

inline int ensure_table(scratch_slot* sl, uint64_t n, bool capture) {
  if (n <= sl->tab_cap && sl->tab_mem) return XYWS_OK;
  if (capture) return XYWS_ERR_CAPACITY;
  uint64_t cap = n < 1024 ? 1024 : n;
  void* mem = nullptr;
  size_t bytes = cap * (8 + 8 + 8 + 4) + 64;
  if (hipMalloc(&mem, bytes) != hipSuccess) return XYWS_ERR_NOMEM;
  if (sl->tab_mem) {
    (void)hipDeviceSynchronize();
    (void)hipFree(sl->tab_mem);
  }
  sl->tab_mem = mem;
  sl->tab_cap = cap;
  return XYWS_OK;
}

inline frame_table table_of(scratch_slot* sl) {
  frame_table t;
  char* m = static_cast<char*>(sl->tab_mem);
  t.start = reinterpret_cast<uint64_t*>(m);
  t.ps = t.start + sl->tab_cap;
  t.pe = t.ps + sl->tab_cap;
  t.count = t.pe + sl->tab_cap;
  t.kw = reinterpret_cast<uint32_t*>(t.count + 8);
  return t;
}

inline int grid_for(uint64_t items, uint32_t per_block, uint32_t cap) {
  uint64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// The iov staging buffer of at least `bytes` (ctx->mu held).
inline int ensure_iov(scratch_slot* sl, uint64_t bytes, bool capture) {
  if (bytes <= sl->iov_cap && sl->iov_mem) return XYWS_OK;
  if (capture) return XYWS_ERR_CAPACITY;
  uint64_t cap = bytes < (1u << 20) ? (1u << 20) : bytes;
  void* mem = nullptr;
  if (hipMalloc(&mem, cap) != hipSuccess) return XYWS_ERR_NOMEM;
  if (sl->iov_mem) {
    (void)hipDeviceSynchronize();
    (void)hipFree(sl->iov_mem);
  }
  sl->iov_mem = mem;
  sl->iov_cap = cap;
  return XYWS_OK;
}

// The slot of `stream` (ctx->mu held).
inline int acquire_slot(xyws_ctx* ctx, hipStream_t stream, bool capture, scratch_slot** out) {
  scratch_slot* pick = nullptr;
  for (auto& sl : ctx->slot)
    if (sl.bound && sl.stream == stream) { pick = &sl; break; }
  if (!pick) {
    bool any_free = false;
    for (auto& sl : ctx->slot) any_free = any_free || !sl.bound;
    if (!any_free) {
      // every slot bound to another stream: wait until all of them are idle
      if (capture) return XYWS_ERR_CAPACITY;
      if (hipDeviceSynchronize() != hipSuccess) return XYWS_ERR_HIP;
      for (auto& sl : ctx->slot) sl.bound = false;
    }
    for (auto& sl : ctx->slot)
      if (!sl.bound) { pick = &sl; break; }
  }
  if (!pick->bound && ctx->reserve_iov && !capture) {
    // (xyws_ctx_reserve_iov's staging buffer, as the per-frame tables below)
    if (const int rc = ensure_iov(pick, ctx->reserve_iov, false)) return rc;
  }
  if (!pick->bound && ctx->reserve_frames && !capture) {
    // xyws_ctx_reserve's per-frame tables go to the slots streams bind (not
    // to all XYWS_SLOTS up front: tens of GB for 2^26 frames)
    if (const int rc = ensure_table(pick, ctx->reserve_frames, false)) return rc;
    if (const int rc = stream_scratch_reserve_frames(&pick->ss, ctx->reserve_bytes, ctx->reserve_frames)) return rc;
  }
  pick->bound = true;
  pick->stream = stream;
  *out = pick;
  return XYWS_OK;
}


// Frame-list kernels' scratch of at least `bytes` (ctx->mu held).
inline int ensure_aux(scratch_slot* sl, uint64_t bytes, bool capture) {
  if (bytes <= sl->aux_cap && sl->aux_mem) return XYWS_OK;
  if (capture) return XYWS_ERR_CAPACITY;
  uint64_t cap = bytes < 65536 ? 65536 : bytes;
  void* mem = nullptr;
  if (hipMalloc(&mem, cap) != hipSuccess) return XYWS_ERR_NOMEM;
  if (sl->aux_mem) {
    (void)hipDeviceSynchronize();
    (void)hipFree(sl->aux_mem);
  }
  sl->aux_mem = mem;
  sl->aux_cap = cap;
  return XYWS_OK;
}

}  // namespace xyws_internal
