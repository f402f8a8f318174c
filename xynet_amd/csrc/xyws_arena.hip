// xyws_arena.hip — the io_uring side of the boundary: per-connection receive
// arenas in pinned host memory, decoded on the device, completion written to an
// eventfd (include/xyws.h, "recv arenas").
//
// Reference anchors (paths relative to the xynet tree): a connection's recv
// loop fills a buffer_sequence and resumes its coroutine on completion
// (include/xynet/socket/impl/recv_all.h:86-121); foreign threads wake the ring
// through an eventfd the ring keeps a poll_add on
// (include/xynet/io_service.h:362-381). Here the "foreign thread" is the HIP
// runtime's callback thread: after H2D -> decode -> D2H on the arena's stream,
// a hipLaunchHostFunc callback marks the submission complete and writes the
// eventfd, so the ring polls the fd like its remote queue and never blocks on
// the GPU. The carry lives on the device and is chained in stream order, so a
// frame cut by a recv boundary decodes exactly as if the bytes were contiguous.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <errno.h>
#include <unistd.h>

#include <atomic>
#include <new>

#include "xyws.h"
#include "xyws_ctx.h"

using namespace xyws_internal;

struct xyws_notifier {
  int fd;
  std::atomic<uint64_t> completed;  // highest completed seq + 1 (in-order completion)
};

namespace {

void notify(xyws_notifier* n, uint64_t seq) {
  uint64_t want = seq + 1, cur = n->completed.load(std::memory_order_relaxed);
  while (cur < want && !n->completed.compare_exchange_weak(cur, want, std::memory_order_release)) {
  }
  if (n->fd >= 0) {
    const uint64_t one = 1;
    ssize_t r;
    do {
      r = write(n->fd, &one, sizeof one);
    } while (r < 0 && errno == EINTR);
  }
}

}  // namespace

struct arena_slot {
  uint64_t seq, offset, len;
  bool consumed;            // its results were returned by poll / wait: the slot can be reused
  xyws_frame* host_frames;  // pinned
  uint8_t* host_meta;       // pinned: count (8 B) | carry (64 B)
  xyws_frame* dev_frames;
  uint64_t* dev_count;
  hipEvent_t done;          // recorded after the submission's last copy: wait() syncs on it alone
};

struct arena_cb {
  xyws_notifier* n;
  uint64_t seq;
};

struct xyws_arena {
  xyws_ctx* ctx;
  hipStream_t stream;
  uint8_t* host;
  bool owned, registered;
  uint64_t bytes, max_frames;
  uint8_t* dev;          // device mirror of the receive area
  xyws_carry* dev_carry;
  xyws_notifier note;
  uint64_t next_seq;
  bool failed;  // a submission failed after work was enqueued: every later submit fails
  arena_slot slot[XYWS_ARENA_SLOTS];
  arena_cb cb[XYWS_ARENA_SLOTS];
};

namespace {

void on_complete(void* p) {
  arena_cb* c = static_cast<arena_cb*>(p);
  notify(c->n, c->seq);
}

void arena_free(xyws_arena* a) {
  if (a->stream) (void)hipStreamSynchronize(a->stream);
  for (auto& s : a->slot) {
    if (s.host_frames) (void)hipHostFree(s.host_frames);
    if (s.host_meta) (void)hipHostFree(s.host_meta);
    if (s.dev_frames) (void)hipFree(s.dev_frames);
    if (s.dev_count) (void)hipFree(s.dev_count);
    if (s.done) (void)hipEventDestroy(s.done);
  }
  if (a->dev) (void)hipFree(a->dev);
  if (a->dev_carry) (void)hipFree(a->dev_carry);
  if (a->host && a->owned) (void)hipHostFree(a->host);
  if (a->host && a->registered) (void)hipHostUnregister(a->host);
  // (the stream is the context's: arena_stream)
  delete a;
}

int fill_result(xyws_arena* a, const arena_slot& s, xyws_arena_result* out) {
  if (!out) return XYWS_OK;
  out->seq = s.seq;
  out->offset = s.offset;
  out->len = s.len;
  memcpy(&out->nframes, s.host_meta, 8);
  out->frames = s.host_frames;
  memcpy(&out->carry, s.host_meta + 8, sizeof(xyws_carry));
  (void)a;
  return XYWS_OK;
}

}  // namespace

extern "C" {

int xyws_notifier_create(int eventfd, xyws_notifier** out) {
  if (!out) return XYWS_ERR_INVALID;
  xyws_notifier* n = new (std::nothrow) xyws_notifier();
  if (!n) return XYWS_ERR_NOMEM;
  n->fd = eventfd;
  n->completed.store(0);
  *out = n;
  return XYWS_OK;
}

int xyws_notifier_destroy(xyws_notifier* n) {
  if (!n) return XYWS_ERR_INVALID;
  delete n;
  return XYWS_OK;
}

int xyws_notifier_signal(xyws_notifier* n, uint64_t seq) {
  if (!n) return XYWS_ERR_INVALID;
  notify(n, seq);
  return XYWS_OK;
}

uint64_t xyws_notifier_completed(const xyws_notifier* n) {
  return n ? n->completed.load(std::memory_order_acquire) : 0;
}

int xyws_arena_create(xyws_ctx* ctx, void* host, uint64_t bytes, uint64_t max_frames, int eventfd,
                      xyws_arena** out) {
  if (!ctx || !out || !bytes) return XYWS_ERR_INVALID;
  *out = nullptr;
  device_guard g(ctx->device);
  if (!g.ok) return XYWS_ERR_HIP;
  xyws_arena* a = new (std::nothrow) xyws_arena();
  if (!a) return XYWS_ERR_NOMEM;
  a->ctx = ctx;
  a->bytes = bytes;
  a->max_frames = max_frames ? max_frames : 1;
  a->note.fd = eventfd;
  a->note.completed.store(0);
  a->next_seq = 0;
  a->failed = false;
  int rc = XYWS_OK;
  {
    // one of the context's arena streams, round robin (created on first use)
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipStream_t& st = ctx->arena_stream[ctx->arena_rr++ % XYWS_ARENA_STREAMS];
    if (!st && hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
      st = nullptr;
      rc = XYWS_ERR_HIP;
    }
    a->stream = st;
  }
  if (!rc) {
    if (host) {
      if (hipHostRegister(host, bytes, hipHostRegisterDefault) != hipSuccess) rc = XYWS_ERR_HIP;
      else { a->host = static_cast<uint8_t*>(host); a->registered = true; }
    } else {
      void* h = nullptr;
      if (hipHostMalloc(&h, bytes, hipHostMallocDefault) != hipSuccess) rc = XYWS_ERR_NOMEM;
      else { a->host = static_cast<uint8_t*>(h); a->owned = true; }
    }
  }
  if (!rc && hipMalloc(&a->dev, bytes + 64) != hipSuccess) { a->dev = nullptr; rc = XYWS_ERR_NOMEM; }
  if (!rc && hipMalloc(&a->dev_carry, sizeof(xyws_carry)) != hipSuccess) { a->dev_carry = nullptr; rc = XYWS_ERR_NOMEM; }
  if (!rc && zero_now(a->dev_carry, sizeof(xyws_carry)) != hipSuccess) rc = XYWS_ERR_HIP;
  for (auto& s : a->slot) {
    if (rc) break;
    s.seq = ~0ull;
    s.consumed = true;
    if (hipHostMalloc(&s.host_frames, a->max_frames * sizeof(xyws_frame), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&s.host_meta, 8 + sizeof(xyws_carry), hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&s.dev_frames, a->max_frames * sizeof(xyws_frame)) != hipSuccess ||
        hipMalloc(&s.dev_count, 8) != hipSuccess)
      rc = XYWS_ERR_NOMEM;
    else if (hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess)
      rc = XYWS_ERR_HIP;
  }
  if (rc) {
    arena_free(a);
    return rc;
  }
  *out = a;
  return XYWS_OK;
}

int xyws_arena_destroy(xyws_arena* a) {
  if (!a) return XYWS_ERR_INVALID;
  device_guard g(a->ctx->device);
  arena_free(a);
  return XYWS_OK;
}

void* xyws_arena_host(xyws_arena* a) { return a ? a->host : nullptr; }

int xyws_arena_submit(xyws_arena* a, uint64_t offset, uint64_t len, uint32_t opts, uint64_t* seq) {
  if (!a || offset > a->bytes || len > a->bytes - offset) return XYWS_ERR_INVALID;
  // a slot is free once the results of the submission that used it were
  // taken (poll / wait): results stay valid until then
  if (a->failed) return XYWS_ERR_HIP;
  const uint64_t s_no = a->next_seq;
  arena_slot& s = a->slot[s_no % XYWS_ARENA_SLOTS];
  if (!s.consumed) return XYWS_ERR_AGAIN;
  device_guard g(a->ctx->device);
  if (!g.ok) return XYWS_ERR_HIP;
  hipStream_t st = a->stream;
  uint8_t* dv = a->dev + offset;
  // nothing enqueued yet: a failure here leaves the arena as it was
  if (len && hipMemcpyAsync(dv, a->host + offset, len, hipMemcpyHostToDevice, st) != hipSuccess) return XYWS_ERR_HIP;
  // from here on the device carry may move: a failure leaves the arena failed
  // (no result would report the bytes it passed; the caller destroys it)
  int rc = xyws_decode_stream(a->ctx, dv, len, a->dev_carry, a->dev_carry, s.dev_frames, a->max_frames,
                              s.dev_count, opts & ~XYWS_OPT_SERIAL_SCAN, st);
  if (!rc && len && !(opts & XYWS_OPT_PARSE_ONLY) &&
      hipMemcpyAsync(a->host + offset, dv, len, hipMemcpyDeviceToHost, st) != hipSuccess)
    rc = XYWS_ERR_HIP;
  if (!rc && (hipMemcpyAsync(s.host_meta, s.dev_count, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
              hipMemcpyAsync(s.host_meta + 8, a->dev_carry, sizeof(xyws_carry), hipMemcpyDeviceToHost, st) !=
                  hipSuccess ||
              hipMemcpyAsync(s.host_frames, s.dev_frames, a->max_frames * sizeof(xyws_frame),
                             hipMemcpyDeviceToHost, st) != hipSuccess))
    rc = XYWS_ERR_HIP;
  arena_cb& c = a->cb[s_no % XYWS_ARENA_SLOTS];
  c.n = &a->note;
  c.seq = s_no;
  if (!rc && hipLaunchHostFunc(st, on_complete, &c) != hipSuccess) rc = XYWS_ERR_HIP;
  if (!rc && hipEventRecord(s.done, st) != hipSuccess) rc = XYWS_ERR_HIP;
  if (rc) {
    a->failed = true;
    return rc;
  }
  // the slot is taken once every enqueue succeeded
  s.seq = s_no;
  s.consumed = false;
  s.offset = offset;
  s.len = len;
  a->next_seq = s_no + 1;
  if (seq) *seq = s_no;
  return XYWS_OK;
}

int xyws_arena_poll(xyws_arena* a, uint64_t seq, xyws_arena_result* out) {
  if (!a || seq >= a->next_seq) return XYWS_ERR_INVALID;
  if (a->note.completed.load(std::memory_order_acquire) <= seq) return XYWS_ERR_AGAIN;
  arena_slot& s = a->slot[seq % XYWS_ARENA_SLOTS];
  if (s.seq != seq) return XYWS_ERR_INVALID;  // (an older submission whose slot was reused)
  s.consumed = true;
  return fill_result(a, s, out);
}

int xyws_arena_wait(xyws_arena* a, uint64_t seq, xyws_arena_result* out) {
  if (!a || seq >= a->next_seq) return XYWS_ERR_INVALID;
  device_guard g(a->ctx->device);
  // the submission's own event, not the stream: arenas share the context's
  // streams, and another connection's later work on this stream is not waited for
  const arena_slot& s = a->slot[seq % XYWS_ARENA_SLOTS];
  if (s.seq != seq) return XYWS_ERR_INVALID;
  if (hipEventSynchronize(s.done) != hipSuccess) return XYWS_ERR_HIP;
  while (a->note.completed.load(std::memory_order_acquire) <= seq) usleep(10);  // (the callback runs after the sync)
  return xyws_arena_poll(a, seq, out);
}

}  // extern "C"
