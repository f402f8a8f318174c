// xyws_stream.h — fused single-pass stream decoder (xyws_stream.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "xyws.h"

// Scratch owned by a context: per-tile status words + records for the
// decoupled look-back, the tile ticket counter and a device error word.
struct stream_scratch {
  void* mem;            // device allocation
  uint64_t bytes;
  uint64_t max_tiles;   // tiles the allocation covers
};

void stream_scratch_init(stream_scratch* s);
void stream_scratch_free(stream_scratch* s);
int stream_scratch_reserve(stream_scratch* s, uint64_t max_batch_bytes);
uint32_t stream_scratch_error(stream_scratch* s);
int stream_scratch_stats(stream_scratch* s, uint64_t out[32]);

// Internal decode option: count resolution events (xyws_debug_stats).
#define XYWS_OPT_STATS 0x100u  // synchronous read of the error word
int stream_decode_fused(stream_scratch* s, uint8_t* base, uint64_t lo, uint64_t hi,
                        const xyws_carry* cin, xyws_carry* cout, xyws_frame* frames, uint64_t cap,
                        uint64_t* nframes, uint32_t opts, hipStream_t stream);
