// xyws_stream.hip — fused single-pass stream decoder (placeholder: not yet built).
#include "xyws_stream.h"

void stream_scratch_init(stream_scratch* s) { s->mem = nullptr; s->bytes = 0; s->max_tiles = 0; }
void stream_scratch_free(stream_scratch* s) { if (s->mem) (void)hipFree(s->mem); s->mem = nullptr; }
int stream_scratch_reserve(stream_scratch*, uint64_t) { return XYWS_OK; }
uint32_t stream_scratch_error(stream_scratch*) { return 0; }
int stream_decode_fused(stream_scratch*, uint8_t*, uint64_t, uint64_t, const xyws_carry*, xyws_carry*,
                        xyws_frame*, uint64_t, uint64_t*, uint32_t, hipStream_t) {
  return XYWS_ERR_INVALID;
}
