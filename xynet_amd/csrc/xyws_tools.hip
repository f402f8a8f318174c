// xyws_tools.hip — device-side synthetic batches and digests.
//
// TEST/BENCH INFRASTRUCTURE (libxyws_tools.so), not the decode path: it builds
// the masked-frame batches of include/xyws_synth.h directly in HBM (so a 2 GiB
// bench batch costs milliseconds, not a host generation + PCIe copy) and
// reduces a batch to the 64-bit digest the golden fixtures record.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xyws_synth.h"

#define TOOLS_OK 0
#define TOOLS_ERR -2

namespace {

// 16-byte output chunk c of a uniform batch.
__global__ void __launch_bounds__(256) k_fill_uniform(uint8_t* __restrict__ buf, uint64_t len,
                                                      uint64_t plen, uint8_t b0, uint64_t seed) {
  const uint64_t H = xyws_synth_hdr_len(plen, 1), S = H + plen;
  const uint64_t dpf = xyws_synth_draws_per_frame(plen);
  const uint64_t nchunks = (len + 15) / 16;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks;
       c += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t out[16];
    uint64_t q = c * 16;
    uint64_t f = q / S, r = q - f * S;
    uint64_t d = f * dpf;
    uint32_t key = xyws_synth_key(seed, d);
    uint64_t cached_k = ~0ull, cached_w = 0;
    for (int t = 0; t < 16; t++) {
      if (r == S) {  // next frame
        f++; r = 0; d = f * dpf; key = xyws_synth_key(seed, d); cached_k = ~0ull;
      }
      uint8_t v;
      if (r < H) {
        v = xyws_synth_hdr_byte(b0, plen, key, (uint32_t)r);
      } else {
        uint64_t j = r - H, k = d + 1 + j / 8;
        if (k != cached_k) { cached_k = k; cached_w = xyws_sm64_at(seed, k); }
        v = (uint8_t)(cached_w >> (8 * (j & 7))) ^ (uint8_t)(key >> (8 * (j & 3)));
      }
      out[t] = v;
      r++;
    }
    if (q + 16 <= len) {
      uint32_t w[4];
      for (int i = 0; i < 4; i++)
        w[i] = (uint32_t)out[4 * i] | ((uint32_t)out[4 * i + 1] << 8) |
               ((uint32_t)out[4 * i + 2] << 16) | ((uint32_t)out[4 * i + 3] << 24);
      typedef uint32_t u4 __attribute__((ext_vector_type(4)));
      u4 v = {w[0], w[1], w[2], w[3]};
      *reinterpret_cast<u4*>(buf + q) = v;
    } else {
      for (int t = 0; q + t < len; t++) buf[q + t] = out[t];
    }
  }
}

// Mixed batch: frame table sorted by offset; chunk -> binary search.
__global__ void __launch_bounds__(256) k_fill_mixed(uint8_t* __restrict__ buf, uint64_t len,
                                                    const xyws_synth_frame* __restrict__ tab,
                                                    uint64_t n, uint64_t seed) {
  const uint64_t nchunks = (len + 15) / 16;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks;
       c += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t q = c * 16;
    uint64_t a = 0, b = n;  // last frame with off <= q
    while (b - a > 1) { uint64_t m = (a + b) >> 1; if (tab[m].off <= q) a = m; else b = m; }
    uint64_t f = a;
    xyws_synth_frame fr = tab[f];
    uint64_t r = q - fr.off;
    uint32_t key = xyws_synth_key(seed, fr.draw);
    uint64_t cached_k = ~0ull, cached_w = 0;
    for (int t = 0; t < 16 && q + t < len; t++) {
      while (r >= (uint64_t)fr.hlen + fr.plen && f + 1 < n) {
        f++; fr = tab[f]; r = 0; key = xyws_synth_key(seed, fr.draw); cached_k = ~0ull;
      }
      uint8_t v;
      if (r < fr.hlen) {
        v = xyws_synth_hdr_byte(fr.b0, fr.plen, key, (uint32_t)r);
      } else {
        uint64_t j = r - fr.hlen, k = fr.draw + 1 + j / 8;
        if (k != cached_k) { cached_k = k; cached_w = xyws_sm64_at(seed, k); }
        v = (uint8_t)(cached_w >> (8 * (j & 7))) ^ (uint8_t)(key >> (8 * (j & 3)));
      }
      buf[q + t] = v;
      r++;
    }
  }
}

__global__ void __launch_bounds__(256) k_digest(const uint8_t* __restrict__ buf, uint64_t len,
                                                unsigned long long* __restrict__ acc) {
  __shared__ uint64_t part[256];
  uint64_t sum = 0;
  const uint64_t nw = (len + 7) / 8;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t w = 0;
    if ((i + 1) * 8 <= len) {
      const uint8_t* p = buf + i * 8;
      if ((reinterpret_cast<uintptr_t>(p) & 7) == 0) {
        w = *reinterpret_cast<const uint64_t*>(p);
      } else {
        for (int b = 0; b < 8; b++) w |= (uint64_t)p[b] << (8 * b);
      }
    } else {
      for (uint64_t b = 0; i * 8 + b < len; b++) w |= (uint64_t)buf[i * 8 + b] << (8 * b);
    }
    sum += xyws_digest_term(i, w);
  }
  part[threadIdx.x] = sum;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < (unsigned)s) part[threadIdx.x] += part[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicAdd(acc, (unsigned long long)part[0]);
}

__global__ void k_digest_finish(unsigned long long* acc, uint64_t len, uint64_t* out) {
  *out = xyws_digest_finish((uint64_t)*acc, len);
}

int grid(uint64_t items) {
  uint64_t g = (items + 255) / 256;
  if (g < 1) g = 1;
  if (g > 16384) g = 16384;
  return (int)g;
}

}  // namespace

extern "C" {

int xyws_tools_fill_uniform(void* dev, uint64_t nframes, uint64_t plen, uint8_t b0, uint64_t seed,
                            void* stream) {
  uint64_t len = nframes * (xyws_synth_hdr_len(plen, 1) + plen);
  if (!len) return TOOLS_OK;
  hipLaunchKernelGGL(k_fill_uniform, dim3(grid((len + 15) / 16)), dim3(256), 0, (hipStream_t)stream,
                     (uint8_t*)dev, len, plen, b0, seed);
  return hipGetLastError() == hipSuccess ? TOOLS_OK : TOOLS_ERR;
}

// Host-side table build for a mixed batch (sequential structure stream).
uint64_t xyws_tools_mixed_table(uint64_t seed, uint64_t target, xyws_synth_frame* out, uint64_t cap,
                                uint64_t* total) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return xyws_synth_mixed_table(seed, target, out, cap, total);
#else
  (void)seed; (void)target; (void)out; (void)cap; (void)total;
  return 0;
#endif
}

int xyws_tools_fill_mixed(void* dev, uint64_t len, const xyws_synth_frame* dev_tab, uint64_t n,
                          uint64_t seed, void* stream) {
  if (!len || !n) return TOOLS_OK;
  hipLaunchKernelGGL(k_fill_mixed, dim3(grid((len + 15) / 16)), dim3(256), 0, (hipStream_t)stream,
                     (uint8_t*)dev, len, dev_tab, n, seed);
  return hipGetLastError() == hipSuccess ? TOOLS_OK : TOOLS_ERR;
}

// Digest of [dev, dev+len) into *dev_out (device u64). dev_scratch: 8 bytes.
int xyws_tools_digest(const void* dev, uint64_t len, uint64_t* dev_out, void* dev_scratch,
                      void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(dev_scratch, 0, 8, s) != hipSuccess) return TOOLS_ERR;
  if (len)
    hipLaunchKernelGGL(k_digest, dim3(grid((len + 7) / 8)), dim3(256), 0, s, (const uint8_t*)dev, len,
                       (unsigned long long*)dev_scratch);
  hipLaunchKernelGGL(k_digest_finish, dim3(1), dim3(1), 0, s, (unsigned long long*)dev_scratch, len,
                     dev_out);
  return hipGetLastError() == hipSuccess ? TOOLS_OK : TOOLS_ERR;
}

}  // extern "C"
