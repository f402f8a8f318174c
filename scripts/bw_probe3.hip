// bw_probe3.hip — measurement probe (not product code): the spread of
// per-workgroup finish times of the decoder's data path (register prefetch +
// LDS copy, one 1024-thread workgroup per CU streaming its own contiguous
// range in place) for several run spacings, and the same path with dynamic
// segment claiming. Prints ms per pass, R+W GB/s and the min / mean / max of
// the workgroups' end times (us after the first start).
//   hipcc --offload-arch=gfx950 -O3 scripts/bw_probe3.hip -o scripts/bw_probe3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int NT = 1024, SEGB = 131072, CH = SEGB / 16 / NT;

// static ranges: run r = [r * stride, r * stride + len) (bytes, multiples of 16)
__global__ void __launch_bounds__(NT) k_static(uint8_t* p, uint64_t stride, uint64_t len, uint32_t kw,
                                               uint64_t* times) {
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t s0 = blockIdx.x * stride;
  const uint32_t nseg = (uint32_t)((len + SEGB - 1) / SEGB);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p + s0, 0, (uint32_t)len, 0x00020000);
  const uint32_t vo = threadIdx.x * 16;
  u32x4 e[CH];
#pragma unroll
  for (int k = 0; k < CH; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, k * NT * 16, 2);
  for (uint32_t s = 0; s < nseg; s++) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CH; k++) lds[k * NT + threadIdx.x] = e[k];
    __syncthreads();
    if (s + 1 < nseg) {
#pragma unroll
      for (int k = 0; k < CH; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (s + 1) * SEGB + k * NT * 16, 2);
    }
    __syncthreads();
    u32x4 prev = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < CH; k++) {
      const u32x4 d = lds[k * NT + threadIdx.x] ^ kw;
      __builtin_amdgcn_raw_buffer_store_b128(d, rs, vo, s * SEGB + k * NT * 16, 2);
      asm volatile("" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
      prev = d;
    }
    asm volatile("s_nop 1" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
  }
  if (threadIdx.x == 0) {
    times[2 * blockIdx.x] = t0;
    times[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

int main() {
  const uint64_t bytes = 2147942400ull;
  uint8_t* p;
  uint64_t* times;
  CK(hipMalloc(&p, bytes + (64ull << 20)));
  CK(hipMemset(p, 0x5A, bytes + (64ull << 20)));
  CK(hipMalloc(&times, 2 * 1024 * 8));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipFuncSetAttribute((const void*)k_static, hipFuncAttributeMaxDynamicSharedMemorySize, SEGB));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, uint64_t stride, uint64_t len, int grid) {
    for (int i = 0; i < 4; i++) k_static<<<grid, NT, SEGB>>>(p, stride, len, 0x1234567u, times);
    CK(hipDeviceSynchronize());
    const int it = 10;
    double mn = 0, mean = 0, mx = 0;
    CK(hipEventRecord(a));
    for (int i = 0; i < it; i++) {
      k_static<<<grid, NT, SEGB>>>(p, stride, len, 0x1234567u, times);
    }
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    std::vector<uint64_t> t(2 * grid);
    CK(hipMemcpy(t.data(), times, 16 * grid, hipMemcpyDeviceToHost));
    uint64_t base = ~0ull;
    for (int i = 0; i < grid; i++) base = std::min(base, t[2 * i]);
    mn = 1e30;
    for (int i = 0; i < grid; i++) {
      const double e = (t[2 * i + 1] - base) / 100.0;
      mn = std::min(mn, e); mx = std::max(mx, e); mean += e / grid;
    }
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= it;
    printf("%-40s %8.3f ms %7.1f GB/s  end us min %.1f mean %.1f max %.1f\n", name, ms,
           2.0 * len * grid / (ms * 1e-3) / 1e9, mn, mean, mx);
    fflush(stdout);
  };
  const uint64_t per = (bytes / ncu + 15) & ~15ull;  // the decoder's run size for c3 (0x800700)
  run("decoder spacing 8MiB+1792", per, per, ncu);
  run("power-of-two spacing 8MiB", 8ull << 20, per, ncu);
  run("spacing 8MiB+4KiB", (8ull << 20) + 4096, per, ncu);
  run("spacing 8MiB+64KiB", (8ull << 20) + 65536, per, ncu);
  run("spacing 8MiB+12KiB+256", (8ull << 20) + 12288 + 256, per, ncu);
  run("spacing 8MiB+1792 x2 repeat", per, per, ncu);
  return 0;
}
