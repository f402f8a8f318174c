// bw_probe5.hip — measurement probe (not product code): the decoder's data
// path (one 1024-thread workgroup per CU streaming its own contiguous range in
// place, 128 KiB segments staged in LDS, one-segment register prefetch) with
// the buffer cache-policy bits of the loads and of the stores varied
// (0 = default, 2 = nt, 16 = sc1, 1 = sc0), and with an explicit drain
// (s_waitcnt vmcnt(0)) before the stores or not.
//   hipcc --offload-arch=gfx950 -O3 scripts/bw_probe5.hip -o scripts/bw_probe5
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

template <int LAUX, int SAUX, bool DRAIN>
__global__ void __launch_bounds__(1024) k_pol(uint8_t* p, uint64_t bytes, uint32_t kw) {
  constexpr int NT = 1024, SEGB = 131072, CH = SEGB / 16 / NT;
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  const uint64_t nseg_total = bytes / SEGB;
  const uint64_t per = (nseg_total + gridDim.x - 1) / gridDim.x;
  const uint64_t s0 = blockIdx.x * per;
  uint64_t s1 = s0 + per;
  if (s1 > nseg_total) s1 = nseg_total;
  if (s0 >= s1) return;
  const uint32_t n = (uint32_t)(s1 - s0);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p + s0 * SEGB, 0, n * SEGB, 0x00020000);
  const uint32_t vo = threadIdx.x * 16;
  u32x4 e[CH];
#pragma unroll
  for (int k = 0; k < CH; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, k * NT * 16, LAUX);
  for (uint32_t s = 0; s < n; s++) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CH; k++) lds[k * NT + threadIdx.x] = e[k];
    __syncthreads();
    if (s + 1 < n) {
#pragma unroll
      for (int k = 0; k < CH; k++)
        e[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (s + 1) * SEGB + k * NT * 16, LAUX);
    }
    if (DRAIN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    u32x4 prev = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < CH; k++) {
      const u32x4 v = lds[k * NT + threadIdx.x] ^ kw;
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, vo, s * SEGB + k * NT * 16, SAUX);
      asm volatile("" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
      prev = v;
    }
    asm volatile("s_nop 1" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
  }
}

int main() {
  const uint64_t bytes = 2147942400ull & ~131071ull;
  uint8_t* p;
  CK(hipMalloc(&p, bytes));
  CK(hipMemset(p, 0x5A, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 4; i++) launch();
    CK(hipDeviceSynchronize());
    const int it = 20;
    CK(hipEventRecord(a));
    for (int i = 0; i < it; i++) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= it;
    printf("%-34s %8.3f ms  %7.1f GB/s (R+W)\n", name, ms, 2.0 * bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
#define V(L, S, D)                                                                                   \
  {                                                                                                  \
    auto kf = k_pol<L, S, D>;                                                                        \
    CK(hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));    \
    run("load " #L " store " #S " drain " #D, [&] { kf<<<ncu, 1024, 131072>>>(p, bytes, 0x1234567u); }); \
  }
  for (int rep = 0; rep < 2; rep++) {
    V(2, 2, false)
    V(2, 2, true)
    V(0, 2, true)
    V(2, 0, true)
    V(0, 0, true)
    V(2, 16, true)
    V(16, 2, true)
    V(1, 2, true)
    V(2, 18, true)
  }
  return 0;
}
