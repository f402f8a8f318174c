// bw_probe4.hip — measurement probe (not product code): the decoder's data
// path (one 1024-thread workgroup per CU streaming its own contiguous range in
// place, the current segment staged in LDS for the header chase) with the
// register prefetch DEPTH segments deep instead of one, and a stand-in for the
// per-segment chase (a dependent lane-0 LDS walk of WALK steps) between the
// prefetch issue and the stores.
//   hipcc --offload-arch=gfx950 -O3 scripts/bw_probe4.hip -o scripts/bw_probe4
// Prints ms per 2 GiB in-place pass and R+W GB/s per variant.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

// a 16-byte nontemporal buffer load the compiler does not track (no implicit
// s_waitcnt): the consumer waits with wait_slot
__device__ __forceinline__ u32x4 ld(__amdgpu_buffer_rsrc_t rs, uint32_t vo, uint32_t so) {
  u32x4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen nt" : "=v"(v) : "v"(vo), "s"(rs), "s"(so) : "memory");
  return v;
}
template <int N, int CH>
__device__ __forceinline__ void wait_slot(u32x4 (&e)[CH]) {
  if constexpr (CH == 8)
    asm volatile("s_waitcnt vmcnt(%8)" : "+v"(e[0]), "+v"(e[1]), "+v"(e[2]), "+v"(e[3]), "+v"(e[4]), "+v"(e[5]),
                 "+v"(e[6]), "+v"(e[7]) : "n"(N) : "memory");
  else if constexpr (CH == 4)
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(e[0]), "+v"(e[1]), "+v"(e[2]), "+v"(e[3]) : "n"(N) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(e[0]), "+v"(e[1]) : "n"(N) : "memory");
}

template <int NT, int SEGB, int DEPTH, int WALK, int SLEEP>
__global__ void __launch_bounds__(NT) k_deep(uint8_t* p, uint64_t bytes, uint32_t kw) {
  constexpr int CH = SEGB / 16 / NT;
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  const uint64_t nseg_total = bytes / SEGB;
  const uint64_t per = (nseg_total + gridDim.x - 1) / gridDim.x;
  const uint64_t s0 = blockIdx.x * per;
  uint64_t s1 = s0 + per;
  if (s1 > nseg_total) s1 = nseg_total;
  if (s0 >= s1) return;
  const uint32_t n = (uint32_t)(s1 - s0);
  // loads past the range read zero (the rsrc covers exactly the range)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p + s0 * SEGB, 0, n * SEGB, 0x00020000);
  const uint32_t vo = threadIdx.x * 16;
  u32x4 e[DEPTH][CH];
  // each slot's loads followed by CH dropped stores: the sequence of memory
  // ops then looks the same at every fill (vmcnt counts loads and stores)
#pragma unroll
  for (int d = 0; d < DEPTH; d++) {
#pragma unroll
    for (int k = 0; k < CH; k++) e[d][k] = ld(rs, vo, d * SEGB + k * NT * 16);
#pragma unroll
    for (int k = 0; k < CH; k++) __builtin_amdgcn_raw_buffer_store_b128(u32x4{0, 0, 0, 0}, rs, 0x80000000u, 0, 2);
  }
  for (uint32_t s = 0; s < n; s += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      const uint32_t t = s + d;
      __syncthreads();
      // the loads are invisible to the compiler (asm): wait for this slot's
      // CH loads explicitly; issued after them: DEPTH segments of stores and
      // DEPTH-1 slots of loads
      wait_slot<(2 * DEPTH - 1) * CH, CH>(e[d]);
#pragma unroll
      for (int k = 0; k < CH; k++) lds[k * NT + threadIdx.x] = e[d][k];
      __syncthreads();
      // the next load into this slot (past the range: offsets the rsrc clips)
#pragma unroll
      for (int k = 0; k < CH; k++)
        e[d][k] = ld(rs, vo, (t + DEPTH) * SEGB + k * NT * 16);
      if (threadIdx.x == 0 && WALK > 0) {
        uint32_t x = 0;
        const uint32_t* lv = reinterpret_cast<const uint32_t*>(lds);
        for (int h = 0; h < WALK; h++) x = (lv[4 * ((x + 17) & (SEGB / 16 - 1))] + h) & (SEGB / 16 - 1);
        if (x == 0xFFFFFFFF) lds[0].w = 0;
      }
      if (SLEEP > 0) __builtin_amdgcn_s_sleep(SLEEP);
      __syncthreads();
      u32x4 prev = {0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < CH; k++) {
        const u32x4 v = lds[k * NT + threadIdx.x] ^ kw;
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, t < n ? vo : 0x80000000u, t * SEGB + k * NT * 16, 2);
        asm volatile("" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
        prev = v;
      }
      asm volatile("s_nop 1" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
    }
  }
}

int main() {
  const uint64_t bytes = 2147942400ull & ~131071ull;
  uint8_t* p;
  CK(hipMalloc(&p, bytes + (1 << 20)));
  CK(hipMemset(p, 0x5A, bytes + (1 << 20)));
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
    uint8_t h[4096];
    CK(hipMemcpy(h, p + bytes / 3 / 4096 * 4096, sizeof h, hipMemcpyDeviceToHost));
    bool ok = true;
    for (int i = 0; i < 4096; i++) ok &= h[i] == 0x5A;  // 24 passes: an even number of XORs
    printf("%-40s %8.3f ms  %7.1f GB/s (R+W)%s\n", name, ms, 2.0 * bytes / (ms * 1e-3) / 1e9, ok ? "" : "  WRONG");
    fflush(stdout);
  };
#define V(NT, SEGB, D, W, S)                                                                              \
  {                                                                                                       \
    auto kf = k_deep<NT, SEGB, D, W, S>;                                                                  \
    CK(hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, SEGB));           \
    run("deep " #NT "t seg " #SEGB " d" #D " walk" #W " sleep" #S,                                         \
        [&] { kf<<<ncu, NT, SEGB>>>(p, bytes, 0x1234567u); });                                            \
  }
  V(1024, 131072, 1, 3, 0)
  V(1024, 131072, 1, 100, 0)
  V(1024, 131072, 1, 3, 20)
  V(1024, 131072, 1, 3, 60)
  V(1024, 131072, 2, 3, 0)
  V(1024, 131072, 2, 60, 0)
  V(1024, 131072, 2, 100, 0)
  V(1024, 131072, 2, 200, 0)
  V(1024, 65536, 1, 3, 0)
  V(1024, 65536, 2, 3, 0)
  V(1024, 65536, 2, 50, 0)
  V(1024, 65536, 3, 3, 0)
  V(1024, 65536, 3, 50, 0)
  V(1024, 65536, 4, 3, 0)
  V(1024, 32768, 4, 3, 0)
  V(1024, 32768, 4, 30, 0)
  V(1024, 32768, 6, 3, 0)
  V(1024, 131072, 1, 3, 0)
  return 0;
}
