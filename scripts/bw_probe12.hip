// bw_probe12.hip — measurement probe (not product code), round 6.
// Q: does the lattice decoder's loop skeleton (15 data waves x K rows of 1 KiB
// staged through LDS, three barriers per segment, sc1|nt stores) read more
// per CU with TWO segments of loads in flight (two register sets, the one
// just written to LDS re-issued for the segment after next) than with one?
// Static segment assignment (workgroup b: b, b + grid, ...) in both forms so
// that only the depth differs; c3-sized in-place XOR, R+W bytes / time.
//   hipcc --offload-arch=gfx950 -O3 scripts/bw_probe12.hip -o scripts/bw_probe12
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
constexpr int AUX_LD = 2, AUX_ST = 18;

template <uint32_t K, uint32_t DEPTH>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4)))
k_depth(uint8_t* p, uint64_t bytes, uint32_t kw) {
  constexpr uint32_t NDW = 15, SEGB = NDW * K * 1024;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t nseg = (uint32_t)((bytes + SEGB - 1) / SEGB);
  uint32_t tid = threadIdx.x;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63u;
  const bool data = wave != 0;
  const uint32_t dw = wave - 1, G = gridDim.x;
  auto rsrc = [&](uint32_t s) {
    const uint64_t off = (uint64_t)s * SEGB;
    const uint64_t room = bytes > off ? bytes - off : 0;
    return __builtin_amdgcn_make_buffer_rsrc(p + off, 0, room < SEGB ? (uint32_t)room : SEGB, 0x00020000);
  };
  u32x4 ea[K], eb[K];
  auto load = [&](u32x4* e, uint32_t s) {
    if (!data || s >= nseg) return;
    const auto r = rsrc(s);
#pragma unroll
    for (uint32_t k = 0; k < K; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16u, (dw + NDW * k) * 1024u, AUX_LD);
  };
  auto body = [&](u32x4* e, uint32_t s, uint32_t snext) {
    asm volatile("" : "+v"(tid));
    __syncthreads();  // (A)
    if (data) {
#pragma unroll
      for (uint32_t k = 0; k < K; k++) *reinterpret_cast<u32x4*>(&lds[(dw + NDW * k) * 1024u + lane * 16u]) = e[k];
    }
    __syncthreads();  // (B)
    load(e, snext);   // (this register set again, DEPTH segments ahead)
    __syncthreads();  // (C)
    if (data) {
      const auto w = rsrc(s);
      u32x4 prev = {0, 0, 0, 0};
#pragma unroll
      for (uint32_t k = 0; k < K; k++) {
        const uint32_t a = (dw + NDW * k) * 1024u + lane * 16u;
        const u32x4 d = *reinterpret_cast<const u32x4*>(&lds[a]) ^ kw;
        __builtin_amdgcn_raw_buffer_store_b128(d, w, lane * 16u, (dw + NDW * k) * 1024u, AUX_ST);
        asm volatile("" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
        prev = d;
      }
      asm volatile("s_nop 1" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
    }
  };
  uint32_t s = blockIdx.x;
  if (DEPTH == 1) {
    load(ea, s);
    while (s < nseg) {
      body(ea, s, s + G);
      s += G;
    }
  } else {
    load(ea, s);
    load(eb, s + G);
    while (s < nseg) {
      body(ea, s, s + 2 * G);
      s += G;
      if (s >= nseg) break;
      body(eb, s, s + 2 * G);
      s += G;
    }
  }
}

int main() {
  const uint64_t bytes = 2147942400ull / 1843200 * 1843200;
  uint8_t* p;
  CK(hipMalloc(&p, bytes + 262144));
  CK(hipMemset(p, 0x5A, bytes + 262144));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 6; i++) launch();
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
    CK(hipMemcpy(h, p + bytes / 2, sizeof h, hipMemcpyDeviceToHost));
    bool ok = true;
    for (int i = 0; i < 4096; i++) ok &= h[i] == 0x5A;
    printf("%-28s %8.4f ms  %7.1f GB/s (R+W) %s\n", name, ms, 2.0 * bytes / (ms * 1e-3) / 1e9, ok ? "" : "WRONG");
    fflush(stdout);
  };
  const uint32_t kw = 0x67676767u;
#define V(KK, D)                                                                                               \
  do {                                                                                                         \
    const size_t sh = 15 * KK * 1024 + 64;                                                                     \
    CK(hipFuncSetAttribute((const void*)k_depth<KK, D>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh)); \
    run("K=" #KK " depth=" #D, [&] { k_depth<KK, D><<<ncu, 1024, sh>>>(p, bytes, kw); });                       \
  } while (0)
  for (int rep = 0; rep < 2; rep++) {
    V(5, 1);
    V(5, 2);
    V(4, 1);
    V(4, 2);
    V(3, 2);
    V(6, 2);
    V(8, 1);
  }
  return 0;
}
