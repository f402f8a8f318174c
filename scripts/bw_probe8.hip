// bw_probe8.hip — measurement probe (not product code), round 4.
// Question: does a barrier-free, per-wave streaming structure reach copy speed
// on the c3-sized 2 GiB in-place XOR (R+W bytes / time)? Each wave claims
// chunks of CT tiles (one atomic per chunk, one chunk ahead), a tile is ROWS
// rows of 1 KiB (one 16-byte load per lane per row), the next tile's loads are
// in flight while the current one is staged in the wave's own LDS region, read
// back, XORed and stored. No workgroup barrier in the loop (each wave's LDS
// region is its own: s_waitcnt lgkmcnt orders it). Variant LDS=false XORs the
// registers directly (the streaming ceiling of the same loop).
//   hipcc --offload-arch=gfx950 -O3 scripts/bw_probe8.hip -o scripts/bw_probe8
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr uint32_t NONE32 = 0xFFFFFFFFu;
constexpr int OOB = 0x40000000;

template <int NT, int ROWS, int CT, bool LDS>
__global__ void __launch_bounds__(NT) k_wave(uint8_t* p, uint64_t bytes, uint32_t kw, uint32_t* ctr) {
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  constexpr uint32_t TILE = ROWS * 1024, CH = TILE * CT;
  const uint32_t nch = (uint32_t)((bytes + CH - 1) / CH);
  uint32_t tid = threadIdx.x;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63u;
  u32x4* my = lds + wave * ROWS * 64;
  uint32_t c = NONE32, ahead = NONE32;
  if (lane == 0) {
    c = atomicAdd(ctr, 1u);
    ahead = atomicAdd(ctr, 1u);
  }
  c = __builtin_amdgcn_readfirstlane(c);
  if (c >= nch) c = NONE32;
  u32x4 e[ROWS];
  auto issue = [&](uint64_t off) {
    const uint64_t room = bytes > off ? bytes - off : 0;
    const auto r = __builtin_amdgcn_make_buffer_rsrc(p + off, 0, room < TILE ? (uint32_t)room : TILE, 0x00020000);
#pragma unroll
    for (int k = 0; k < ROWS; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16u, k * 1024u, 2);
  };
  auto dummy = [&](uint64_t off) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(p + off, 0, 0, 0x00020000);
#pragma unroll
    for (int k = 0; k < ROWS; k++) __builtin_amdgcn_raw_buffer_store_b128(u32x4{0, 0, 0, 0}, r, OOB, k * 1024u, 2);
  };
  if (c != NONE32) {
    issue((uint64_t)c * CH);
    dummy((uint64_t)c * CH);
  }
  uint32_t j = 0;
  while (c != NONE32) {
    asm volatile("" : "+v"(tid));
    const uint64_t cur = (uint64_t)c * CH + (uint64_t)j * TILE;
    // the next tile: the chunk's next, or the chunk claimed ahead
    uint32_t nc = c, nj = j + 1;
    if (nj == CT) {
      nj = 0;
      nc = __builtin_amdgcn_readfirstlane(ahead);
      if (nc >= nch) nc = NONE32;
      if (nc != NONE32 && lane == 0) ahead = atomicAdd(ctr, 1u);
    }
    u32x4 v[ROWS];
    if constexpr (LDS) {
#pragma unroll
      for (int k = 0; k < ROWS; k++) my[k * 64 + lane] = e[k];
    } else {
#pragma unroll
      for (int k = 0; k < ROWS; k++) v[k] = e[k];
    }
    if (nc != NONE32) issue((uint64_t)nc * CH + (uint64_t)nj * TILE);
    const uint64_t room = bytes > cur ? bytes - cur : 0;
    const auto w = __builtin_amdgcn_make_buffer_rsrc(p + cur, 0, room < TILE ? (uint32_t)room : TILE, 0x00020000);
    u32x4 prev = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < ROWS; k++) {
      // (other lanes' chunks: a rotation inside the row, as a decoder's
      // header reads cross lanes)
      const u32x4 d = (LDS ? my[k * 64 + ((lane + 1) & 63)] : v[k]) ^ kw;
      __builtin_amdgcn_raw_buffer_store_b128(d, w, (LDS ? ((lane + 1) & 63) : lane) * 16u, k * 1024u, 2);
      asm volatile("" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
      prev = d;
    }
    asm volatile("s_nop 1" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
    c = nc;
    j = nj;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t d = atomicAdd(ctr + 1, 1u);
    if (d + 1 == gridDim.x) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

int main() {
  const uint64_t bytes = 2147942400ull / 65536 * 65536;
  uint8_t* p;
  CK(hipMalloc(&p, bytes));
  CK(hipMemset(p, 0x5A, bytes));
  uint32_t* ctr;
  CK(hipMalloc(&ctr, 64));
  CK(hipMemset(ctr, 0, 64));
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
    const bool ok = h[0] == 0x5A;  // (26 passes: even)
    printf("%-48s %8.4f ms  %7.1f GB/s (R+W) %s\n", name, ms, 2.0 * bytes / (ms * 1e-3) / 1e9, ok ? "" : "WRONG");
    fflush(stdout);
  };
  const uint32_t kw = 0x67676767u;
#define WAVE(NT, ROWS, CT, LDS, WPC)                                                                         \
  do {                                                                                                       \
    const size_t sh = LDS ? (size_t)(NT / 64) * ROWS * 1024 : 16;                                            \
    CK(hipFuncSetAttribute((const void*)k_wave<NT, ROWS, CT, LDS>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                           (int)sh));                                                                        \
    run("wave " #NT "t rows" #ROWS " ct" #CT " lds" #LDS " x" #WPC "/CU",                                    \
        [&] { k_wave<NT, ROWS, CT, LDS><<<ncu * (WPC), NT, sh>>>(p, bytes, kw, ctr); });                    \
  } while (0)
  WAVE(256, 8, 8, true, 4);
  WAVE(256, 8, 8, false, 4);
  WAVE(256, 8, 8, false, 8);
  WAVE(256, 16, 4, true, 2);
  WAVE(256, 16, 4, false, 4);
  WAVE(512, 8, 8, true, 2);
  WAVE(1024, 8, 8, true, 1);
  WAVE(256, 4, 16, true, 4);
  WAVE(256, 4, 16, true, 8);
  WAVE(256, 8, 8, true, 4);
  return 0;
}
