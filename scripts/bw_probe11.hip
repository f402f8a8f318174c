// bw_probe11.hip — measurement probe (not product code), round 6.
// xyws_unmask's kernel (k_unmask_range, xyws.hip) on the c3-sized batch,
// in-place XOR, R+W bytes / time, with its geometry and store policy as
// template parameters: U 16-byte chunks per lane per tile (tile = 1024 x U
// chunks), WPC 1024-thread workgroups per CU, the store's cache policy (2 nt,
// 18 sc1|nt: the lattice decoder's). Claimed tiles from one counter, one claim
// ahead, the next tile's loads in flight while the current one is stored.
//   hipcc --offload-arch=gfx950 -O3 scripts/bw_probe11.hip -o scripts/bw_probe11
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

template <uint32_t U, uint32_t WPC, int AST>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4 * WPC)))
k_unmask(uint8_t* __restrict__ base, uint64_t lo, uint64_t hi, uint32_t kw, uint32_t* __restrict__ ctr) {
  constexpr uint32_t NT = 1024, TILE = NT * U;
  const uint64_t c0 = lo >> 4, c1 = (hi + 15) >> 4;
  const uint64_t ntiles = (c1 - c0 + TILE - 1) / TILE;
  const uint32_t t = threadIdx.x;
  __shared__ uint64_t s_tile;
  uint64_t ahead = ~0ull;
  if (t == 0) {
    const uint64_t a = atomicAdd(ctr, 1u);
    s_tile = a < ntiles ? a : ~0ull;
    if (a < ntiles) {
      const uint64_t b = atomicAdd(ctr, 1u);
      ahead = b < ntiles ? b : ~0ull;
    }
  }
  __syncthreads();
  uint64_t cur = s_tile;
  const uint64_t nbytes = (c1 - c0) * 16;
  auto rsrc = [&](uint64_t tile) {
    const uint64_t off = tile * TILE * 16;
    const uint64_t room = nbytes - off;
    return __builtin_amdgcn_make_buffer_rsrc(base + c0 * 16 + off, 0, room < TILE * 16 ? (uint32_t)room : TILE * 16,
                                             0x00020000);
  };
  u32x4 e[U];
  if (cur != ~0ull) {
    const auto r = rsrc(cur);
#pragma unroll
    for (uint32_t u = 0; u < U; u++) e[u] = __builtin_amdgcn_raw_buffer_load_b128(r, t * 16u, u * NT * 16u, 2);
  }
  while (cur != ~0ull) {
    __syncthreads();
    if (t == 0) {
      s_tile = ahead;
      if (ahead != ~0ull) {
        const uint64_t b = atomicAdd(ctr, 1u);
        ahead = b < ntiles ? b : ~0ull;
      }
    }
    __syncthreads();
    const uint64_t nx = s_tile;
    u32x4 d[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) d[u] = e[u] ^ kw;
    if (nx != ~0ull) {
      const auto r = rsrc(nx);
#pragma unroll
      for (uint32_t u = 0; u < U; u++) e[u] = __builtin_amdgcn_raw_buffer_load_b128(r, t * 16u, u * NT * 16u, 2);
    }
    const auto w = rsrc(cur);
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      __builtin_amdgcn_raw_buffer_store_b128(d[u], w, t * 16u, u * NT * 16u, AST);
      asm volatile("" ::"v"(d[u].x), "v"(d[u].y), "v"(d[u].z), "v"(d[u].w));
    }
    asm volatile("s_nop 1" ::: "memory");
    cur = nx;
  }
  __syncthreads();
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const uint32_t n = atomicAdd(ctr + 1, 1u);
    if (n + 1 == gridDim.x) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

int main() {
  const uint64_t bytes = 2147942400ull;
  uint8_t* p;
  CK(hipMalloc(&p, bytes + 4096));
  CK(hipMemset(p, 0x5A, bytes + 4096));
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
    bool ok = true;
    for (int i = 0; i < 4096; i++) ok &= h[i] == 0x5A;
    printf("%-36s %8.4f ms  %7.1f GB/s (R+W) %s\n", name, ms, 2.0 * bytes / (ms * 1e-3) / 1e9, ok ? "" : "WRONG");
    fflush(stdout);
  };
  const uint32_t kw = 0x21963C5Au;
#define V(U, WPC, AST) run("U=" #U " WPC=" #WPC " store aux " #AST, [&] { \
    k_unmask<U, WPC, AST><<<ncu * WPC, 1024>>>(p, 0, bytes, kw, ctr); })
  for (int rep = 0; rep < 2; rep++) {
    V(4, 2, 2);
    V(4, 2, 18);
    V(4, 1, 18);
    V(5, 1, 18);
    V(8, 1, 18);
    V(8, 1, 2);
    V(2, 2, 18);
    V(3, 2, 18);
    V(6, 1, 18);
  }
  return 0;
}
