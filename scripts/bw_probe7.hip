// bw_probe7.hip — measurement probe (not product code), round 4.
// Two questions, on the c3-sized 2 GiB in-place XOR (R+W bytes / time):
//  (1) xyws_unmask: the fixed 2048-block grid-stride kernel (r03) against
//      persistent workgroups that claim tiles from one counter, with the next
//      tile's loads in flight while the current one is XORed and stored;
//  (2) a lattice decoder's data path: claimed 128 KiB segments staged in LDS
//      (bw_probe6 "dynamic"), plus what an exact speculative-free decoder has
//      to add: every segment publishes an aggregate status word after its fill,
//      looks back (decoupled look-back, 64 predecessors per round) until an
//      inclusive "prefix verified" status, publishes its own inclusive status
//      and only then stores. Variant "deferred": 64 KiB segments, two LDS
//      buffers, the stores of segment i-1 issued during iteration i (the
//      look-back off the critical path).
//   hipcc --offload-arch=gfx950 -O3 scripts/bw_probe7.hip -o scripts/bw_probe7
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr uint32_t NONE32 = 0xFFFFFFFFu;

__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- (1) unmask
// r03's kernel: grid-stride tiles of U x 256 chunks, 2048 blocks
template <int U>
__global__ void __launch_bounds__(256) k_gs(u32x4* p, uint64_t n, uint32_t kw) {
  const uint64_t tile = (uint64_t)U * 256u, nt = (n + tile - 1) / tile;
  for (uint64_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const uint64_t cb = t * tile + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = cb + u * 256 < n ? __builtin_nontemporal_load(p + cb + u * 256) : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; u++) if (cb + u * 256 < n) __builtin_nontemporal_store(v[u] ^ kw, p + cb + u * 256);
  }
}

// persistent, claimed tiles of NT x U chunks; the next tile's loads are issued
// before the current tile's stores (register double buffer). Counter reset by
// the last workgroup (done count), so launches need no memset.
template <int NT, int U>
__global__ void __launch_bounds__(NT) k_claim(uint8_t* p, uint64_t bytes, uint32_t kw, uint32_t* ctr) {
  constexpr uint32_t TILE = NT * U * 16;
  const uint32_t ntiles = (uint32_t)((bytes + TILE - 1) / TILE);
  __shared__ uint32_t s_t;
  uint32_t ahead = NONE32;
  if (threadIdx.x == 0) {
    const uint32_t t = atomicAdd(ctr, 1u);
    s_t = t < ntiles ? t : NONE32;
    if (t < ntiles) { const uint32_t a = atomicAdd(ctr, 1u); ahead = a < ntiles ? a : NONE32; }
  }
  __syncthreads();
  uint32_t cur = s_t;
  u32x4 e[U];
  auto rsrc = [&](uint32_t t) {
    const uint64_t off = (uint64_t)t * TILE;
    const uint64_t room = bytes - off;
    return __builtin_amdgcn_make_buffer_rsrc(p + off, 0, room < TILE ? (uint32_t)room : TILE, 0x00020000);
  };
  if (cur != NONE32) {
    const auto r = rsrc(cur);
#pragma unroll
    for (int u = 0; u < U; u++) e[u] = __builtin_amdgcn_raw_buffer_load_b128(r, threadIdx.x * 16u, u * NT * 16u, 2);
  }
  while (cur != NONE32) {
    __syncthreads();  // (s_t is rewritten below)
    if (threadIdx.x == 0) {
      s_t = ahead;
      if (ahead != NONE32) { const uint32_t a = atomicAdd(ctr, 1u); ahead = a < ntiles ? a : NONE32; }
    }
    __syncthreads();
    const uint32_t nx = s_t;
    u32x4 d[U];
#pragma unroll
    for (int u = 0; u < U; u++) d[u] = e[u] ^ kw;
    if (nx != NONE32) {
      const auto r = rsrc(nx);
#pragma unroll
      for (int u = 0; u < U; u++) e[u] = __builtin_amdgcn_raw_buffer_load_b128(r, threadIdx.x * 16u, u * NT * 16u, 2);
    }
    const auto w = rsrc(cur);
#pragma unroll
    for (int u = 0; u < U; u++) {
      __builtin_amdgcn_raw_buffer_store_b128(d[u], w, threadIdx.x * 16u, u * NT * 16u, 2);
      asm volatile("" ::"v"(d[u].x), "v"(d[u].y), "v"(d[u].z), "v"(d[u].w));
    }
    asm volatile("s_nop 1" ::: "memory");
    cur = nx;
  }
  // reset: the last workgroup out zeroes the counter and the done count
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t d = atomicAdd(ctr + 1, 1u);
    if (d + 1 == gridDim.x) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------- (2) lattice data path
struct ctl_t {
  uint32_t ctr, done, pad[62];
};

// decoupled look-back over status words (wave 0, all lanes; result in every
// lane): 1 = prefix verified, 0 = a break before s. Status: (E << 2) | st,
// st 1 = aggregate ok, 2 = inclusive ok, 3 = break.
__device__ int lookback(const uint64_t* status, uint64_t s, uint64_t E, uint32_t lane, uint32_t* spins) {
  uint64_t j = s;
  for (uint32_t it = 0; it < (1u << 22); it++) {
    const bool valid = j >= 1 + (uint64_t)lane;
    const uint64_t v = valid ? ld_agent(status + (j - 1 - lane)) : ((E << 2) | 2u);
    const bool pub = (v >> 2) == E;
    const uint32_t st = (uint32_t)v & 3u;
    const uint64_t stop = __ballot(!pub || st >= 2u);
    if (!stop) { j -= 64; continue; }
    const uint32_t f = __builtin_ctzll(stop);
    const uint64_t vf = __shfl(v, (int)f);
    if ((vf >> 2) != E) { __builtin_amdgcn_s_sleep(1); (*spins)++; j = s; continue; }
    return ((uint32_t)vf & 3u) == 2u ? 1 : 0;
  }
  return 0;
}

template <int NT, int SEGB, bool LB>
__global__ void __launch_bounds__(NT) k_seg(uint8_t* p, uint64_t bytes, uint32_t kw, ctl_t* ctl, uint64_t* status,
                                            uint64_t E, uint64_t* spins_out) {
  constexpr int CH = SEGB / 16 / NT;
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  __shared__ uint32_t nxt;
  __shared__ int ok;
  const uint32_t nseg = (uint32_t)(bytes / SEGB);
  const uint32_t vo = threadIdx.x * 16, lane = threadIdx.x & 63;
  uint32_t ahead = NONE32, spins = 0;
  if (threadIdx.x == 0) {
    uint32_t s = atomicAdd(&ctl->ctr, 1u);
    nxt = s < nseg ? s : NONE32;
    if (nxt != NONE32) { s = atomicAdd(&ctl->ctr, 1u); ahead = s < nseg ? s : NONE32; }
  }
  __syncthreads();
  uint32_t cur = nxt;
  if (cur != NONE32) {
    u32x4 e[CH];
    {
      const auto r = __builtin_amdgcn_make_buffer_rsrc(p + (uint64_t)cur * SEGB, 0, SEGB, 0x00020000);
#pragma unroll
      for (int k = 0; k < CH; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(r, vo, k * NT * 16, 2);
    }
    for (;;) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < CH; k++) lds[k * NT + threadIdx.x] = e[k];
      if (threadIdx.x == 0) {
        nxt = ahead;
        if (ahead != NONE32) { const uint32_t s = atomicAdd(&ctl->ctr, 1u); ahead = s < nseg ? s : NONE32; }
        if (LB) st_agent(status + cur, (E << 2) | 1u);  // aggregate: this segment's own lattice checks passed
      }
      __syncthreads();
      const uint32_t n = nxt;
      if (n != NONE32) {
        const auto r = __builtin_amdgcn_make_buffer_rsrc(p + (uint64_t)n * SEGB, 0, SEGB, 0x00020000);
#pragma unroll
        for (int k = 0; k < CH; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(r, vo, k * NT * 16, 2);
      }
      if (LB && threadIdx.x < 64) {
        const int r = lookback(status, cur, E, lane, &spins);
        if (lane == 0) {
          ok = r;
          if (r) st_agent(status + cur, (E << 2) | 2u);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const auto w = __builtin_amdgcn_make_buffer_rsrc(p + (uint64_t)cur * SEGB, 0, (!LB || ok) ? SEGB : 0, 0x00020000);
      u32x4 prev = {0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < CH; k++) {
        const u32x4 d = lds[k * NT + threadIdx.x] ^ kw;
        __builtin_amdgcn_raw_buffer_store_b128(d, w, vo, k * NT * 16, 2);
        asm volatile("" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
        prev = d;
      }
      asm volatile("s_nop 1" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
      if (n == NONE32) break;
      cur = n;
    }
  }
  if (threadIdx.x == 0 && spins) atomicAdd((unsigned long long*)spins_out, (unsigned long long)spins);
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t d = atomicAdd(&ctl->done, 1u);
    if (d + 1 == gridDim.x) {
      __hip_atomic_store(&ctl->ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&ctl->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// deferred stores: two LDS buffers of SEGB; iteration i fills segment i, and
// stores segment i-1 (whose look-back ran during iteration i's load wait)
template <int NT, int SEGB>
__global__ void __launch_bounds__(NT) k_defer(uint8_t* p, uint64_t bytes, uint32_t kw, ctl_t* ctl, uint64_t* status,
                                              uint64_t E, uint64_t* spins_out) {
  constexpr int CH = SEGB / 16 / NT;
  constexpr int Q = SEGB / 16;  // u32x4 per buffer
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  __shared__ uint32_t nxt;
  __shared__ int ok;
  const uint32_t nseg = (uint32_t)(bytes / SEGB);
  const uint32_t vo = threadIdx.x * 16, lane = threadIdx.x & 63;
  uint32_t ahead = NONE32, spins = 0;
  if (threadIdx.x == 0) {
    uint32_t s = atomicAdd(&ctl->ctr, 1u);
    nxt = s < nseg ? s : NONE32;
    if (nxt != NONE32) { s = atomicAdd(&ctl->ctr, 1u); ahead = s < nseg ? s : NONE32; }
  }
  __syncthreads();
  uint32_t cur = nxt, prevseg = NONE32;
  int buf = 0;
  if (cur != NONE32) {
    u32x4 e[CH];
    {
      const auto r = __builtin_amdgcn_make_buffer_rsrc(p + (uint64_t)cur * SEGB, 0, SEGB, 0x00020000);
#pragma unroll
      for (int k = 0; k < CH; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(r, vo, k * NT * 16, 2);
    }
    for (;;) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < CH; k++) lds[buf * Q + k * NT + threadIdx.x] = e[k];
      if (threadIdx.x == 0) {
        nxt = ahead;
        if (ahead != NONE32) { const uint32_t s = atomicAdd(&ctl->ctr, 1u); ahead = s < nseg ? s : NONE32; }
        st_agent(status + cur, (E << 2) | 1u);
      }
      __syncthreads();
      const uint32_t n = nxt;
      if (n != NONE32) {
        const auto r = __builtin_amdgcn_make_buffer_rsrc(p + (uint64_t)n * SEGB, 0, SEGB, 0x00020000);
#pragma unroll
        for (int k = 0; k < CH; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(r, vo, k * NT * 16, 2);
      }
      // store the previous segment (its look-back was done last iteration)
      if (prevseg != NONE32) {
        const auto w = __builtin_amdgcn_make_buffer_rsrc(p + (uint64_t)prevseg * SEGB, 0, ok ? SEGB : 0, 0x00020000);
        u32x4 pv = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < CH; k++) {
          const u32x4 d = lds[(buf ^ 1) * Q + k * NT + threadIdx.x] ^ kw;
          __builtin_amdgcn_raw_buffer_store_b128(d, w, vo, k * NT * 16, 2);
          asm volatile("" ::"v"(pv.x), "v"(pv.y), "v"(pv.z), "v"(pv.w));
          pv = d;
        }
        asm volatile("s_nop 1" ::"v"(pv.x), "v"(pv.y), "v"(pv.z), "v"(pv.w));
      }
      __syncthreads();  // (ok is rewritten below; the other buffer is refilled next iteration)
      if (threadIdx.x < 64) {
        const int r = lookback(status, cur, E, lane, &spins);
        if (lane == 0) {
          ok = r;
          if (r) st_agent(status + cur, (E << 2) | 2u);
        }
      }
      prevseg = cur;
      buf ^= 1;
      if (n == NONE32) break;
      cur = n;
    }
    __syncthreads();
    {  // the last segment
      const auto w = __builtin_amdgcn_make_buffer_rsrc(p + (uint64_t)prevseg * SEGB, 0, ok ? SEGB : 0, 0x00020000);
#pragma unroll
      for (int k = 0; k < CH; k++) {
        const u32x4 d = lds[(buf ^ 1) * Q + k * NT + threadIdx.x] ^ kw;
        __builtin_amdgcn_raw_buffer_store_b128(d, w, vo, k * NT * 16, 2);
        asm volatile("" ::"v"(d.x), "v"(d.y), "v"(d.z), "v"(d.w));
      }
      asm volatile("s_nop 1" ::: "memory");
    }
  }
  if (threadIdx.x == 0 && spins) atomicAdd((unsigned long long*)spins_out, (unsigned long long)spins);
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t d = atomicAdd(&ctl->done, 1u);
    if (d + 1 == gridDim.x) {
      __hip_atomic_store(&ctl->ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&ctl->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

int main() {
  const uint64_t bytes = 2147942400ull / 131072 * 131072;  // c3 batch, whole 128 KiB segments
  uint8_t* p;
  CK(hipMalloc(&p, bytes));
  CK(hipMemset(p, 0x5A, bytes));
  ctl_t* ctl;
  CK(hipMalloc(&ctl, sizeof(ctl_t)));
  CK(hipMemset(ctl, 0, sizeof(ctl_t)));
  uint64_t *status, *spins;
  const uint64_t maxseg = bytes / 32768 + 64;
  CK(hipMalloc(&status, 8 * maxseg));
  CK(hipMemset(status, 0, 8 * maxseg));
  CK(hipMalloc(&spins, 8));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  uint64_t E = 0;
  auto check = [&](const char* name, int passes) {
    // after an even number of in-place passes the buffer is unchanged
    uint8_t h[4096];
    CK(hipDeviceSynchronize());
    for (uint64_t off : {(uint64_t)0, bytes / 3 / 4096 * 4096, bytes - 4096}) {
      CK(hipMemcpy(h, p + off, sizeof h, hipMemcpyDeviceToHost));
      for (int i = 0; i < 4096; i++)
        if (h[i] != ((passes & 1) ? (0x5A ^ 0x67) : 0x5A)) { printf("%s: WRONG BYTES at %llu\n", name, (unsigned long long)off); return; }
    }
  };
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 6; i++) launch();
    CK(hipDeviceSynchronize());
    CK(hipMemset(spins, 0, 8));
    const int it = 20;
    CK(hipEventRecord(a));
    for (int i = 0; i < it; i++) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= it;
    uint64_t sp = 0;
    CK(hipMemcpy(&sp, spins, 8, hipMemcpyDeviceToHost));
    printf("%-44s %8.4f ms  %7.1f GB/s (R+W)  spins/pass %.0f\n", name, ms, 2.0 * bytes / (ms * 1e-3) / 1e9,
           (double)sp / it);
    fflush(stdout);
    check(name, 26);
  };
  const uint32_t kw = 0x67676767u;
  const uint64_t n16 = bytes / 16;
  run("unmask r03: grid-stride 2048x256 U8", [&] { k_gs<8><<<2048, 256>>>((u32x4*)p, n16, kw); });
  run("unmask grid-stride 4096x256 U4", [&] { k_gs<4><<<4096, 256>>>((u32x4*)p, n16, kw); });
#define CLAIM(NT, U, WPC)                                                                        \
  run("unmask claimed " #NT "t U" #U " x" #WPC "/CU (" #NT "*" #U "*16 B tiles)",                \
      [&] { k_claim<NT, U><<<ncu * (WPC), NT>>>(p, bytes, kw, &ctl->ctr); });
  CLAIM(256, 8, 4)
  CLAIM(256, 8, 8)
  CLAIM(256, 16, 4)
  CLAIM(512, 8, 2)
  CLAIM(512, 8, 4)
  CLAIM(1024, 8, 1)
  CLAIM(1024, 8, 2)
  CLAIM(1024, 4, 2)
  CK(hipFuncSetAttribute((const void*)k_seg<1024, 131072, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)k_seg<1024, 131072, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)k_seg<512, 65536, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
  CK(hipFuncSetAttribute((const void*)k_defer<1024, 65536>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)k_defer<512, 32768>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
  run("seg 1024t 128K (probe6 dynamic)", [&] { k_seg<1024, 131072, false><<<ncu, 1024, 131072>>>(p, bytes, kw, ctl, status, ++E, spins); });
  run("seg 1024t 128K + look-back before store", [&] { k_seg<1024, 131072, true><<<ncu, 1024, 131072>>>(p, bytes, kw, ctl, status, ++E, spins); });
  run("seg 512t 64K x2/CU + look-back", [&] { k_seg<512, 65536, true><<<ncu * 2, 512, 65536>>>(p, bytes, kw, ctl, status, ++E, spins); });
  run("defer 1024t 2x64K + look-back", [&] { k_defer<1024, 65536><<<ncu, 1024, 131072>>>(p, bytes, kw, ctl, status, ++E, spins); });
  run("defer 512t 2x32K x2/CU + look-back", [&] { k_defer<512, 32768><<<ncu * 2, 512, 65536>>>(p, bytes, kw, ctl, status, ++E, spins); });
  run("seg 1024t 128K (again)", [&] { k_seg<1024, 131072, false><<<ncu, 1024, 131072>>>(p, bytes, kw, ctl, status, ++E, spins); });
  run("unmask r03 (again)", [&] { k_gs<8><<<2048, 256>>>((u32x4*)p, n16, kw); });
  return 0;
}
