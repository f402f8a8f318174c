// bw_probe6.hip — measurement probe (not product code): what dynamic load
// balancing can win on the decoder's data path (one 1024-thread workgroup per
// CU, 128 KiB segments staged in LDS, one-segment register prefetch, in-place
// XOR of a 2 GiB batch), whose static per-CU ranges end over a spread of tens
// of microseconds (bw_probe3).
//
// Variants:
//  * static       each workgroup streams its own range (the decoder today);
//  * steal D      static ranges, and a workgroup that has finished takes the
//                 tail half of the range with most segments left (one 64-bit
//                 word per range: limit << 32 | next, the owner claims each
//                 segment with an atomic add before it prefetches it, a thief
//                 lowers the limit with a CAS), paying D us before it streams
//                 its piece (the stand-in for the piece's entry search); a
//                 piece is itself a range others can steal from;
//  * dynamic      every segment claimed from one global counter (the ideal:
//                 no chain, no entry search).
// Prints ms per pass, R+W GB/s and the spread of workgroup end times.
//   hipcc --offload-arch=gfx950 -O3 scripts/bw_probe6.hip -o scripts/bw_probe6
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <cstring>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int NT = 1024, SEGB = 131072, CH = SEGB / 16 / NT;
constexpr int MAXR = 2048;

struct ctl_t {
  unsigned long long word[MAXR];  // per range: limit << 32 | next (segments, absolute)
  unsigned int nranges;           // ranges handed out (pieces appended)
  unsigned int gnext;             // dynamic: next segment
  unsigned int pad[62];
};

__device__ __forceinline__ unsigned long long ld_sc1(const unsigned long long* p) {
  return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// stream segments [seg, ...) of the batch while claim() hands them out
template <class Claim>
__device__ void stream(uint8_t* p, uint64_t bytes, uint32_t kw, u32x4* lds, Claim claim) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7FFFFFFF, 0x00020000);
  (void)rs;
  const uint32_t vo = threadIdx.x * 16;
  __shared__ uint32_t nxt;
  uint32_t ahead = 0xFFFFFFFFu;  // (thread 0) the claim issued one segment earlier
  if (threadIdx.x == 0) {
    nxt = claim();
    if (nxt != 0xFFFFFFFFu) ahead = claim();
  }
  __syncthreads();
  uint32_t cur = nxt;
  if (cur == 0xFFFFFFFFu) return;
  u32x4 e[CH];
  {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p + (uint64_t)cur * SEGB, 0, SEGB, 0x00020000);
#pragma unroll
    for (int k = 0; k < CH; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(r, vo, k * NT * 16, 2);
  }
  for (;;) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CH; k++) lds[k * NT + threadIdx.x] = e[k];
    if (threadIdx.x == 0) {
      nxt = ahead;
      ahead = ahead != 0xFFFFFFFFu ? claim() : 0xFFFFFFFFu;
    }
    __syncthreads();
    const uint32_t n = nxt;
    if (n != 0xFFFFFFFFu) {
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p + (uint64_t)n * SEGB, 0, SEGB, 0x00020000);
#pragma unroll
      for (int k = 0; k < CH; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(r, vo, k * NT * 16, 2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc(p + (uint64_t)cur * SEGB, 0, SEGB, 0x00020000);
    u32x4 prev = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < CH; k++) {
      const u32x4 d = lds[k * NT + threadIdx.x] ^ kw;
      __builtin_amdgcn_raw_buffer_store_b128(d, w, vo, k * NT * 16, 2);
      asm volatile("" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
      prev = d;
    }
    asm volatile("s_nop 1" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
    if (n == 0xFFFFFFFFu) break;
    cur = n;
  }
}

// mode 0 static, 1 steal, 2 dynamic
__global__ void __launch_bounds__(NT) k_bal(uint8_t* p, uint64_t bytes, uint32_t kw, ctl_t* ctl, int mode,
                                            uint32_t delay_us, uint64_t* times) {
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t nseg = (uint32_t)(bytes / SEGB);
  const uint32_t G = gridDim.x;
  __shared__ uint32_t myr;
  __shared__ uint32_t steals;
  if (threadIdx.x == 0) { myr = blockIdx.x; steals = 0; }
  __syncthreads();
  if (mode == 2) {
    stream(p, bytes, kw, lds, [&]() -> uint32_t {
      const uint32_t s = atomicAdd(&ctl->gnext, 1u);
      return s < nseg ? s : 0xFFFFFFFFu;
    });
  } else {
    for (;;) {
      const uint32_t r = myr;
      stream(p, bytes, kw, lds, [&]() -> uint32_t {
        const unsigned long long o = atomicAdd(&ctl->word[r], 1ull);
        const uint32_t nx = (uint32_t)o, lim = (uint32_t)(o >> 32);
        return nx < lim ? nx : 0xFFFFFFFFu;
      });
      if (mode == 0) break;
      // steal: the range with most segments left; its tail half
      __shared__ uint32_t victim, from;
      if (threadIdx.x == 0) victim = 0xFFFFFFFFu;
      __syncthreads();
      for (int attempt = 0; attempt < 4; attempt++) {
        __shared__ unsigned long long best;
        if (threadIdx.x == 0) best = 0;
        __syncthreads();
        const uint32_t nr = __hip_atomic_load(&ctl->nranges, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t j = threadIdx.x; j < nr; j += NT) {
          const unsigned long long w = ld_sc1(&ctl->word[j]);
          const uint32_t nx = (uint32_t)w, lim = (uint32_t)(w >> 32);
          const uint32_t left = lim > nx ? lim - nx : 0;
          if (left >= 4) atomicMax(&best, ((unsigned long long)left << 32) | j);
        }
        __syncthreads();
        if (!best) break;
        if (threadIdx.x == 0) {
          const uint32_t j = (uint32_t)best;
          unsigned long long w = ld_sc1(&ctl->word[j]);
          for (int t = 0; t < 8; t++) {
            const uint32_t nx = (uint32_t)w, lim = (uint32_t)(w >> 32);
            if (lim <= nx || lim - nx < 4) break;
            const uint32_t cut = nx + 1 + (lim - nx - 1) / 2;  // the owner keeps at least one more
            const unsigned long long nw = ((unsigned long long)cut << 32) | nx;
            const unsigned long long o = atomicCAS(&ctl->word[j], w, nw);
            if (o == w) {
              const uint32_t k = atomicAdd(&ctl->nranges, 1u);
              if (k < MAXR) {
                atomicExch(&ctl->word[k], ((unsigned long long)lim << 32) | cut);
                victim = k;
              }
              break;
            }
            w = o;
          }
        }
        __syncthreads();
        if (victim != 0xFFFFFFFFu) break;
      }
      if (victim == 0xFFFFFFFFu) break;
      if (threadIdx.x == 0) {
        myr = victim;
        steals++;
        const uint64_t tw = __builtin_amdgcn_s_memrealtime() + (uint64_t)delay_us * 100;
        while (__builtin_amdgcn_s_memrealtime() < tw) __builtin_amdgcn_s_sleep(8);
      }
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) {
    times[3 * blockIdx.x] = t0;
    times[3 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    times[3 * blockIdx.x + 2] = steals;
  }
  (void)G;
}

// dynamic + look-back: every segment, after its prefetch is issued, spends C us
// (the stand-in for its entry scan and chase), publishes a 16-byte granule
// tagged with the pass's epoch, and waits for the previous segment's granule
// before its stores (the covering frame it takes from its predecessor)
__global__ void __launch_bounds__(NT) k_sweep(uint8_t* p, uint64_t bytes, uint32_t kw, ctl_t* ctl, uint64_t* gran,
                                              uint64_t epoch, uint32_t c_us, uint64_t* times) {
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t nseg = (uint32_t)(bytes / SEGB);
  const uint32_t vo = threadIdx.x * 16;
  __shared__ uint32_t nxt;
  __shared__ uint64_t waited;
  uint32_t ahead = 0xFFFFFFFFu;
  if (threadIdx.x == 0) {
    waited = 0;
    uint32_t s = atomicAdd(&ctl->gnext, 1u);
    nxt = s < nseg ? s : 0xFFFFFFFFu;
    if (nxt != 0xFFFFFFFFu) { s = atomicAdd(&ctl->gnext, 1u); ahead = s < nseg ? s : 0xFFFFFFFFu; }
  }
  __syncthreads();
  uint32_t cur = nxt;
  if (cur != 0xFFFFFFFFu) {
    u32x4 e[CH];
    {
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p + (uint64_t)cur * SEGB, 0, SEGB, 0x00020000);
#pragma unroll
      for (int k = 0; k < CH; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(r, vo, k * NT * 16, 2);
    }
    for (;;) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < CH; k++) lds[k * NT + threadIdx.x] = e[k];
      if (threadIdx.x == 0) {
        nxt = ahead;
        if (ahead != 0xFFFFFFFFu) { const uint32_t s = atomicAdd(&ctl->gnext, 1u); ahead = s < nseg ? s : 0xFFFFFFFFu; }
      }
      __syncthreads();
      const uint32_t n = nxt;
      if (n != 0xFFFFFFFFu) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p + (uint64_t)n * SEGB, 0, SEGB, 0x00020000);
#pragma unroll
        for (int k = 0; k < CH; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(r, vo, k * NT * 16, 2);
      }
      if (threadIdx.x == 0) {
        const uint64_t tw = __builtin_amdgcn_s_memrealtime() + (uint64_t)c_us * 100;
        while (__builtin_amdgcn_s_memrealtime() < tw) __builtin_amdgcn_s_sleep(1);
        const u32x4 v = {(uint32_t)epoch, (uint32_t)(epoch >> 32), cur, 0u};
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(gran + 2 * (uint64_t)cur), "v"(v) : "memory");
        if (cur > 0) {
          const uint64_t tq = __builtin_amdgcn_s_memrealtime();
          for (uint32_t it = 0; it < (1u << 22); it++) {
            u32x4 g;
            asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(g)
                         : "v"(gran + 2 * (uint64_t)(cur - 1)) : "memory");
            if (((uint64_t)g.x | ((uint64_t)g.y << 32)) == epoch) break;
            __builtin_amdgcn_s_sleep(1);
          }
          waited += __builtin_amdgcn_s_memrealtime() - tq;
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc(p + (uint64_t)cur * SEGB, 0, SEGB, 0x00020000);
      u32x4 prev = {0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < CH; k++) {
        const u32x4 d = lds[k * NT + threadIdx.x] ^ kw;
        __builtin_amdgcn_raw_buffer_store_b128(d, w, vo, k * NT * 16, 2);
        asm volatile("" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
        prev = d;
      }
      asm volatile("s_nop 1" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
      if (n == 0xFFFFFFFFu) break;
      cur = n;
    }
  }
  if (threadIdx.x == 0) {
    times[3 * blockIdx.x] = t0;
    times[3 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    times[3 * blockIdx.x + 2] = waited / 100;  // us spent waiting for predecessors
  }
}

int main() {
  const uint64_t bytes = 2147942400ull / SEGB * SEGB;
  const uint32_t nseg = (uint32_t)(bytes / SEGB);
  uint8_t* p;
  uint64_t* times;
  ctl_t* ctl;
  CK(hipMalloc(&p, bytes));
  CK(hipMemset(p, 0x5A, bytes));
  CK(hipMalloc(&times, 3 * 1024 * 8));
  CK(hipMalloc(&ctl, sizeof(ctl_t)));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipFuncSetAttribute((const void*)k_bal, hipFuncAttributeMaxDynamicSharedMemorySize, SEGB));
  CK(hipFuncSetAttribute((const void*)k_sweep, hipFuncAttributeMaxDynamicSharedMemorySize, SEGB));
  uint64_t* gran;
  CK(hipMalloc(&gran, 16ull * nseg));
  CK(hipMemset(gran, 0, 16ull * nseg));
  uint64_t epoch = 0;
  std::vector<unsigned long long> init(MAXR, 0);
  for (int r = 0; r < ncu; r++) {
    const uint32_t s0 = (uint32_t)((uint64_t)nseg * r / ncu), s1 = (uint32_t)((uint64_t)nseg * (r + 1) / ncu);
    init[r] = ((unsigned long long)s1 << 32) | s0;
  }
  std::vector<uint8_t> hctl(sizeof(ctl_t), 0);
  std::memcpy(hctl.data(), init.data(), 8 * MAXR);
  reinterpret_cast<ctl_t*>(hctl.data())->nranges = ncu;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, int mode, uint32_t delay) {
    const int it = 10;
    float tot = 0;
    double mn = 0, mean = 0, mx = 0, st = 0;
    for (int i = 0; i < it + 3; i++) {
      CK(hipMemcpy(ctl, hctl.data(), sizeof(ctl_t), hipMemcpyHostToDevice));
      CK(hipEventRecord(a));
      if (mode >= 3) k_sweep<<<ncu, NT, SEGB>>>(p, bytes, 0x1234567u, ctl, gran, ++epoch, delay, times);
      else k_bal<<<ncu, NT, SEGB>>>(p, bytes, 0x1234567u, ctl, mode, delay, times);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      if (i < 3) continue;
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      tot += ms;
      std::vector<uint64_t> t(3 * ncu);
      CK(hipMemcpy(t.data(), times, 24 * ncu, hipMemcpyDeviceToHost));
      uint64_t base = ~0ull;
      for (int w = 0; w < ncu; w++) base = std::min(base, t[3 * w]);
      double lmn = 1e30, lmx = 0, lme = 0;
      for (int w = 0; w < ncu; w++) {
        const double e = (t[3 * w + 1] - base) / 100.0;
        lmn = std::min(lmn, e); lmx = std::max(lmx, e); lme += e / ncu;
        st += (double)t[3 * w + 2] / it;
      }
      mn += lmn / it; mx += lmx / it; mean += lme / it;
    }
    const double ms = tot / it;
    printf("%-28s %8.3f ms %7.1f GB/s  end us min %.1f mean %.1f max %.1f  steals(or wait us)/pass %.1f\n", name, ms,
           2.0 * bytes / (ms * 1e-3) / 1e9, mn, mean, mx, st);
    fflush(stdout);
  };
  run("static", 0, 0);
  run("steal D=0us", 1, 0);
  run("dynamic", 2, 0);
  run("sweep C=0us", 3, 0);
  run("sweep C=2us", 3, 2);
  run("sweep C=4us", 3, 4);
  run("sweep C=8us", 3, 8);
  run("sweep C=12us", 3, 12);
  run("dynamic (again)", 2, 0);
  run("static (again)", 0, 0);
  return 0;
}
