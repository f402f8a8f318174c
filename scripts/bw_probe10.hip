// bw_probe10.hip — measurement probe (not product code), round 6.
// Q1: can the lattice decoder's segment loop (xyws_lattice.h: 15 data waves
//     of K 1 KiB rows, a control wave, claimed segments, three barriers per
//     segment, sc1|nt stores) go faster with its rows staged by LDS-DMA
//     (global_load_lds_dwordx4 straight into an LDS ring of NB segments, no
//     prefetch registers, no ds_write pass) than by register staging (rows
//     loaded one segment ahead into VGPRs, written to LDS at the next fill)?
//     Both on the c3-sized ~2 GiB in-place XOR, R+W bytes / time.
// Q2: what does an empty full-grid launch cost (the run decoder's hand-over
//     check after every lattice call: 4.7 us in the c3 trace), by the
//     resources the kernel declares (dynamic LDS, scratch, workgroup size)?
//   hipcc --offload-arch=gfx950 -O3 scripts/bw_probe10.hip -o scripts/bw_probe10
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr uint32_t NONE32 = 0xFFFFFFFFu;
constexpr uint32_t OOB = 0x40000000u;
constexpr int AUX_LD = 2, AUX_ST = 18;  // nt loads; sc1|nt stores (the decoder's)

struct ctl_t { uint32_t ctr, done; uint64_t pad[7]; };

// ---- register staging: the decoder's loop skeleton (bw_probe9 CW|AC|B3|XL)
template <uint32_t K>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4)))
k_reg(uint8_t* p, uint64_t bytes, uint32_t kw, ctl_t* ctl) {
  constexpr uint32_t NDW = 15, SEGB = NDW * K * 1024;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ uint32_t s_nxt;
  const uint32_t nseg = (uint32_t)((bytes + SEGB - 1) / SEGB);
  uint32_t tid = threadIdx.x;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63u;
  const bool data = wave != 0;
  const uint32_t dw = wave - 1;
  uint32_t ahead = NONE32, cx = 0;
  if (tid == 64) {
    const uint32_t c = atomicAdd(&ctl->ctr, 1u);
    s_nxt = c < nseg ? c : NONE32;
    ahead = atomicAdd(&ctl->ctr, 1u);
  }
  __syncthreads();
  uint32_t cur = s_nxt;
  u32x4 e[K];
  auto rsrc = [&](uint64_t off) {
    const uint64_t room = bytes > off ? bytes - off : 0;
    return __builtin_amdgcn_make_buffer_rsrc(p + off, 0, room < SEGB ? (uint32_t)room : SEGB, 0x00020000);
  };
  auto issue = [&](uint32_t s, bool claim) {
    if (!data) return;
    if (wave == 1) {
      if (lane == 0) {
        if (claim) asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(ahead) : "v"(&ctl->ctr), "v"(1u) : "memory");
        else ahead = NONE32;
      }
      const uint64_t q = (uint64_t)s * SEGB + 4u * (tid & 63u);
      cx = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p + (q + 4 < bytes ? q : 0)));
    }
    const auto r = rsrc((uint64_t)s * SEGB);
#pragma unroll
    for (uint32_t k = 0; k < K; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16u, (dw + NDW * k) * 1024u, AUX_LD);
  };
  if (cur != NONE32 && data) {
    const uint32_t a0 = ahead;
    issue(cur, false);
    ahead = a0;
    const auto r = rsrc((uint64_t)cur * SEGB);
#pragma unroll
    for (uint32_t k = 0; k < K; k++) __builtin_amdgcn_raw_buffer_store_b128(u32x4{0, 0, 0, 0}, r, OOB, k * 1024u, AUX_ST);
  }
  while (cur != NONE32) {
    asm volatile("" : "+v"(tid));
    __syncthreads();  // (A)
    if (data) {
#pragma unroll
      for (uint32_t k = 0; k < K; k++) *reinterpret_cast<u32x4*>(&lds[(dw + NDW * k) * 1024u + lane * 16u]) = e[k];
    }
    if (data && wave == 1) {
      asm volatile("" : "+v"(ahead), "+v"(cx) : "v"(e[K - 1].x));
      if ((tid & 63u) < 9) *reinterpret_cast<uint32_t*>(&lds[SEGB + 4u * (tid & 63u)]) = cx;
      if (lane == 0) s_nxt = ahead < nseg ? ahead : NONE32;
    }
    __syncthreads();  // (B)
    const uint32_t nxt = s_nxt;
    if (nxt != NONE32) issue(nxt, true);
    __syncthreads();  // (C)
    if (data) {
      const auto w = rsrc((uint64_t)cur * SEGB);
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
    cur = nxt;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t d = atomicAdd(&ctl->done, 1u);
    if (d + 1 == gridDim.x) {
      __hip_atomic_store(&ctl->ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&ctl->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---- LDS-DMA staging: a ring of NB segment buffers; iteration i processes
// segment seg[i] from buffer i % NB while the DMAs of seg[i+1 .. i+NB-1] are
// in flight. Per data wave and iteration: K DMA instructions (1 KiB rows) for
// seg[i+NB-1] into the buffer freed by iteration i-1, a counted vmcnt for
// seg[i]'s own rows, barriers, the XOR from LDS and K stores. The control
// wave (0) claims segments (returning atomic, value read an iteration later)
// and issues no row traffic.
__device__ __forceinline__ void dma16(const uint8_t* g, uint32_t lds_row) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds_row) : "memory");
}
template <uint32_t N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <uint32_t K, uint32_t NB>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4)))
k_dma(uint8_t* p, uint64_t bytes, uint32_t kw, ctl_t* ctl) {
  constexpr uint32_t NDW = 15, SEGB = NDW * K * 1024, BUF = SEGB + 64;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ uint32_t s_seg[NB + 1];
  const uint32_t nseg = (uint32_t)((bytes + SEGB - 1) / SEGB);
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63u;
  const bool data = wave != 0;
  const uint32_t dw = wave - 1;
  const uint32_t lbase = (uint32_t)(uintptr_t)lds;
  // static first NB segments (b + j * grid), then claims offset by NB * grid
  if (tid < NB) {
    const uint32_t s = blockIdx.x + tid * gridDim.x;
    s_seg[tid] = s < nseg ? s : NONE32;
  }
  uint32_t claimed = NONE32;
  if (tid == 0) claimed = atomicAdd(&ctl->ctr, 1u);  // (for iteration NB)
  __syncthreads();
  uint32_t q[NB];  // seg[i .. i+NB-1]
#pragma unroll
  for (uint32_t j = 0; j < NB; j++) q[j] = s_seg[j];
  auto dma_seg = [&](uint32_t s, uint32_t buf) {
    if (!data || s == NONE32) return;
#pragma unroll
    for (uint32_t k = 0; k < K; k++) {
      const uint32_t row = dw + NDW * k;
      dma16(p + (uint64_t)s * SEGB + row * 1024u + lane * 16u, lbase + buf * BUF + row * 1024u);
    }
  };
  // prologue: seg[0 .. NB-2] in flight (seg[NB-1] goes at iteration 0)
#pragma unroll
  for (uint32_t j = 0; j + 1 < NB; j++) dma_seg(q[j], j);
  uint32_t i = 0;
  while (q[0] != NONE32) {
    const uint32_t buf = i % NB;
    // (A) iteration i-1's LDS reads are done; the claim for seg[i+NB-1] lands
    if (tid == 0) {
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(claimed)::"memory");
      const uint32_t c = claimed + NB * gridDim.x;
      s_seg[NB] = c < nseg ? c : NONE32;
      if (c < nseg) claimed = atomicAdd(&ctl->ctr, 1u);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const uint32_t snew = q[NB - 1] == NONE32 ? NONE32 : s_seg[NB];
    // seg[i+NB-1] into the buffer iteration i-1 used
    dma_seg(q[NB - 1] == NONE32 ? NONE32 : q[NB - 1], (i + NB - 1) % NB);
    // seg[i]'s rows landed: ops after them are, per later iteration issued
    // so far, K stores and K DMAs (fewer at the end: a conservative 0 there)
    if (data) {
      const bool full = q[NB - 1] != NONE32;
      if (full) wait_vm<2 * K * (NB - 1)>();
      else wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();  // (B) every wave's rows of seg[i] are in LDS
    __builtin_amdgcn_s_barrier();  // (C) (the decoder's table barrier)
    if (data) {
      const uint64_t ss = (uint64_t)q[0] * SEGB;
      const uint64_t room = bytes > ss ? bytes - ss : 0;
      const auto w = __builtin_amdgcn_make_buffer_rsrc(p + ss, 0, room < SEGB ? (uint32_t)room : SEGB, 0x00020000);
      u32x4 prev = {0, 0, 0, 0};
#pragma unroll
      for (uint32_t k = 0; k < K; k++) {
        const uint32_t row = dw + NDW * k;
        const u32x4 d = *reinterpret_cast<const u32x4*>(&lds[buf * BUF + row * 1024u + lane * 16u]) ^ kw;
        __builtin_amdgcn_raw_buffer_store_b128(d, w, lane * 16u, row * 1024u, AUX_ST);
        asm volatile("" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
        prev = d;
      }
      asm volatile("s_nop 1" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
    }
#pragma unroll
    for (uint32_t j = 0; j + 1 < NB; j++) q[j] = q[j + 1];
    q[NB - 1] = snew;
    i++;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t d = atomicAdd(&ctl->done, 1u);
    if (d + 1 == gridDim.x) {
      __hip_atomic_store(&ctl->ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&ctl->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---- Q2: launches that exit at once (a word read from memory says "nothing")
__global__ void __launch_bounds__(1024) k_empty(const uint64_t* w, uint64_t* out) {
  if (*w == 0) return;
  out[threadIdx.x] = *w;
}
__global__ void __launch_bounds__(1024) k_empty_wave0(const uint64_t* w, uint64_t* out) {
  // only lane 0 of the workgroup reads; the answer through LDS
  __shared__ uint64_t s;
  if (threadIdx.x == 0) s = *w;
  __syncthreads();
  if (s == 0) return;
  out[threadIdx.x] = s;
}
__global__ void __launch_bounds__(1024) k_empty_scratch(const uint64_t* w, uint64_t* out, uint32_t idx) {
  if (*w == 0) return;
  volatile uint32_t a[48];
  for (int i = 0; i < 48; i++) a[i] = (uint32_t)(*w >> (i & 31));
  out[threadIdx.x] = a[idx % 48];
}
__global__ void __launch_bounds__(64) k_empty64(const uint64_t* w, uint64_t* out) {
  if (*w == 0) return;
  out[threadIdx.x] = *w;
}

int main(int argc, char** argv) {
  const bool only_launch = argc > 1 && argv[1][0] == 'L';
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  {
    uint64_t *w, *out;
    CK(hipMalloc(&w, 64));
    CK(hipMalloc(&out, 8192));
    CK(hipMemset(w, 0, 64));
    const int dyn = 136 * 1024;
    CK(hipFuncSetAttribute((const void*)k_empty, hipFuncAttributeMaxDynamicSharedMemorySize, dyn));
    CK(hipFuncSetAttribute((const void*)k_empty_scratch, hipFuncAttributeMaxDynamicSharedMemorySize, dyn));
    CK(hipFuncSetAttribute((const void*)k_empty_wave0, hipFuncAttributeMaxDynamicSharedMemorySize, dyn));
    auto lrun = [&](const char* name, auto launch) {
      for (int i = 0; i < 20; i++) launch();
      CK(hipDeviceSynchronize());
      const int it = 200;
      CK(hipEventRecord(a));
      for (int i = 0; i < it; i++) launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("launch %-44s %7.2f us per launch (back to back)\n", name, 1000.0 * ms / it);
      fflush(stdout);
    };
    lrun("256x1024, no LDS", [&] { k_empty<<<ncu, 1024>>>(w, out); });
    lrun("256x1024, 136 KiB dynamic LDS", [&] { k_empty<<<ncu, 1024, dyn>>>(w, out); });
    lrun("256x1024, 136 KiB LDS, one reader", [&] { k_empty_wave0<<<ncu, 1024, dyn>>>(w, out); });
    lrun("256x1024, 136 KiB LDS, scratch", [&] { k_empty_scratch<<<ncu, 1024, dyn>>>(w, out, 3); });
    lrun("256x64", [&] { k_empty64<<<ncu, 64>>>(w, out); });
    lrun("1x64", [&] { k_empty64<<<1, 64>>>(w, out); });
  }
  if (only_launch) return 0;
  const uint64_t bytes = 2147942400ull / 1843200 * 1843200;
  uint8_t* p;
  CK(hipMalloc(&p, bytes + 262144));
  CK(hipMemset(p, 0x5A, bytes + 262144));
  ctl_t* ctl;
  CK(hipMalloc(&ctl, sizeof(ctl_t)));
  CK(hipMemset(ctl, 0, sizeof(ctl_t)));
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
    printf("%-40s %8.4f ms  %7.1f GB/s (R+W) %s\n", name, ms, 2.0 * bytes / (ms * 1e-3) / 1e9, ok ? "" : "WRONG");
    fflush(stdout);
  };
  const uint32_t kw = 0x67676767u;
#define REG(KK)                                                                                                \
  do {                                                                                                         \
    const size_t sh = 15 * KK * 1024 + 64;                                                                     \
    CK(hipFuncSetAttribute((const void*)k_reg<KK>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh));      \
    run("reg K=" #KK, [&] { k_reg<KK><<<ncu, 1024, sh>>>(p, bytes, kw, ctl); });                              \
  } while (0)
#define DMA(KK, NB)                                                                                            \
  do {                                                                                                         \
    const size_t sh = (size_t)NB * (15 * KK * 1024 + 64);                                                      \
    CK(hipFuncSetAttribute((const void*)k_dma<KK, NB>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh));  \
    run("dma K=" #KK " NB=" #NB, [&] { k_dma<KK, NB><<<ncu, 1024, sh>>>(p, bytes, kw, ctl); });               \
  } while (0)
  REG(5);
  REG(8);
  DMA(5, 2);
  DMA(4, 2);
  DMA(3, 3);
  DMA(2, 4);
  DMA(2, 5);
  REG(5);
  DMA(5, 2);
  DMA(3, 3);
  return 0;
}
