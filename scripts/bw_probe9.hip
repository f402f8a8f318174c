// bw_probe9.hip — measurement probe (not product code), round 4.
// Question: which part of the lattice decoder's segment loop (xyws_lattice.h)
// costs bandwidth against bw_probe7's k_seg (128 KiB claimed segments staged in
// LDS, 6.43 TB/s)? The same skeleton with the lattice loop's features switched
// on one at a time, on the c3-sized 2 GiB in-place XOR (R+W bytes / time):
//   CW   wave 0 is a control wave (no rows): 15 data waves, 120 KiB segments
//   AC   the claim by lane 0 of the first data wave (inline-asm atomic issued
//        before its rows, value read after the next fill), not by thread 0
//   B3   three barriers per segment (fill | issue+table | stores), not two
//   XL   the claim wave's extra dword loads (header / pad words)
//   ST   the control wave's per-segment status store, group count and load
//   WV   k_seg's vmcnt(0) (the next segment landed) before the stores
//   hipcc --offload-arch=gfx950 -O3 scripts/bw_probe9.hip -o scripts/bw_probe9
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr uint32_t NONE32 = 0xFFFFFFFFu;
constexpr uint32_t OOB = 0x40000000u;
enum { CW = 1, AC = 2, B3 = 4, XL = 8, ST = 16, WV = 32, S_ST = 64, S_GR = 128, S_LD = 256, S_NW = 512, S_SP = 1024,
       S_REP = 2048, S_EV4 = 4096 };

struct ctl_t { uint32_t ctr, done; uint64_t pad[7]; uint64_t stat[1 << 16]; uint64_t grp[1 << 12]; uint64_t rep[64 * 32]; };

template <uint32_t F>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4)))
k_skel(uint8_t* p, uint64_t bytes, uint32_t kw, ctl_t* ctl, uint64_t E) {
  constexpr bool CTRL = F & CW;
  constexpr uint32_t NDW = CTRL ? 15 : 16, K = 8, SEGB = NDW * K * 1024;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ uint32_t s_nxt;
  const uint32_t nseg = (uint32_t)((bytes + SEGB - 1) / SEGB);
  uint32_t tid = threadIdx.x;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63u;
  const bool data = !CTRL || wave != 0;
  const uint32_t dw = CTRL ? wave - 1 : wave;
  constexpr uint32_t CLAIM = (F & AC) ? (CTRL ? 64u : 0u) : 0u;
  uint32_t ahead = NONE32, cx = 0;
  if (tid == CLAIM) {
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
    if ((F & AC) && wave == CLAIM / 64) {
      if (lane == 0) {
        if (claim) asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(ahead) : "v"(&ctl->ctr), "v"(1u) : "memory");
        else ahead = NONE32;
      }
      if (F & XL) {
        const uint64_t q = (uint64_t)s * SEGB + 4u * (tid & 63u);
        cx = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p + (q + 4 < bytes ? q : 0)));
      }
    }
    const auto r = rsrc((uint64_t)s * SEGB);
#pragma unroll
    for (uint32_t k = 0; k < K; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16u, (dw + NDW * k) * 1024u, 2);
  };
  if (cur != NONE32 && data) {
    const uint32_t a0 = ahead;
    issue(cur, false);
    ahead = a0;
    const auto r = rsrc((uint64_t)cur * SEGB);
#pragma unroll
    for (uint32_t k = 0; k < K; k++) __builtin_amdgcn_raw_buffer_store_b128(u32x4{0, 0, 0, 0}, r, OOB, k * 1024u, 2);
  }
  uint64_t brk_seen = 0;
  uint32_t it = 0;
  while (cur != NONE32) {
    it++;
    asm volatile("" : "+v"(tid));
    __syncthreads();  // (A)
    if (data) {
#pragma unroll
      for (uint32_t k = 0; k < K; k++) *reinterpret_cast<u32x4*>(&lds[(dw + NDW * k) * 1024u + lane * 16u]) = e[k];
    }
    if (F & AC) {
      if (data && wave == CLAIM / 64) {
        asm volatile("" : "+v"(ahead), "+v"(cx) : "v"(e[K - 1].x));
        if ((tid & 63u) < 9) *reinterpret_cast<uint32_t*>(&lds[SEGB + 4u * (tid & 63u)]) = cx;
        if (lane == 0) s_nxt = ahead < nseg ? ahead : NONE32;
      }
    } else if (tid == 0) {
      s_nxt = ahead < nseg ? ahead : NONE32;
      if (ahead < nseg) ahead = atomicAdd(&ctl->ctr, 1u);
    }
    __syncthreads();  // (B)
    const uint32_t nxt = s_nxt;
    if (nxt != NONE32) issue(nxt, true);
    if ((F & ST) && CTRL && wave == 0 && lane == 0) {
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(brk_seen)::"memory");
      __hip_atomic_store(&ctl->stat[cur & 0xFFFF], (E << 2) | 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&ctl->grp[(cur / 64) & 0xFFF], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(brk_seen) : "v"(&ctl->pad[0]) : "memory");
    }
    // (the parts of ST one at a time; S_NW: no wait; S_SP: the status words
    // and group counters spread 1 per 256 B instead of packed)
    constexpr uint32_t SPR = (F & S_SP) ? 32u : 1u;
    if ((F & (S_ST | S_GR | S_LD)) && CTRL && wave == 0 && lane == 0) {
      if (!(F & S_NW)) asm volatile("s_waitcnt vmcnt(0)" : "+v"(brk_seen)::"memory");
      if (F & S_ST) __hip_atomic_store(&ctl->stat[(cur * SPR) & 0xFFFF], (E << 2) | 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (F & S_GR) __hip_atomic_fetch_add(&ctl->grp[((cur / 64) * SPR) & 0xFFF], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // (S_REP: one of 64 replicas, 256 B apart, by workgroup; S_EV4: every 4th segment)
      const uint64_t* src = (F & S_REP) ? &ctl->rep[(blockIdx.x & 63u) * 32u] : &ctl->pad[0];
      if ((F & S_LD) && (!(F & S_EV4) || (it & 3u) == 0))
        asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(brk_seen) : "v"(src) : "memory");
    }
    if (F & WV) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (F & B3) __syncthreads();  // (C)
    if (data) {
      const auto w = rsrc((uint64_t)cur * SEGB);
      u32x4 prev = {0, 0, 0, 0};
#pragma unroll
      for (uint32_t k = 0; k < K; k++) {
        const uint32_t a = (dw + NDW * k) * 1024u + lane * 16u;
        const u32x4 d = *reinterpret_cast<const u32x4*>(&lds[a]) ^ kw;
        __builtin_amdgcn_raw_buffer_store_b128(d, w, lane * 16u, (dw + NDW * k) * 1024u, 2);
        asm volatile("" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
        prev = d;
      }
      asm volatile("s_nop 1" ::"v"(prev.x), "v"(prev.y), "v"(prev.z), "v"(prev.w));
    }
    cur = nxt;
  }
  if ((F & (ST | S_LD)) && brk_seen == 12345) ctl->pad[1] = 1;  // (keeps the loads)
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

int main() {
  const uint64_t bytes = 2147942400ull / 122880 * 122880;
  uint8_t* p;
  CK(hipMalloc(&p, bytes + 131072));
  CK(hipMemset(p, 0x5A, bytes + 131072));
  ctl_t* ctl;
  CK(hipMalloc(&ctl, sizeof(ctl_t)));
  CK(hipMemset(ctl, 0, sizeof(ctl_t)));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  uint64_t E = 0;
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
    printf("%-40s %8.4f ms  %7.1f GB/s (R+W) %s\n", name, ms, 2.0 * bytes / (ms * 1e-3) / 1e9, h[0] == 0x5A ? "" : "WRONG");
    fflush(stdout);
  };
  const uint32_t kw = 0x67676767u;
#define SKEL(FL)                                                                                            \
  do {                                                                                                      \
    const size_t sh = 131072 + 64;                                                                          \
    CK(hipFuncSetAttribute((const void*)k_skel<FL>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh)); \
    run("skel flags " #FL, [&] { k_skel<FL><<<ncu, 1024, sh>>>(p, bytes, kw, ctl, ++E); });               \
  } while (0)
  SKEL(CW | AC | B3 | XL);
  SKEL(CW | AC | B3 | XL | S_LD);
  SKEL(CW | AC | B3 | XL | S_LD | S_REP);
  SKEL(CW | AC | B3 | XL | S_LD | S_EV4);
  SKEL(CW | AC | B3 | XL | S_LD | S_REP | S_EV4);
  SKEL(CW | AC | B3 | XL | S_ST | S_GR | S_LD | S_REP);
  SKEL(CW | AC | B3 | XL);
  return 0;
}
