// bw_probe2.hip — measurement probe (not product code): the in-place XOR
// ceiling on gfx950 for data paths the stream decoder could use, beside the
// round-1 register-prefetch + LDS-copy pattern (scripts/bw_probe.hip, "lds2").
//   hipcc --offload-arch=gfx950 -O3 scripts/bw_probe2.hip -o scripts/bw_probe2
// Prints one line per variant: ms per 2 GiB in-place pass and R+W GB/s.
//
// ring<NT, SLOT, R, D, BAR>: each workgroup streams its own contiguous range
// through an LDS ring of R slots of SLOT bytes filled by LDS-DMA
// (global_load_lds_dwordx4, nt), D slots in flight; every wave XORs and
// stores (nt buffer stores) the 1 KiB pieces it loaded itself, so without BAR
// the waves are independent; BAR adds one workgroup barrier per slot (what a
// decoder that shares the slot between waves for its header chase needs).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int NT, int SLOT, int R, int D, bool BAR>
__global__ void __launch_bounds__(NT) k_ring(uint8_t* p, uint64_t bytes, uint32_t kw) {
  extern __shared__ __attribute__((aligned(16))) uint8_t ring[];
  constexpr int NW = NT / 64;               // waves
  constexpr int PER = SLOT / 1024 / NW;     // 1 KiB pieces per wave per slot
  static_assert(PER >= 1 && D < R, "geometry");
  const uint64_t nslot_total = bytes / SLOT;
  const uint64_t per = (nslot_total + gridDim.x - 1) / gridDim.x;
  const uint64_t s0 = blockIdx.x * per;
  uint64_t s1 = s0 + per;
  if (s1 > nslot_total) s1 = nslot_total;
  if (s0 >= s1) return;
  const uint32_t n = (uint32_t)(s1 - s0);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  uint8_t* base = p + s0 * SLOT;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, n * SLOT, 0x00020000);
  auto issue = [&](uint32_t i) {
    uint8_t* lslot = ring + (i % R) * SLOT;
#pragma unroll
    for (int j = 0; j < PER; j++) {
      const uint32_t piece = j * NW + wave;
      __builtin_amdgcn_global_load_lds((const void*)(base + (uint64_t)i * SLOT + piece * 1024 + lane * 16),
                                       (lds_ptr_t)(lslot + piece * 1024), 16, 0, 2);
    }
  };
  for (uint32_t i = 0; i < D && i < n; i++) issue(i);
  for (uint32_t i = 0; i < n; i++) {
    const bool more = i + D < n;
    if (more) issue(i + D);
    if (more && i >= D) wait_vm<2 * PER * D>(); else wait_vm<0>();  // (first D iterations: fewer ops after)
    if (BAR) __builtin_amdgcn_s_barrier();
    const uint8_t* lslot = ring + (i % R) * SLOT;
    u32x4 v[PER];
#pragma unroll
    for (int j = 0; j < PER; j++) v[j] = *reinterpret_cast<const u32x4*>(lslot + (j * NW + wave) * 1024 + lane * 16);
    // (store data kept live past the next instruction: hipcc on gfx950 may
    // otherwise overwrite a dwordx4 store's data VGPRs right after it)
    u32x4 d[PER];
#pragma unroll
    for (int j = 0; j < PER; j++) d[j] = v[j] ^ kw;
#pragma unroll
    for (int j = 0; j < PER; j++) {
      __builtin_amdgcn_raw_buffer_store_b128(d[j], rs, (j * NW + wave) * 1024 + lane * 16, i * SLOT, 2);
      asm volatile("" ::"v"(d[j].x), "v"(d[j].y), "v"(d[j].z), "v"(d[j].w));
    }
    asm volatile("s_nop 1" ::"v"(d[PER - 1].x), "v"(d[PER - 1].y), "v"(d[PER - 1].z), "v"(d[PER - 1].w));
    if (BAR) __builtin_amdgcn_s_barrier();  // (the slot is refilled next iteration)
  }
}

// register double buffer + LDS copy + barriers: the round-1 decoder's data path
template <int NT, int SEGB>
__global__ void __launch_bounds__(NT) k_lds2(u32x4* p, uint64_t bytes, uint32_t kw) {
  constexpr int CH = SEGB / 16 / NT;
  extern __shared__ __attribute__((aligned(16))) u32x4 lds2[];
  const uint64_t nseg_total = bytes / SEGB;
  const uint64_t per = (nseg_total + gridDim.x - 1) / gridDim.x;
  uint64_t s0 = blockIdx.x * per, s1 = s0 + per;
  if (s1 > nseg_total) s1 = nseg_total;
  if (s0 >= s1) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (uint8_t*)p + s0 * SEGB, 0, (uint32_t)((s1 - s0) * SEGB), 0x00020000);
  const uint32_t vo = threadIdx.x * 16;
  u32x4 e[CH];
#pragma unroll
  for (int k = 0; k < CH; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, k * NT * 16, 2);
  for (uint64_t s = s0; s < s1; s++) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CH; k++) lds2[k * NT + threadIdx.x] = e[k];
    __syncthreads();
    if (s + 1 < s1) {
#pragma unroll
      for (int k = 0; k < CH; k++)
        e[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (uint32_t)((s + 1 - s0) * SEGB + k * NT * 16), 2);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CH; k++)
      __builtin_amdgcn_raw_buffer_store_b128(lds2[k * NT + threadIdx.x] ^ kw, rs, vo,
                                             (uint32_t)((s - s0) * SEGB + k * NT * 16), 2);
  }
}

__global__ void __launch_bounds__(256) k_gs_nt(u32x4* p, uint64_t n, uint32_t kw) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    u32x4 v = __builtin_nontemporal_load(p + i);
    __builtin_nontemporal_store(v ^ kw, p + i);
  }
}

// 4 chunks in flight per lane
__global__ void __launch_bounds__(256) k_gs4_nt(u32x4* p, uint64_t n, uint32_t kw) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += 4 * stride) {
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = i + k * stride < n ? __builtin_nontemporal_load(p + i + k * stride) : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; k++) if (i + k * stride < n) __builtin_nontemporal_store(v[k] ^ kw, p + i + k * stride);
  }
}

__global__ void __launch_bounds__(256) k_copy_nt(const u32x4* p, u32x4* q, uint64_t n, uint32_t kw) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load(p + i) ^ kw, q + i);
}

int main(int argc, char** argv) {
  const uint64_t bytes = 2147942400ull & ~131071ull;  // c3 batch, whole 128 KiB segments
  u32x4 *p, *q;
  CK(hipMalloc(&p, bytes));
  CK(hipMalloc(&q, bytes));
  CK(hipMemset(p, 0x5A, bytes));
  CK(hipMemset(q, 0x00, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  // check: after an even number of in-place passes the buffer is unchanged
  auto verify = [&](const char* name) {
    uint8_t h[4096];
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, (uint8_t*)p + bytes / 3 / 4096 * 4096, sizeof h, hipMemcpyDeviceToHost));
    for (int i = 0; i < 4096; i++)
      if (h[i] != 0x5A) { printf("%s: WRONG BYTES\n", name); return; }
  };
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
    printf("%-36s %8.3f ms  %7.1f GB/s (R+W)\n", name, ms, 2.0 * bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
    verify(name);
  };
  const uint64_t n16 = bytes / 16;
#define RING(NT, SLOT, R, D, BAR, WGPC)                                                                        \
  {                                                                                                           \
    auto kf = k_ring<NT, SLOT, R, D, BAR>;                                                                    \
    CK(hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, (SLOT) * (R)));        \
    run("ring " #NT "t " #SLOT "x" #R " d" #D " bar" #BAR " wg" #WGPC,                                        \
        [&] { kf<<<ncu * (WGPC), NT, (SLOT) * (R)>>>((uint8_t*)p, bytes, 0x1234567u); });                    \
  }
  CK(hipFuncSetAttribute((const void*)k_lds2<1024, 131072>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  run("lds2 1024t 128K (r01 decoder path)", [&] { k_lds2<1024, 131072><<<ncu, 1024, 131072>>>(p, bytes, 0x1234567u); });
  run("grid-stride nt 16B", [&] { k_gs_nt<<<ncu * 8, 256>>>(p, n16, 0x1234567u); });
  run("grid-stride nt 4x16B", [&] { k_gs4_nt<<<ncu * 8, 256>>>(p, n16, 0x1234567u); });
  run("copy p->q nt (out of place)", [&] { k_copy_nt<<<ncu * 8, 256>>>(p, q, n16, 0x1234567u); });
  RING(1024, 32768, 4, 3, false, 1)
  RING(1024, 32768, 4, 3, true, 1)
  RING(1024, 16384, 8, 7, false, 1)
  RING(1024, 16384, 8, 6, true, 1)
  RING(1024, 65536, 2, 1, false, 1)
  RING(1024, 65536, 2, 1, true, 1)
  RING(1024, 49152, 3, 2, true, 1)
  RING(512, 16384, 4, 3, false, 2)
  RING(512, 16384, 4, 3, true, 2)
  RING(1024, 16384, 4, 3, true, 1)
  return 0;
}
