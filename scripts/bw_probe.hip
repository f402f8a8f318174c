// bw_probe.hip — measurement probe (not product code): achievable in-place
// XOR bandwidth on gfx950 for the access shapes the stream decoder can use.
//   hipcc --offload-arch=gfx950 -O3 scripts/bw_probe.hip -o scripts/bw_probe
// Prints one line per variant: ms per 2 GiB in-place pass and R+W GB/s.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

// 1. grid-stride, one 16-B chunk per lane per iteration
__global__ void __launch_bounds__(256) k_gs(u32x4* p, uint64_t n, uint32_t kw) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    u32x4 v = p[i];
    v ^= kw;
    p[i] = v;
  }
}

// 2. grid-stride nontemporal
__global__ void __launch_bounds__(256) k_gs_nt(u32x4* p, uint64_t n, uint32_t kw) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    u32x4 v = __builtin_nontemporal_load(p + i);
    v ^= kw;
    __builtin_nontemporal_store(v, p + i);
  }
}

// 3. contiguous runs per workgroup, 64 KiB segments, register double buffer
template <int NT, bool NTMP>
__global__ void __launch_bounds__(NT) k_runs_reg(u32x4* p, uint64_t nseg_total, uint32_t kw) {
  constexpr int CH = 65536 / 16 / NT;
  const uint64_t per = (nseg_total + gridDim.x - 1) / gridDim.x;
  uint64_t s0 = blockIdx.x * per, s1 = s0 + per;
  if (s1 > nseg_total) s1 = nseg_total;
  if (s0 >= s1) return;
  u32x4 a[CH], b[CH];
  auto ld = [&](u32x4 (&d)[CH], uint64_t s) {
#pragma unroll
    for (int k = 0; k < CH; k++) {
      u32x4* q = p + s * 4096 + k * NT + threadIdx.x;
      d[k] = NTMP ? __builtin_nontemporal_load(q) : *q;
    }
  };
  auto st = [&](u32x4 (&d)[CH], uint64_t s) {
#pragma unroll
    for (int k = 0; k < CH; k++) {
      u32x4* q = p + s * 4096 + k * NT + threadIdx.x;
      u32x4 v = d[k] ^ kw;
      if (NTMP) __builtin_nontemporal_store(v, q); else *q = v;
    }
  };
  ld(a, s0);
  for (uint64_t s = s0; s < s1; s += 2) {
    if (s + 1 < s1) ld(b, s + 1);
    st(a, s);
    if (s + 1 >= s1) break;
    if (s + 2 < s1) ld(a, s + 2);
    st(b, s + 1);
  }
}

// 4. contiguous runs, 64 KiB LDS staging (write regs -> LDS, sync, prefetch
//    next, read LDS, XOR, store): the decoder's data movement without parsing
template <int NT>
__global__ void __launch_bounds__(NT) k_runs_lds(u32x4* p, uint64_t nseg_total, uint32_t kw) {
  constexpr int CH = 65536 / 16 / NT;
  __shared__ u32x4 lds[4096];
  const uint64_t per = (nseg_total + gridDim.x - 1) / gridDim.x;
  uint64_t s0 = blockIdx.x * per, s1 = s0 + per;
  if (s1 > nseg_total) s1 = nseg_total;
  if (s0 >= s1) return;
  u32x4 e[CH];
#pragma unroll
  for (int k = 0; k < CH; k++) e[k] = p[s0 * 4096 + k * NT + threadIdx.x];
  for (uint64_t s = s0; s < s1; s++) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CH; k++) lds[k * NT + threadIdx.x] = e[k];
    __syncthreads();
    if (s + 1 < s1) {
#pragma unroll
      for (int k = 0; k < CH; k++) e[k] = p[(s + 1) * 4096 + k * NT + threadIdx.x];
    }
    // a dependent LDS walk (stand-in for the header chase)
    if (threadIdx.x == 0) {
      uint32_t x = 0;
      for (int h = 0; h < 2; h++) x = lds[(x + 17) & 4095].x & 4095;
      lds[4095].w ^= (x == 0xFFFFFFFF);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CH; k++) p[s * 4096 + k * NT + threadIdx.x] = lds[k * NT + threadIdx.x] ^ kw;
  }
}


// 5. calibration: out-of-place copy (read p, write q), read-only, write-only
template <int NT>
__global__ void __launch_bounds__(NT) k_copy_runs(const u32x4* p, u32x4* q, uint64_t nseg_total, uint32_t kw) {
  constexpr int CH = 65536 / 16 / NT;
  const uint64_t per = (nseg_total + gridDim.x - 1) / gridDim.x;
  uint64_t s0 = blockIdx.x * per, s1 = s0 + per;
  if (s1 > nseg_total) s1 = nseg_total;
  for (uint64_t s = s0; s < s1; s++) {
    u32x4 d[CH];
#pragma unroll
    for (int k = 0; k < CH; k++) d[k] = __builtin_nontemporal_load(p + s * 4096 + k * NT + threadIdx.x);
#pragma unroll
    for (int k = 0; k < CH; k++) __builtin_nontemporal_store(d[k] ^ kw, q + s * 4096 + k * NT + threadIdx.x);
  }
}
__global__ void __launch_bounds__(256) k_read(const u32x4* p, uint64_t n, uint32_t* out) {
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    acc ^= __builtin_nontemporal_load(p + i);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345) out[0] = 1;
}
__global__ void __launch_bounds__(256) k_write(u32x4* p, uint64_t n, uint32_t kw) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    __builtin_nontemporal_store(u32x4{kw, kw, kw, kw}, p + i);
}
// 6. runs with buffer loads/stores and explicit cache-policy aux bits; SEGB bytes
//    per iteration, 2-deep register pipeline
template <int NT, int SEGB, int LAUX, int SAUX>
__global__ void __launch_bounds__(NT) k_runs_buf(u32x4* p, uint64_t bytes, uint32_t kw) {
  constexpr int CH = SEGB / 16 / NT;
  const uint64_t nseg_total = bytes / SEGB;
  const uint64_t per = (nseg_total + gridDim.x - 1) / gridDim.x;
  uint64_t s0 = blockIdx.x * per, s1 = s0 + per;
  if (s1 > nseg_total) s1 = nseg_total;
  if (s0 >= s1) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (uint8_t*)p + s0 * SEGB, 0, (uint32_t)((s1 - s0) * SEGB), 0x00020000);
  u32x4 a[CH], b[CH];
  const uint32_t vo = threadIdx.x * 16;
  auto ld = [&](u32x4 (&d)[CH], uint64_t s) {
#pragma unroll
    for (int k = 0; k < CH; k++)
      d[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (uint32_t)((s - s0) * SEGB + k * NT * 16), LAUX);
  };
  auto st = [&](u32x4 (&d)[CH], uint64_t s) {
#pragma unroll
    for (int k = 0; k < CH; k++)
      __builtin_amdgcn_raw_buffer_store_b128(d[k] ^ kw, rs, vo, (uint32_t)((s - s0) * SEGB + k * NT * 16), SAUX);
  };
  ld(a, s0);
  for (uint64_t s = s0; s < s1; s += 2) {
    if (s + 1 < s1) ld(b, s + 1);
    st(a, s);
    if (s + 1 >= s1) break;
    if (s + 2 < s1) ld(a, s + 2);
    st(b, s + 1);
  }
}


// 7. 1024-thread runs, SEGB per iteration, nt buffer ops, LDS copy of the
//    current segment for header access. XFROM_LDS: XOR source is the LDS copy
//    (else a register copy kept alongside).
template <int NT, int SEGB, bool XFROM_LDS, int WALK = 3, int XOPS = 0>
__global__ void __launch_bounds__(NT) k_runs_lds2(u32x4* p, uint64_t bytes, uint32_t kw) {
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
  u32x4 e[CH], c[CH];
#pragma unroll
  for (int k = 0; k < CH; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, k * NT * 16, 2);
  for (uint64_t s = s0; s < s1; s++) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CH; k++) { lds2[k * NT + threadIdx.x] = e[k]; c[k] = e[k]; }
    __syncthreads();
    if (s + 1 < s1) {
#pragma unroll
      for (int k = 0; k < CH; k++)
        e[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (uint32_t)((s + 1 - s0) * SEGB + k * NT * 16), 2);
    }
    if (threadIdx.x == 0) {  // dependent LDS walk (stand-in for the chase)
      uint32_t x = 0;
      const volatile uint32_t* lv = reinterpret_cast<const volatile uint32_t*>(lds2);
      for (int h = 0; h < WALK; h++) x = (lv[4 * ((x + 17) & (SEGB / 16 - 1))] + h) & (SEGB / 16 - 1);
      if (x == 0xFFFFFFFF) lds2[0].w = 0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CH; k++) {
      u32x4 v = XFROM_LDS ? lds2[k * NT + threadIdx.x] : c[k];
      uint32_t kk = kw;
#pragma unroll
      for (int o = 0; o < XOPS; o++) kk = __builtin_amdgcn_alignbyte(kk, v.x, o & 3) ^ (kk >> 1);
      if (XOPS) v.y ^= kk & 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(v ^ kw, rs, vo, (uint32_t)((s - s0) * SEGB + k * NT * 16), 2);
    }
  }
}

int main(int argc, char** argv) {
  const uint64_t bytes = 2147942400ull & ~65535ull;  // c3 batch, whole segments
  const uint64_t nseg = bytes / 65536;
  u32x4* p;
  CK(hipMalloc(&p, bytes));
  CK(hipMemset(p, 0x5A, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; i++) launch();
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

  CK(hipFuncSetAttribute((const void*)k_runs_lds2<1024, 131072, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)k_runs_lds2<1024, 131072, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  run("lds2 1024t 128K fromLDS x1", [&] { k_runs_lds2<1024, 131072, true><<<ncu, 1024, 131072>>>(p, bytes, 0x1234567u); });
#define WV(W, X) \
  CK(hipFuncSetAttribute((const void*)k_runs_lds2<1024, 131072, true, W, X>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072)); \
  run("lds2 128K walk " #W " xops " #X, [&] { k_runs_lds2<1024, 131072, true, W, X><<<ncu, 1024, 131072>>>(p, bytes, 0x1234567u); });
  WV(30, 0) WV(60, 0) WV(100, 0) WV(150, 0) WV(200, 0) WV(100, 8) WV(100, 16) WV(60, 16) WV(3, 16)
  if (argc > 1) return 0;
  run("lds2 1024t 128K fromREG x1", [&] { k_runs_lds2<1024, 131072, false><<<ncu, 1024, 131072>>>(p, bytes, 0x1234567u); });
  run("lds2 1024t 64K fromLDS x2", [&] { k_runs_lds2<1024, 65536, true><<<ncu * 2, 1024, 65536>>>(p, bytes, 0x1234567u); });
  run("lds2 512t 64K fromLDS x2", [&] { k_runs_lds2<512, 65536, true><<<ncu * 2, 512, 65536>>>(p, bytes, 0x1234567u); });
  run("lds2 1024t 64K fromLDS x1", [&] { k_runs_lds2<1024, 65536, true><<<ncu, 1024, 65536>>>(p, bytes, 0x1234567u); });
  run("buf 1024t 256K nt/nt x1", [&] { k_runs_buf<1024, 262144, 2, 2><<<ncu * 1, 1024>>>(p, bytes, 0x1234567u); });
  run("buf 1024t 64K nt/nt x1", [&] { k_runs_buf<1024, 65536, 2, 2><<<ncu * 1, 1024>>>(p, bytes, 0x1234567u); });
  run("buf 1024t 64K nt/nt x2", [&] { k_runs_buf<1024, 65536, 2, 2><<<ncu * 2, 1024>>>(p, bytes, 0x1234567u); });
  run("buf 1024t 128K nt/nt x1 (again)", [&] { k_runs_buf<1024, 131072, 2, 2><<<ncu * 1, 1024>>>(p, bytes, 0x1234567u); });
  return 0;
}
