// Experiment: which part of k_zs_compact produces WRITE_SIZE traffic at density 0?
// Variants of the compaction kernel on an all-zero 256 MiB input (nothing should be written).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256;

template <int V>
__global__ __launch_bounds__(kBlock) void k_var(const uint32_t* __restrict__ in, int64_t nblk,
                                                const int64_t* __restrict__ offs, uint32_t* __restrict__ vals) {
  __shared__ uint32_t stage[4][1024];
  const int lane = threadIdx.x & 63;
  uint32_t* st = stage[threadIdx.x >> 6];
  const uint64_t lt = (1ull << lane) - 1;
  const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t b0 = wave * 4; b0 < nblk; b0 += nwaves * 4) {
    uint32_t v[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const u32x4 t = (V == 4) ? *reinterpret_cast<const u32x4*>(in + (b0 + u) * 256 + lane * 4)
                               : __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in + (b0 + u) * 256 + lane * 4));
      __builtin_memcpy(v[u], &t, 16);
    }
    if (V == 0) continue;                       // loads only
    const int64_t base = offs[b0];
    const int total = (int)(offs[b0 + 4 < nblk ? b0 + 4 : nblk] - base);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      int q = (int)(offs[b0 + u] - base);
#pragma unroll
      for (int k = 0; k < 4; ++k) q += __popcll(__ballot(v[u][k] != 0) & lt);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (v[u][k] != 0) st[q++] = v[u][k];
    }
    if (V == 1) continue;                       // + LDS staging, no global stores
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < total; i += 64) vals[base + i] = st[i];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
}

int main() {
  const int64_t n = 64ll << 20, nblk = n / 256;
  uint32_t *in, *vals;
  int64_t* offs;
  hipMalloc(&in, n * 4);
  hipMalloc(&vals, n * 4);
  hipMalloc(&offs, (nblk + 1) * 8);
  hipMemset(in, 0, n * 4);
  hipMemset(offs, 0, (nblk + 1) * 8);
  hipDeviceSynchronize();
  const int g = 2048;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_var<0>, dim3(g), dim3(kBlock), 0, 0, in, nblk, offs, vals);
    hipLaunchKernelGGL(k_var<1>, dim3(g), dim3(kBlock), 0, 0, in, nblk, offs, vals);
    hipLaunchKernelGGL(k_var<2>, dim3(g), dim3(kBlock), 0, 0, in, nblk, offs, vals);
    hipLaunchKernelGGL(k_var<4>, dim3(g), dim3(kBlock), 0, 0, in, nblk, offs, vals);
  }
  hipError_t e = hipDeviceSynchronize();
  printf("done %d\n", (int)e);
  return (int)e;
}
