// Standalone sweep of 1 GB device-copy variants (the N=1 bench step is one K1 NIN=1 launch):
// loads/stores nontemporal or not, vectors per lane, block size, one-shot grid vs persistent
// grid-stride.  Prints GB/s of (read + write) bytes / 2, i.e. the bench's algbw definition.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

template <bool NTL>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NTL) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NTS>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if constexpr (NTS) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// one tile of B*U vectors per block, all U loads issued before the stores
template <int B, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(B) void k_tile(u32x4* __restrict__ out, const u32x4* __restrict__ in, long nvec) {
  const long base = (long)blockIdx.x * B * U + threadIdx.x;
  if (base + (long)(U - 1) * B < nvec) {
    u32x4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = ld<NTL>(in + base + u * B);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NTS>(out + base + u * B, r[u]);
  } else {
    for (int u = 0; u < U; ++u) {
      long v = base + (long)u * B;
      if (v < nvec) out[v] = in[v];
    }
  }
}

// persistent grid-stride: G blocks, each moves B*U vectors per iteration
template <int B, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(B) void k_stride(u32x4* __restrict__ out, const u32x4* __restrict__ in, long nvec) {
  const long step = (long)gridDim.x * B * U;
  for (long base = (long)blockIdx.x * B * U + threadIdx.x; base < nvec; base += step) {
    if (base + (long)(U - 1) * B < nvec) {
      u32x4 r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) r[u] = ld<NTL>(in + base + u * B);
#pragma unroll
      for (int u = 0; u < U; ++u) st<NTS>(out + base + u * B, r[u]);
    } else {
      for (int u = 0; u < U; ++u) {
        long v = base + (long)u * B;
        if (v < nvec) out[v] = in[v];
      }
    }
  }
}

static float time_it(void (*launch)(u32x4*, const u32x4*, long), u32x4* o, const u32x4* i, long nvec) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) launch(o, i, nvec);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f, tot = 0;
  const int it = 20;
  for (int k = 0; k < it; ++k) {
    CHECK(hipEventRecord(a, 0));
    launch(o, i, nvec);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
    tot += ms;
  }
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return tot / it;
}

#define TILE(B, U, L, S)                                                                         \
  {                                                                                              \
    "tile B" #B " U" #U " ntl" #L " nts" #S, [](u32x4* o, const u32x4* i, long n) {               \
      long g = (n + (long)B * U - 1) / ((long)B * U);                                            \
      hipLaunchKernelGGL((k_tile<B, U, L, S>), dim3((unsigned)g), dim3(B), 0, 0, o, i, n);       \
    }                                                                                            \
  }
#define STRIDE(B, U, L, S, G)                                                                    \
  {                                                                                              \
    "stride B" #B " U" #U " ntl" #L " nts" #S " G" #G, [](u32x4* o, const u32x4* i, long n) {     \
      hipLaunchKernelGGL((k_stride<B, U, L, S>), dim3(G), dim3(B), 0, 0, o, i, n);               \
    }                                                                                            \
  }

struct V {
  const char* name;
  void (*launch)(u32x4*, const u32x4*, long);
};

int main() {
  const long bytes = 1000000000L;
  const long nvec = bytes / 16;
  u32x4 *in, *out;
  CHECK(hipMalloc(&in, bytes));
  CHECK(hipMalloc(&out, bytes));
  CHECK(hipMemset(in, 1, bytes));
  V vs[] = {
      TILE(256, 4, true, true),         STRIDE(256, 4, true, true, 4096),  STRIDE(256, 4, true, true, 3072),
      STRIDE(256, 4, true, true, 6144), STRIDE(256, 4, true, true, 8192),  STRIDE(256, 2, true, true, 4096),
      STRIDE(256, 2, true, true, 8192), STRIDE(256, 4, true, false, 4096), STRIDE(256, 8, true, true, 2048),
      STRIDE(256, 8, true, true, 4096), STRIDE(128, 4, true, true, 8192),  STRIDE(256, 4, true, true, 2560),
      STRIDE(256, 4, true, true, 5120),
  };
  // hipMemcpyAsync D2D for reference
  {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) CHECK(hipMemcpyAsync(out, in, bytes, hipMemcpyDeviceToDevice, 0));
    float tot = 0;
    for (int k = 0; k < 20; ++k) {
      CHECK(hipEventRecord(a, 0));
      CHECK(hipMemcpyAsync(out, in, bytes, hipMemcpyDeviceToDevice, 0));
      CHECK(hipEventRecord(b, 0));
      CHECK(hipEventSynchronize(b));
      float ms;
      CHECK(hipEventElapsedTime(&ms, a, b));
      tot += ms;
    }
    printf("%-40s %8.1f us  %7.0f GB/s\n", "hipMemcpyAsync D2D", tot / 20 * 1e3, bytes / (tot / 20 * 1e-3) / 1e9);
  }
  for (auto& v : vs) {
    float ms = time_it(v.launch, out, in, nvec);
    printf("%-40s %8.1f us  %7.0f GB/s\n", v.name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
  }
  CHECK(hipFree(in));
  CHECK(hipFree(out));
  return 0;
}
