// K4 / K5 / K7 / K8 — sparse Map<String, T> collectives on the GPU (gfx950).
//
// Reference hot loops: hash partitioning of map keys (ProcessCommSlave.java:2059-2072), the
// MapReduce deserializer's per-key merge (J/operand/DoubleOperand.java:225-257) and the
// Set/List specials built on it (ProcessCommSlave.java:1583-1720).  On the device, string
// keys travel as 64-bit ids (host dictionary) and a map is a (keys[n], vals[n, dim]) pair:
//
//   K4  owner + histogram:  dest = id % p, per-block LDS histogram, one atomic per bucket;
//       the stable radix sort by dest (hipCUB) then gives the all-to-all send layout.
//   K5  reduce-by-key:      stable radix sort by id (rank order preserved inside a key),
//       head flags + DeviceSelect give run starts, then one wave per run reduces its rows
//       (lanes over `dim`) in run order => deterministic, no float atomics.
//   K7  set union / intersection / concat reuse the same runs (count == p for intersection).
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace mp4x {

__global__ __launch_bounds__(kBlock) void k_key_owner(const int64_t* __restrict__ keys, int64_t n, int p,
                                                      int32_t* __restrict__ dest, int32_t* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) int32_t lh[];
  for (int i = threadIdx.x; i < p; i += kBlock) lh[i] = 0;
  __syncthreads();
  const int64_t nthr = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += nthr) {
    int d = (int)((uint64_t)keys[i] % (uint64_t)p);
    dest[i] = d;
    atomicAdd(&lh[d], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < p; i += kBlock)
    if (lh[i]) atomicAdd(&hist[i], lh[i]);
}

__global__ __launch_bounds__(kBlock) void k_head_flags(const int64_t* __restrict__ k, int64_t n,
                                                       int32_t* __restrict__ flags) {
  const int64_t nthr = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += nthr)
    flags[i] = (i == 0 || k[i] != k[i - 1]) ? 1 : 0;
}

// One wave per run; lanes stride over the row.  Rows are combined in run order (= rank order
// after the stable sort), local-first like the reference's MapReduce serializer.
template <int DT, int OP>
__global__ __launch_bounds__(kBlock) void k_segment_reduce(const int64_t* __restrict__ sk, const int64_t* __restrict__ perm,
                                                           const int64_t* __restrict__ starts,
                                                           const int64_t* __restrict__ nruns_dev, int64_t n,
                                                           const void* __restrict__ vals_, int64_t dim,
                                                           int64_t* __restrict__ out_keys, void* __restrict__ out_vals_,
                                                           int32_t* __restrict__ out_count) {
  using E = Elem<DT>;
  using S = typename E::S;
  using A = typename E::A;
  const S* vals = reinterpret_cast<const S*>(vals_);
  S* out_vals = reinterpret_cast<S*>(out_vals_);
  const int lane = threadIdx.x & 63;
  const int64_t nruns = *nruns_dev;
  const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t u = wave; u < nruns; u += nwaves) {
    const int64_t s = starts[u];
    const int64_t e = (u + 1 < nruns) ? starts[u + 1] : n;
    if (lane == 0) {
      out_keys[u] = sk[s];
      if (out_count) out_count[u] = (int32_t)(e - s);
    }
    if (!vals) continue;
    for (int64_t d = lane; d < dim; d += 64) {
      A acc = E::load(vals[perm[s] * dim + d]);
      for (int64_t j = s + 1; j < e; ++j) acc = combine<DT, OP>(acc, E::load(vals[perm[j] * dim + d]));
      out_vals[u * dim + d] = E::store(acc);
    }
  }
}

// Vectorised form: rows of V 16-byte vectors, G lanes per run (64/G runs per wave), each lane
// accumulates one 16-byte vector of the row across the run's rows (2 rows per step in flight).
template <int DT, int OP>
__global__ __launch_bounds__(kBlock) void k_segment_reduce_vec(const int64_t* __restrict__ sk,
                                                               const int64_t* __restrict__ perm,
                                                               const int64_t* __restrict__ starts,
                                                               const int64_t* __restrict__ nruns_dev, int64_t n,
                                                               const u32x4* __restrict__ vals, int64_t V, int G,
                                                               int64_t* __restrict__ out_keys,
                                                               u32x4* __restrict__ out_vals,
                                                               int32_t* __restrict__ out_count) {
  using E = Elem<DT>;
  using S = typename E::S;
  using A = typename E::A;
  constexpr int W = 16 / sizeof(S);
  const int lane = threadIdx.x & 63;
  const int grp = lane / G, sub = lane % G, R = 64 / G;
  const int64_t nruns = *nruns_dev;
  const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t u0 = wave * R; u0 < nruns; u0 += nwaves * R) {
    const int64_t u = u0 + grp;
    if (u >= nruns) continue;
    const int64_t s = starts[u];
    const int64_t e = (u + 1 < nruns) ? starts[u + 1] : n;
    if (sub == 0) {
      out_keys[u] = sk[s];
      if (out_count) out_count[u] = (int32_t)(e - s);
    }
    for (int64_t v = sub; v < V; v += G) {
      S x[W];
      u32x4 t = vals[perm[s] * V + v];
      __builtin_memcpy(x, &t, 16);
      A acc[W];
#pragma unroll
      for (int j = 0; j < W; ++j) acc[j] = E::load(x[j]);
      int64_t j = s + 1;
      for (; j + 1 < e; j += 2) {          // two rows in flight
        u32x4 t0 = vals[perm[j] * V + v];
        u32x4 t1 = vals[perm[j + 1] * V + v];
        S y0[W], y1[W];
        __builtin_memcpy(y0, &t0, 16);
        __builtin_memcpy(y1, &t1, 16);
#pragma unroll
        for (int q = 0; q < W; ++q) acc[q] = combine<DT, OP>(combine<DT, OP>(acc[q], E::load(y0[q])), E::load(y1[q]));
      }
      if (j < e) {
        u32x4 t0 = vals[perm[j] * V + v];
        S y0[W];
        __builtin_memcpy(y0, &t0, 16);
#pragma unroll
        for (int q = 0; q < W; ++q) acc[q] = combine<DT, OP>(acc[q], E::load(y0[q]));
      }
#pragma unroll
      for (int q = 0; q < W; ++q) x[q] = E::store(acc[q]);
      u32x4 o;
      __builtin_memcpy(&o, x, 16);
      out_vals[u * V + v] = o;
    }
  }
}

template <int DT, int OP>
static int launch_sr(const int64_t* sk, const int64_t* perm, const int64_t* starts, const int64_t* nr, int64_t n,
                     int64_t max_runs, const void* vals, int64_t dim, int64_t* ok, void* ov, int32_t* oc,
                     hipStream_t st) {
  if constexpr (!op_valid<DT, OP>()) {
    return MP4X_E_UNSUPPORTED;
  } else {
    using S = typename Elem<DT>::S;
    const int64_t row_bytes = dim * (int64_t)sizeof(S);
    if (vals && (row_bytes & 15) == 0 && ((((uintptr_t)vals | (uintptr_t)ov) & 15) == 0)) {
      const int64_t V = row_bytes / 16;
      int G = 1;
      while (G < V && G < 64) G <<= 1;
      int g = grid_for((max_runs * G + 63) / 64 * 64, 1);
      hipLaunchKernelGGL((k_segment_reduce_vec<DT, OP>), dim3(g), dim3(kBlock), 0, st, sk, perm, starts, nr, n,
                         (const u32x4*)vals, V, G, ok, (u32x4*)ov, oc);
      return (int)hipGetLastError();
    }
    int g = grid_for(max_runs * 64, 1);
    hipLaunchKernelGGL((k_segment_reduce<DT, OP>), dim3(g), dim3(kBlock), 0, st, sk, perm, starts, nr, n, vals, dim,
                       ok, ov, oc);
    return (int)hipGetLastError();
  }
}

template <int DT>
static int sr_dt(int op, const int64_t* sk, const int64_t* perm, const int64_t* starts, const int64_t* nr, int64_t n,
                 int64_t mr, const void* vals, int64_t dim, int64_t* ok, void* ov, int32_t* oc, hipStream_t st) {
  switch (op) {
    case MP4X_SUM: return launch_sr<DT, MP4X_SUM>(sk, perm, starts, nr, n, mr, vals, dim, ok, ov, oc, st);
    case MP4X_MAX: return launch_sr<DT, MP4X_MAX>(sk, perm, starts, nr, n, mr, vals, dim, ok, ov, oc, st);
    case MP4X_MIN: return launch_sr<DT, MP4X_MIN>(sk, perm, starts, nr, n, mr, vals, dim, ok, ov, oc, st);
    case MP4X_PROD: return launch_sr<DT, MP4X_PROD>(sk, perm, starts, nr, n, mr, vals, dim, ok, ov, oc, st);
    case MP4X_BAND: return launch_sr<DT, MP4X_BAND>(sk, perm, starts, nr, n, mr, vals, dim, ok, ov, oc, st);
    case MP4X_BOR: return launch_sr<DT, MP4X_BOR>(sk, perm, starts, nr, n, mr, vals, dim, ok, ov, oc, st);
    case MP4X_BXOR: return launch_sr<DT, MP4X_BXOR>(sk, perm, starts, nr, n, mr, vals, dim, ok, ov, oc, st);
    default: return MP4X_E_UNSUPPORTED;
  }
}

}  // namespace mp4x

using namespace mp4x;

extern "C" int mp4x_key_owner(const int64_t* keys, int64_t n, int p, int32_t* dest, int32_t* hist, void* stream) {
  if (n <= 0) return 0;
  if (p < 1 || p > 4096) return MP4X_E_BADARG;
  int g = grid_for(n, 8);
  hipLaunchKernelGGL(k_key_owner, dim3(g), dim3(kBlock), p * sizeof(int32_t), (hipStream_t)stream, keys, n, p, dest,
                     hist);
  return (int)hipGetLastError();
}

extern "C" size_t mp4x_sort_pairs_temp_bytes(int64_t n, int key_is_i32) {
  size_t bytes = 0;
  if (key_is_i32)
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr,
                                       (const int64_t*)nullptr, (int64_t*)nullptr, (int)n, 0, 32, (hipStream_t)0);
  else
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int64_t*)nullptr, (int64_t*)nullptr,
                                       (const int64_t*)nullptr, (int64_t*)nullptr, (int)n, 0, 64, (hipStream_t)0);
  return bytes;
}

extern "C" int mp4x_sort_pairs_i64(const int64_t* keys_in, int64_t* keys_out, const int64_t* idx_in, int64_t* idx_out,
                                   int64_t n, int begin_bit, int end_bit, void* temp, size_t temp_bytes,
                                   void* stream) {
  if (n <= 0) return 0;
  return (int)hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, idx_in, idx_out, (int)n,
                                                 begin_bit, end_bit, (hipStream_t)stream);
}

extern "C" int mp4x_sort_pairs_i32key(const int32_t* keys_in, int32_t* keys_out, const int64_t* idx_in,
                                      int64_t* idx_out, int64_t n, int begin_bit, int end_bit, void* temp,
                                      size_t temp_bytes, void* stream) {
  if (n <= 0) return 0;
  return (int)hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, idx_in, idx_out, (int)n,
                                                 begin_bit, end_bit, (hipStream_t)stream);
}

extern "C" size_t mp4x_rle_temp_bytes(int64_t n) {
  size_t bytes = 0;
  hipcub::CountingInputIterator<int64_t> it(0);
  (void)hipcub::DeviceSelect::Flagged(nullptr, bytes, it, (const int32_t*)nullptr, (int64_t*)nullptr, (int64_t*)nullptr,
                                (int)n, (hipStream_t)0);
  return bytes;
}

extern "C" int mp4x_run_starts(const int64_t* sorted_keys, int64_t n, int64_t* starts, int64_t* nruns_dev,
                               int32_t* flags, void* temp, size_t temp_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (n <= 0) return (int)hipMemsetAsync(nruns_dev, 0, sizeof(int64_t), st);
  int g = grid_for(n, 4);
  hipLaunchKernelGGL(k_head_flags, dim3(g), dim3(kBlock), 0, st, sorted_keys, n, flags);
  hipcub::CountingInputIterator<int64_t> it(0);
  return (int)hipcub::DeviceSelect::Flagged(temp, temp_bytes, it, flags, starts, nruns_dev, (int)n, st);
}

extern "C" int mp4x_segment_reduce_rows(int dtype, int op, const int64_t* sk, const int64_t* perm, const int64_t* starts,
                                        const int64_t* nruns_dev, int64_t n, int64_t max_runs, const void* vals,
                                        int64_t dim, int64_t* out_keys, void* out_vals, int32_t* out_count,
                                        void* stream) {
  if (n <= 0 || max_runs <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case MP4X_F64: return sr_dt<MP4X_F64>(op, sk, perm, starts, nruns_dev, n, max_runs, vals, dim, out_keys, out_vals, out_count, st);
    case MP4X_F32: return sr_dt<MP4X_F32>(op, sk, perm, starts, nruns_dev, n, max_runs, vals, dim, out_keys, out_vals, out_count, st);
    case MP4X_I64: return sr_dt<MP4X_I64>(op, sk, perm, starts, nruns_dev, n, max_runs, vals, dim, out_keys, out_vals, out_count, st);
    case MP4X_I32: return sr_dt<MP4X_I32>(op, sk, perm, starts, nruns_dev, n, max_runs, vals, dim, out_keys, out_vals, out_count, st);
    case MP4X_BF16: return sr_dt<MP4X_BF16>(op, sk, perm, starts, nruns_dev, n, max_runs, vals, dim, out_keys, out_vals, out_count, st);
    case MP4X_F16: return sr_dt<MP4X_F16>(op, sk, perm, starts, nruns_dev, n, max_runs, vals, dim, out_keys, out_vals, out_count, st);
    default: return MP4X_E_UNSUPPORTED;
  }
}
