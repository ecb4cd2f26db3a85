// K4 / K5 / K7 / K8 — sparse Map<String, T> collectives on the GPU (gfx950).
//
// Reference hot loops: hash partitioning of map keys (ProcessCommSlave.java:2059-2072), the
// MapReduce deserializer's per-key merge (J/operand/DoubleOperand.java:225-257) and the
// Set/List specials built on it (ProcessCommSlave.java:1583-1720).  On the device, string
// keys travel as 64-bit ids (host dictionary) and a map is a (keys[n], vals[n, dim]) pair:
//
//   K4  owner + histogram:  dest = id % p, per-block LDS histogram, one atomic per bucket;
//       the stable radix sort by dest (rocPRIM) then gives the all-to-all send layout.
//   K5  reduce-by-key:      stable radix sort by id (rank order preserved inside a key),
//       head flags + DeviceSelect give run starts, then one wave per run reduces its rows
//       (lanes over `dim`) in run order => deterministic, no float atomics.
//   K7  set union / intersection / concat reuse the same runs (count == p for intersection).
//   K8  map merge (gather / allgather map): the same runs with OP = FIRST keep the first
//       row of every key in rank order (dedupe-by-key).
// rocPRIM directly (64-bit sizes everywhere: no (int) narrowing of element counts)
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

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
  const int64_t wave = wave_id();
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
      if constexpr (OP != MP4X_FIRST)
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
  const int64_t wave = wave_id();
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t u0 = wave * R; u0 < nruns; u0 += nwaves * R) {
    const int64_t u = u0 + grp;
    if (u >= nruns) continue;
    const int64_t s = starts[u];
    const int64_t e = (u + 1 < nruns) ? starts[u + 1] : n;
    MP4X_DASSERT(s >= 0 && s < e && e <= n);
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
      int64_t j = (OP == MP4X_FIRST) ? e : s + 1;   // FIRST (K8 dedupe): the run's first row only
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
    case MP4X_FIRST: return launch_sr<DT, MP4X_FIRST>(sk, perm, starts, nr, n, mr, vals, dim, ok, ov, oc, st);
    default: return MP4X_E_UNSUPPORTED;
  }
}


// K4b — fused owner partition + pack (LDS multisplit).  Replaces owner -> radix sort by
// owner -> two row gathers with three passes over the keys and ONE pass over the rows:
//   k_pack_hist     per-256-key tile LDS histogram -> hist[d * nblk + tile] (no global atomics)
//   DeviceScan      exclusive sum over (owner-major, tile-minor) -> every (owner, tile) base
//   k_pack_scatter  per wave, a ballot "match" loop ranks lanes that share an owner (stable:
//                   lane order), per-wave counts go through LDS for the block prefix; keys
//                   scatter directly, destination row offsets are staged in LDS and the rows
//                   then move with lane groups (contiguous 16-B loads, nontemporal stores).
// The result is exactly the stable sort by owner (same layout as the radix-sort path) with
// no contended atomics: deterministic run to run.
constexpr int kPackMaxP = 2048;

__device__ __forceinline__ int owner_of(int64_t k, int p) { return (int)((uint64_t)k % (uint64_t)p); }

// bmin / bmax (optional): the tile's smallest / largest key, for the key range the count
// exchange carries (k_pack_scatter block 0 reduces them).
__global__ __launch_bounds__(kBlock) void k_pack_hist(const int64_t* __restrict__ keys, int64_t n, int p, int64_t nblk,
                                                      int64_t* __restrict__ hist, int64_t* __restrict__ bmin,
                                                      int64_t* __restrict__ bmax) {
  extern __shared__ __attribute__((aligned(16))) int32_t lh[];
  __shared__ int64_t wmin[kBlock / 64], wmax[kBlock / 64];
  for (int i = threadIdx.x; i < p; i += kBlock) lh[i] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t k = i < n ? keys[i] : 0;
  if (i < n) atomicAdd(&lh[owner_of(k, p)], 1);
  if (bmin) {
    int64_t lo = i < n ? k : INT64_MAX, hi = i < n ? k : INT64_MIN;
    for (int o = 32; o > 0; o >>= 1) {
      const int64_t a = __shfl_xor(lo, o, 64), b = __shfl_xor(hi, o, 64);
      lo = a < lo ? a : lo;
      hi = b > hi ? b : hi;
    }
    if ((threadIdx.x & 63) == 0) {
      wmin[threadIdx.x >> 6] = lo;
      wmax[threadIdx.x >> 6] = hi;
    }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < p; d += kBlock) hist[(int64_t)d * nblk + blockIdx.x] = lh[d];
  if (bmin && threadIdx.x == 0) {
    int64_t lo = wmin[0], hi = wmax[0];
    for (int q = 1; q < kBlock / 64; ++q) {
      lo = wmin[q] < lo ? wmin[q] : lo;
      hi = wmax[q] > hi ? wmax[q] : hi;
    }
    bmin[blockIdx.x] = lo;
    bmax[blockIdx.x] = hi;
  }
}

// One block: counts[q] = rows for owner q (from the scanned (owner, tile) bases) and, when asked,
// range = the smallest / largest key (every tile's min / max from k_pack_hist).
__global__ __launch_bounds__(kBlock) void k_pack_counts(const int64_t* __restrict__ off,
                                                        const int64_t* __restrict__ hist, int p, int64_t nblk,
                                                        int64_t* __restrict__ counts,
                                                        const int64_t* __restrict__ bmin,
                                                        const int64_t* __restrict__ bmax,
                                                        int64_t* __restrict__ range) {
  __shared__ int64_t rmin[kBlock / 64], rmax[kBlock / 64];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int64_t last = (int64_t)p * nblk - 1;
  for (int q = tid; q < p; q += kBlock) {
    const int64_t end = (q + 1 < p) ? off[(int64_t)(q + 1) * nblk] : off[last] + hist[last];
    counts[q] = end - off[(int64_t)q * nblk];
  }
  if (!range) return;
  int64_t lo = INT64_MAX, hi = INT64_MIN;
  for (int64_t q = tid; q < nblk; q += kBlock) {
    lo = bmin[q] < lo ? bmin[q] : lo;
    hi = bmax[q] > hi ? bmax[q] : hi;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t a = __shfl_xor(lo, o, 64), c = __shfl_xor(hi, o, 64);
    lo = a < lo ? a : lo;
    hi = c > hi ? c : hi;
  }
  if (lane == 0) {
    rmin[w] = lo;
    rmax[w] = hi;
  }
  __syncthreads();
  if (tid == 0) {
    for (int q = 1; q < kBlock / 64; ++q) {
      lo = rmin[q] < lo ? rmin[q] : lo;
      hi = rmax[q] > hi ? rmax[q] : hi;
    }
    range[0] = lo;
    range[1] = hi;
  }
}

__global__ __launch_bounds__(kBlock) void k_pack_scatter(const int64_t* __restrict__ keys,
                                                         const u32x4* __restrict__ vals, int64_t n, int64_t V,
                                                         int G, int p, int64_t nblk,
                                                         const int64_t* __restrict__ off,
                                                         int64_t* __restrict__ out_keys, int key_stride,
                                                         u32x4* __restrict__ out_vals,
                                                         int64_t* __restrict__ out_perm) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int32_t* wcnt = reinterpret_cast<int32_t*>(smem);                         // [4][p]
  int64_t* pos = reinterpret_cast<int64_t*>(smem + ((4 * p * 4 + 15) & ~15));  // [kBlock]
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int64_t b = blockIdx.x, t0 = b * kBlock, i = t0 + tid;
  const bool valid = i < n;
  for (int j = tid; j < 4 * p; j += kBlock) wcnt[j] = 0;
  __syncthreads();
  const int64_t k = valid ? keys[i] : 0;
  const int d = valid ? owner_of(k, p) : -1;
  uint64_t active = __ballot(valid);
  int rank = 0;
  while (active) {                       // wave-uniform: one trip per distinct owner in the wave
    const int leader = __ffsll((unsigned long long)active) - 1;
    const int ld = __shfl(d, leader);
    const uint64_t m = __ballot(d == ld) & active;
    if (d == ld) rank = __popcll(m & ((1ull << lane) - 1));
    if (lane == leader) wcnt[w * p + ld] = __popcll(m);
    active &= ~m;
  }
  __syncthreads();
  if (valid) {
    int inb = rank;
    for (int q = 0; q < w; ++q) inb += wcnt[q * p + d];
    const int64_t ps = off[(int64_t)d * nblk + b] + inb;
    MP4X_DASSERT(ps >= 0 && ps < n);
    out_keys[ps * key_stride] = k;       // stride 2: the key half of a 16-byte {key, -} vector
    if (out_perm) out_perm[ps] = i;
    pos[tid] = ps;
  }
  if (!vals) return;
  __syncthreads();
  const int64_t rows = (n - t0) < kBlock ? (n - t0) : kBlock;
  const int grp = lane / G, sub = lane % G, R = 64 / G;
  constexpr int UNR = 4;
  for (int r0 = w * R + grp; r0 < rows; r0 += 4 * R * UNR) {
    for (int64_t v = sub; v < V; v += G) {
      u32x4 x[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int r = r0 + u * 4 * R;
        if (r < rows) x[u] = __builtin_nontemporal_load(vals + (t0 + r) * V + v);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int r = r0 + u * 4 * R;
        if (r < rows) __builtin_nontemporal_store(x[u], out_vals + pos[r] * V + v);
      }
    }
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

// rocPRIM's dispatch sorts up to 1 M items by block sort + merge passes (log2 of the block count,
// whatever the key width); onesweep runs one pass per 8 key bits.  A sort over few bits (dense
// ids, the key range the sparse count exchange carries) can force onesweep: MergeSortLimit = 0.
using OnesweepSort = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                rocprim::default_config, 0>;

extern "C" size_t mp4x_sort_pairs_temp_bytes(int64_t n, int key_is_i32) {
  size_t bytes = 0, ob = 0;
  const size_t sz = (size_t)(n < 1 ? 1 : n);
  if (key_is_i32) {
    (void)rocprim::radix_sort_pairs(nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr,
                                    (const int64_t*)nullptr, (int64_t*)nullptr, sz, 0, 32, (hipStream_t)0);
  } else {
    (void)rocprim::radix_sort_pairs(nullptr, bytes, (const int64_t*)nullptr, (int64_t*)nullptr,
                                    (const int64_t*)nullptr, (int64_t*)nullptr, sz, 0, 64, (hipStream_t)0);
    (void)rocprim::radix_sort_pairs<OnesweepSort>(nullptr, ob, (const int64_t*)nullptr, (int64_t*)nullptr,
                                                  (const int64_t*)nullptr, (int64_t*)nullptr, sz, 0, 64,
                                                  (hipStream_t)0);
  }
  return bytes > ob ? bytes : ob;
}

// algo: 0 = rocPRIM's own choice, 1 = onesweep (one pass per 8 bits of [begin_bit, end_bit)).
extern "C" int mp4x_sort_pairs_i64_ex(const int64_t* keys_in, int64_t* keys_out, const int64_t* idx_in,
                                      int64_t* idx_out, int64_t n, int begin_bit, int end_bit, int algo, void* temp,
                                      size_t temp_bytes, void* stream) {
  if (n <= 0) return 0;
  if (algo == 1)
    return (int)rocprim::radix_sort_pairs<OnesweepSort>(temp, temp_bytes, keys_in, keys_out, idx_in, idx_out,
                                                        (size_t)n, (unsigned)begin_bit, (unsigned)end_bit,
                                                        (hipStream_t)stream);
  return (int)rocprim::radix_sort_pairs(temp, temp_bytes, keys_in, keys_out, idx_in, idx_out, (size_t)n,
                                        (unsigned)begin_bit, (unsigned)end_bit, (hipStream_t)stream);
}

extern "C" int mp4x_sort_pairs_i64(const int64_t* keys_in, int64_t* keys_out, const int64_t* idx_in, int64_t* idx_out,
                                   int64_t n, int begin_bit, int end_bit, void* temp, size_t temp_bytes,
                                   void* stream) {
  return mp4x_sort_pairs_i64_ex(keys_in, keys_out, idx_in, idx_out, n, begin_bit, end_bit, 0, temp, temp_bytes, stream);
}

extern "C" int mp4x_sort_pairs_i32key(const int32_t* keys_in, int32_t* keys_out, const int64_t* idx_in,
                                      int64_t* idx_out, int64_t n, int begin_bit, int end_bit, void* temp,
                                      size_t temp_bytes, void* stream) {
  if (n <= 0) return 0;
  return (int)rocprim::radix_sort_pairs(temp, temp_bytes, keys_in, keys_out, idx_in, idx_out, (size_t)n,
                                        (unsigned)begin_bit, (unsigned)end_bit, (hipStream_t)stream);
}

extern "C" size_t mp4x_rle_temp_bytes(int64_t n) {
  size_t bytes = 0;
  rocprim::counting_iterator<int64_t> it(0);
  (void)rocprim::select(nullptr, bytes, it, (const int32_t*)nullptr, (int64_t*)nullptr, (int64_t*)nullptr,
                        (size_t)(n < 1 ? 1 : n), (hipStream_t)0);
  return bytes;
}

extern "C" int mp4x_run_starts(const int64_t* sorted_keys, int64_t n, int64_t* starts, int64_t* nruns_dev,
                               int32_t* flags, void* temp, size_t temp_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (n <= 0) return (int)hipMemsetAsync(nruns_dev, 0, sizeof(int64_t), st);
  int g = grid_for(n, 4);
  hipLaunchKernelGGL(k_head_flags, dim3(g), dim3(kBlock), 0, st, sorted_keys, n, flags);
  rocprim::counting_iterator<int64_t> it(0);
  return (int)rocprim::select(temp, temp_bytes, it, flags, starts, nruns_dev, (size_t)n, st);
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
    case MP4X_I16: return sr_dt<MP4X_I16>(op, sk, perm, starts, nruns_dev, n, max_runs, vals, dim, out_keys, out_vals, out_count, st);
    case MP4X_I8: return sr_dt<MP4X_I8>(op, sk, perm, starts, nruns_dev, n, max_runs, vals, dim, out_keys, out_vals, out_count, st);
    case MP4X_U8: return sr_dt<MP4X_U8>(op, sk, perm, starts, nruns_dev, n, max_runs, vals, dim, out_keys, out_vals, out_count, st);
    default: return MP4X_E_UNSUPPORTED;
  }
}

static size_t pack_align(size_t x) { return (x + 255) & ~(size_t)255; }

extern "C" size_t mp4x_partition_pack_scratch_bytes(int64_t n, int p) {
  const int64_t nblk = (n + kBlock - 1) / kBlock;
  const int64_t m = (int64_t)p * (nblk < 1 ? 1 : nblk);
  size_t cub_bytes = 0;
  (void)rocprim::exclusive_scan(nullptr, cub_bytes, (const int64_t*)nullptr, (int64_t*)nullptr, (int64_t)0, (size_t)m,
                                rocprim::plus<int64_t>(), (hipStream_t)0);
  return 2 * pack_align(m * sizeof(int64_t)) + 2 * pack_align((nblk < 1 ? 1 : nblk) * sizeof(int64_t)) +
         pack_align(cub_bytes);
}

namespace {
struct PackScratch {
  int64_t nblk, m;
  int64_t *hist, *off, *bmin, *bmax;
  void* temp;
  size_t temp_bytes;
};

PackScratch pack_scratch(void* scratch, size_t scratch_bytes, int64_t n, int p) {
  PackScratch S;
  S.nblk = (n + kBlock - 1) / kBlock;
  S.m = (int64_t)p * S.nblk;
  char* sc = (char*)scratch;
  S.hist = (int64_t*)sc;
  S.off = (int64_t*)(sc + pack_align(S.m * sizeof(int64_t)));
  S.bmin = (int64_t*)(sc + 2 * pack_align(S.m * sizeof(int64_t)));
  S.bmax = (int64_t*)((char*)S.bmin + pack_align(S.nblk * sizeof(int64_t)));
  const size_t head = 2 * pack_align(S.m * sizeof(int64_t)) + 2 * pack_align(S.nblk * sizeof(int64_t));
  S.temp = sc + head;
  S.temp_bytes = scratch_bytes - head;
  return S;
}
}  // namespace

// K4b in two halves, so a caller can exchange the counts before it picks where the packed rows
// go (the sparse owner exchange scatters them straight into its IPC staging buffer).
// Count: per-tile owner histogram + scan -> counts[p] (rows per owner) and range[2] (optional: the
// smallest and largest key; 0, 0 when n == 0).  The scratch then holds the scan for the scatter.
extern "C" int mp4x_partition_pack_count(const int64_t* keys, int64_t n, int p, int64_t* counts, int64_t* range,
                                         void* scratch, size_t scratch_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (p < 1 || p > kPackMaxP || !counts) return MP4X_E_BADARG;
  if (n <= 0) {
    if (hipError_t e = hipMemsetAsync(counts, 0, p * sizeof(int64_t), st)) return (int)e;
    return range ? (int)hipMemsetAsync(range, 0, 2 * sizeof(int64_t), st) : 0;
  }
  if (n > INT32_MAX / 2) return MP4X_E_BADARG;
  if (scratch_bytes < mp4x_partition_pack_scratch_bytes(n, p)) return MP4X_E_BADARG;
  PackScratch S = pack_scratch(scratch, scratch_bytes, n, p);
  hipLaunchKernelGGL(k_pack_hist, dim3(S.nblk), dim3(kBlock), p * sizeof(int32_t), st, keys, n, p, S.nblk, S.hist,
                     range ? S.bmin : nullptr, range ? S.bmax : nullptr);
  int e = (int)hipGetLastError();
  if (e) return e;
  e = (int)rocprim::exclusive_scan(S.temp, S.temp_bytes, S.hist, S.off, (int64_t)0, (size_t)S.m,
                                   rocprim::plus<int64_t>(), st);
  if (e) return e;
  hipLaunchKernelGGL(k_pack_counts, dim3(1), dim3(kBlock), 0, st, (const int64_t*)S.off, (const int64_t*)S.hist, p,
                     S.nblk, counts, (const int64_t*)S.bmin, (const int64_t*)S.bmax, range);
  return (int)hipGetLastError();
}

// Scatter (after mp4x_partition_pack_count on the same keys, p and scratch): out_keys (key_stride
// 1: int64[n]; 2: the key half of n 16-byte vectors) / out_vals (rows of row_bytes, 16-B aligned;
// vals may be NULL) in owner-major, input-stable order; out_perm (optional) = source row of
// every slot.
extern "C" int mp4x_partition_pack_scatter(const int64_t* keys, const void* vals, int64_t n, int64_t row_bytes,
                                           int p, int64_t* out_keys, int key_stride, void* out_vals,
                                           int64_t* out_perm, void* scratch, size_t scratch_bytes, void* stream) {
  if (n <= 0) return 0;
  if (p < 1 || p > kPackMaxP || n > INT32_MAX / 2 || (key_stride != 1 && key_stride != 2)) return MP4X_E_BADARG;
  if (vals && ((row_bytes & 15) || ((((uintptr_t)vals | (uintptr_t)out_vals) & 15)))) return MP4X_E_BADARG;
  if (scratch_bytes < mp4x_partition_pack_scratch_bytes(n, p)) return MP4X_E_BADARG;
  const PackScratch S = pack_scratch(scratch, scratch_bytes, n, p);
  const int64_t V = vals ? row_bytes / 16 : 0;
  int G = 1;
  while (G < V && G < 64) G <<= 1;
  const size_t lds = ((4 * p * 4 + 15) & ~15) + kBlock * sizeof(int64_t);
  hipLaunchKernelGGL(k_pack_scatter, dim3(S.nblk), dim3(kBlock), lds, (hipStream_t)stream, keys, (const u32x4*)vals,
                     n, V, G, p, S.nblk, (const int64_t*)S.off, out_keys, key_stride, (u32x4*)out_vals, out_perm);
  return (int)hipGetLastError();
}

// Both halves: keys[n] (+ rows vals[n][row_bytes]) -> stable-by-owner layout out_keys / out_vals,
// optional out_perm, counts[p] and range[2] (optional).
extern "C" int mp4x_partition_pack(const int64_t* keys, const void* vals, int64_t n, int64_t row_bytes, int p,
                                   int64_t* out_keys, void* out_vals, int64_t* out_perm, int64_t* counts,
                                   int64_t* range, void* scratch, size_t scratch_bytes, void* stream) {
  if (vals && ((row_bytes & 15) || ((((uintptr_t)vals | (uintptr_t)out_vals) & 15)))) return MP4X_E_BADARG;
  if (int e = mp4x_partition_pack_count(keys, n, p, counts, range, scratch, scratch_bytes, stream)) return e;
  return mp4x_partition_pack_scatter(keys, vals, n, row_bytes, p, out_keys, 1, out_vals, out_perm, scratch,
                                     scratch_bytes, stream);
}
