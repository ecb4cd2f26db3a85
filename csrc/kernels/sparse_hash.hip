// K5h — hash reduce-by-key (gfx950): open addressing + atomic combine, the opt-in alternative to
// the sort-based K5 of sparse.hip (MP4X_SPARSE_RBK=hash; VERDICT r5 Next #6).
//
// Reference hot loop: the MapReduce deserializer's per-key merge
// (/root/reference/src/main/java/com/fenbi/mp4j/operand/DoubleOperand.java:225-257) and the map
// branch of threadReduce (:458-477) — a HashMap<String, T> probe + combine per received entry.
// Here the keys are 64-bit ids and a map is (keys[n], rows[n][dim]):
//
//   memset   the table's keys to EMPTY (-1: all 0xFF bytes, one hipMemsetAsync)
//   insert   one lane per row: splitmix64 hash, linear probing, 64-bit CAS on an EMPTY slot
//            (table >= 2n slots, power of two: an empty slot always exists); the row's slot is kept
//   compact  one lane per slot: occupied slots get a dense index u (one wave-aggregated atomic per
//            wave: ballot + popcount), out_keys[u] / the slot -> u map are written
//   fill     out_rows[0, m) <- the operator's identity (coalesced; m read from device memory)
//   combine  G lanes per row, one 16-byte vector each: device-scope atomic add / max / min of
//            every element into out_rows[u] (global_atomic_add_f32 / _f64 on gfx950, CAS for max /
//            min of floats), counts[u] += 1
//
// Differences from the sort path (why it is opt-in): the output keys come in table order, not
// ascending; float sums are combined in arrival order (exact for integer-valued data, otherwise
// not bit-reproducible run to run); MAX / MIN skip NaN like fmax.  SUM / MAX / MIN of f32 / f64 /
// i32 / i64 only; a key equal to -1 (the EMPTY marker) makes the call report it (flag) and the
// caller falls back to the sort path.
#include "common.hpp"

namespace mp4x {

namespace {
constexpr unsigned long long kHashEmpty = ~0ull;

__device__ __forceinline__ uint64_t hash_mix(uint64_t k) {   // splitmix64 finalizer
  k ^= k >> 30;
  k *= 0xbf58476d1ce4e5b9ull;
  k ^= k >> 27;
  k *= 0x94d049bb133111ebull;
  k ^= k >> 31;
  return k;
}

__global__ __launch_bounds__(kBlock) void k_hash_insert(const int64_t* __restrict__ keys, int64_t n,
                                                        unsigned long long* __restrict__ tkeys, uint64_t mask,
                                                        int32_t* __restrict__ row_slot, int32_t* __restrict__ flag) {
  const int64_t nthr = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += nthr) {
    const unsigned long long k = (unsigned long long)keys[i];
    if (k == kHashEmpty) {
      atomicOr(flag, 1);
      row_slot[i] = -1;
      continue;
    }
    uint64_t h = hash_mix(k) & mask;
    for (;;) {
      unsigned long long cur = __hip_atomic_load(&tkeys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == kHashEmpty) {
        cur = atomicCAS(&tkeys[h], kHashEmpty, k);
        if (cur == kHashEmpty) cur = k;                  // inserted here
      }
      if (cur == k) break;
      h = (h + 1) & mask;
    }
    row_slot[i] = (int32_t)h;
  }
}

// One lane per slot; the grid covers the table exactly once (no grid-stride: the wave-aggregated
// counter needs every lane of a wave in the same iteration).
__global__ __launch_bounds__(kBlock) void k_hash_compact(const unsigned long long* __restrict__ tkeys, int64_t nslots,
                                                         int32_t* __restrict__ tidx, int64_t* __restrict__ out_keys,
                                                         int32_t* __restrict__ out_count,
                                                         unsigned long long* __restrict__ counter) {
  const int64_t h = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const unsigned long long k = h < nslots ? tkeys[h] : kHashEmpty;
  const bool occ = k != kHashEmpty;
  const unsigned long long ballot = __ballot(occ);
  if (ballot == 0) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)ballot) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(counter, (unsigned long long)__popcll(ballot));
  base = __shfl(base, leader);
  if (!occ) return;
  const int64_t u = (int64_t)base + __popcll(ballot & ((1ull << lane) - 1ull));
  tidx[h] = (int32_t)u;
  out_keys[u] = (int64_t)k;
  if (out_count) out_count[u] = 0;
}

template <typename S>
__global__ __launch_bounds__(kBlock) void k_hash_fill(S* __restrict__ out, const unsigned long long* __restrict__ m_dev,
                                                      int64_t dim, S ident) {
  const int64_t total = (int64_t)(*m_dev) * dim;
  const int64_t nthr = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total; i += nthr) out[i] = ident;
}

template <typename S, int OP>
__device__ __forceinline__ void atomic_combine(S* p, S v) {
  if constexpr (OP == MP4X_SUM) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (OP == MP4X_MAX) {
    __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// G lanes per row (64 / G rows per wave and step), lane `sub` combines 16-byte vector v of the row
// (W elements); rows whose byte size is not a multiple of 16 use one lane per element (G = 64,
// W = 1 through the scalar loop).
template <typename S, int OP>
__global__ __launch_bounds__(kBlock) void k_hash_combine(const S* __restrict__ vals, int64_t n, int64_t dim,
                                                         const int32_t* __restrict__ row_slot,
                                                         const int32_t* __restrict__ tidx, S* __restrict__ out,
                                                         int32_t* __restrict__ out_count, int G) {
  constexpr int W = 16 / sizeof(S);
  const int lane = threadIdx.x & 63;
  const int grp = lane / G, sub = lane % G, R = 64 / G;
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  const bool vec = (dim * (int64_t)sizeof(S)) % 16 == 0;
  const int64_t V = vec ? dim / W : dim;
  for (int64_t r0 = wave_id() * R; r0 < n; r0 += nwaves * R) {
    const int64_t i = r0 + grp;
    if (i >= n) continue;
    const int32_t s = row_slot[i];
    if (s < 0) continue;
    const int64_t u = tidx[s];
    if (sub == 0 && out_count) atomicAdd(&out_count[u], 1);
    if (vec) {
      const u32x4* src = reinterpret_cast<const u32x4*>(vals + i * dim);
      S* dst = out + u * dim;
      for (int64_t v = sub; v < V; v += G) {
        u32x4 t = src[v];
        S x[W];
        __builtin_memcpy(x, &t, 16);
#pragma unroll
        for (int q = 0; q < W; ++q) atomic_combine<S, OP>(dst + v * W + q, x[q]);
      }
    } else {
      for (int64_t d = sub; d < dim; d += G) atomic_combine<S, OP>(out + u * dim + d, vals[i * dim + d]);
    }
  }
}

template <typename S> S ident_of(int op) {
  if (op == MP4X_SUM) return S(0);
  if constexpr (sizeof(S) == 8 && S(0.5) == S(0)) {   // int64
    return op == MP4X_MAX ? (S)INT64_MIN : (S)INT64_MAX;
  } else if constexpr (S(0.5) == S(0)) {              // int32
    return op == MP4X_MAX ? (S)INT32_MIN : (S)INT32_MAX;
  } else {
    return op == MP4X_MAX ? -__builtin_huge_val() : __builtin_huge_val();
  }
}

template <typename S>
int launch_hash_combine(int op, const void* vals, int64_t n, int64_t dim, const int32_t* row_slot, const int32_t* tidx,
                        void* out, int32_t* count, const unsigned long long* m_dev, hipStream_t st) {
  const S ident = ident_of<S>(op);
  hipLaunchKernelGGL(k_hash_fill<S>, dim3(grid_for(n * dim, 4)), dim3(kBlock), 0, st, (S*)out, m_dev, dim, ident);
  const int64_t V = (dim * (int64_t)sizeof(S)) % 16 == 0 ? dim * (int64_t)sizeof(S) / 16 : 64;
  int G = 1;
  while (G < V && G < 64) G <<= 1;
  const int g = grid_for((n * G + 63) / 64 * 64, 1);
  const S* v = (const S*)vals;
  switch (op) {
    case MP4X_SUM: hipLaunchKernelGGL((k_hash_combine<S, MP4X_SUM>), dim3(g), dim3(kBlock), 0, st, v, n, dim, row_slot,
                                      tidx, (S*)out, count, G); break;
    case MP4X_MAX: hipLaunchKernelGGL((k_hash_combine<S, MP4X_MAX>), dim3(g), dim3(kBlock), 0, st, v, n, dim, row_slot,
                                      tidx, (S*)out, count, G); break;
    case MP4X_MIN: hipLaunchKernelGGL((k_hash_combine<S, MP4X_MIN>), dim3(g), dim3(kBlock), 0, st, v, n, dim, row_slot,
                                      tidx, (S*)out, count, G); break;
    default: return MP4X_E_UNSUPPORTED;
  }
  return (int)hipGetLastError();
}

int64_t table_slots(int64_t n) {
  int64_t t = 1024;
  while (t < 2 * n) t <<= 1;
  return t;
}
}  // namespace

}  // namespace mp4x

using namespace mp4x;

// Scratch of mp4x_hash_reduce_by_key for n rows: the table (8 B keys + 4 B indices per slot),
// the row -> slot map, the counter and the EMPTY-key flag.
extern "C" size_t mp4x_hash_rbk_scratch_bytes(int64_t n) {
  const int64_t t = table_slots(n);
  return (size_t)(t * 8 + t * 4 + ((n * 4 + 15) / 16) * 16 + 16);
}

// Does the hash path serve (dtype, op)?  1 / 0.
extern "C" int mp4x_hash_rbk_supported(int dtype, int op) {
  const bool dt = dtype == MP4X_F32 || dtype == MP4X_F64 || dtype == MP4X_I32 || dtype == MP4X_I64;
  return dt && (op == MP4X_SUM || op == MP4X_MAX || op == MP4X_MIN) ? 1 : 0;
}

// keys[n], vals[n][dim] -> out_keys[m] (table order), out_vals[m][dim], out_count[m] (optional);
// m_flag[0] = m and m_flag[1] = 1 when a key equal to -1 was seen (result invalid: use the sort
// path), both written on the device (stream-ordered).  out_* must hold n rows.
extern "C" int mp4x_hash_reduce_by_key(int dtype, int op, const int64_t* keys, int64_t n, const void* vals, int64_t dim,
                                       void* scratch, size_t scratch_bytes, int64_t* out_keys, void* out_vals,
                                       int32_t* out_count, int64_t* m_flag, void* stream) {
  if (!mp4x_hash_rbk_supported(dtype, op) || n < 0 || dim <= 0 || n >= (1ll << 30)) return MP4X_E_UNSUPPORTED;
  if (scratch_bytes < mp4x_hash_rbk_scratch_bytes(n) || ((uintptr_t)scratch & 15) || ((uintptr_t)m_flag & 7))
    return MP4X_E_BADARG;
  hipStream_t st = (hipStream_t)stream;
  const int64_t t = table_slots(n);
  char* p = (char*)scratch;
  unsigned long long* tkeys = (unsigned long long*)p;
  int32_t* tidx = (int32_t*)(p + t * 8);
  int32_t* row_slot = (int32_t*)(p + t * 12);
  unsigned long long* counter = (unsigned long long*)m_flag;      // m_flag[0]: the counter IS m
  int32_t* flag = (int32_t*)(m_flag + 1);
  if (hipError_t e = hipMemsetAsync(tkeys, 0xFF, (size_t)t * 8, st)) return (int)e;
  if (hipError_t e = hipMemsetAsync(m_flag, 0, 16, st)) return (int)e;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_hash_insert, dim3(grid_for(n, 1)), dim3(kBlock), 0, st, keys, n, tkeys, (uint64_t)(t - 1),
                     row_slot, flag);
  hipLaunchKernelGGL(k_hash_compact, dim3((unsigned)((t + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                     (const unsigned long long*)tkeys, t, tidx, out_keys, out_count, counter);
  switch (dtype) {
    case MP4X_F32: return launch_hash_combine<float>(op, vals, n, dim, row_slot, tidx, out_vals, out_count, counter, st);
    case MP4X_F64: return launch_hash_combine<double>(op, vals, n, dim, row_slot, tidx, out_vals, out_count, counter, st);
    case MP4X_I32: return launch_hash_combine<int32_t>(op, vals, n, dim, row_slot, tidx, out_vals, out_count, counter, st);
    case MP4X_I64: return launch_hash_combine<int64_t>(op, vals, n, dim, row_slot, tidx, out_vals, out_count, counter,
                                                       st);
    default: return MP4X_E_UNSUPPORTED;
  }
}
