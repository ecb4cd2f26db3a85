// K5h — hash reduce-by-key (gfx950): the opt-in alternative to the sort-based K5 of sparse.hip
// (MP4X_SPARSE_RBK=hash; VERDICT r5 Next #6).
//
// Reference hot loop: the MapReduce deserializer's per-key merge
// (/root/reference/src/main/java/com/fenbi/mp4j/operand/DoubleOperand.java:225-257) and the map
// branch of threadReduce (:458-477) — a HashMap<String, T> probe + combine per received entry.
// Here the keys are 64-bit ids and a map is (keys[n], rows[n][dim]).
//
// The sort path radix-sorts the full 64-bit keys (8 onesweep passes over keys + indices) to find
// the runs.  The hash path finds them with ONE pass over the keys instead, then groups the rows
// by a counting sort over the dense key index:
//
//   memset   table keys <- EMPTY (-1: all 0xFF bytes), slot counts / run counters <- 0
//   insert   one lane per row: splitmix64 hash, linear probing, 64-bit CAS on an EMPTY slot
//            (table >= 2n slots, power of two: an empty slot always exists); the slot's row count
//            += 1 (an int atomic spread over the table) and the row's slot are kept
//   compact  4 slots per lane, one atomic per BLOCK (LDS prefix over the block's lanes): every
//            occupied slot gets a dense run index u and its run length
//   scan     exclusive sum of the run lengths (rocPRIM) -> run starts
//   scatter  one lane per row: position = start[u] + (atomic cursor of u); perm / sorted keys
//   order    one lane per run: the run's row indices sorted ascending (runs up to 64 rows), so
//            rows combine in input (= rank) order — the same values, bit for bit, as the sort path
//   reduce   the sort path's segmented reduce (k_segment_reduce_vec: G lanes per run, 16-byte
//            vectors, two rows in flight), unchanged
//
// Differences from the sort path (why it stays opt-in): the output keys come in table order, not
// ascending, and a run longer than 64 rows combines in scatter order (float SUM / PROD of such a
// key is then not bit-reproducible; integer-valued data and MAX / MIN are exact either way).
// MP4X_FIRST (K8, the first row in rank order) is not served.  Rows whose key equals -1 (the
// table's EMPTY marker) never enter the table: they are counted aside and form one extra run.
#include <rocprim/device/device_scan.hpp>

#include "common.hpp"

extern "C" int mp4x_segment_reduce_rows(int dtype, int op, const int64_t* sk, const int64_t* perm,
                                        const int64_t* starts, const int64_t* nruns_dev, int64_t n, int64_t max_runs,
                                        const void* vals, int64_t dim, int64_t* out_keys, void* out_vals,
                                        int32_t* out_count, void* stream);

namespace mp4x {

namespace {
constexpr unsigned long long kHashEmpty = ~0ull;
constexpr int kCompactPer = 4;             // slots per lane in k_hash_compact (>= 2 blocks per CU at 2n = 400k)
constexpr int kOrderMax = 64;              // longest run whose rows are put in input order

__device__ __forceinline__ uint64_t hash_mix(uint64_t k) {   // splitmix64 finalizer
  k ^= k >> 30;
  k *= 0xbf58476d1ce4e5b9ull;
  k ^= k >> 27;
  k *= 0x94d049bb133111ebull;
  k ^= k >> 31;
  return k;
}

// The side run of rows keyed -1 (the EMPTY marker): its row count and, once compacted, its run.
struct SideRun {
  int32_t rows;
  int32_t u;
};

__global__ __launch_bounds__(kBlock) void k_hash_insert(const int64_t* __restrict__ keys, int64_t n,
                                                        unsigned long long* __restrict__ tkeys,
                                                        int32_t* __restrict__ tcount, uint64_t mask,
                                                        int32_t* __restrict__ row_slot, SideRun* __restrict__ side) {
  const int64_t nthr = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += nthr) {
    const unsigned long long k = (unsigned long long)keys[i];
    if (k == kHashEmpty) {
      atomicAdd(&side->rows, 1);
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
    atomicAdd(&tcount[h], 1);
    row_slot[i] = (int32_t)h;
  }
}

// A tile of kBlock * kCompactPer slots per block (slot = tile + j * kBlock + lane, coalesced);
// the block's occupied slots take consecutive run indices from ONE atomic on the run counter.
__global__ __launch_bounds__(kBlock) void k_hash_compact(const unsigned long long* __restrict__ tkeys,
                                                         const int32_t* __restrict__ tcount, int64_t nslots,
                                                         int32_t* __restrict__ tidx, int32_t* __restrict__ run_len,
                                                         unsigned long long* __restrict__ counter,
                                                         SideRun* __restrict__ side) {
  __shared__ int s_pre[kBlock];
  __shared__ unsigned long long s_base;
  if (blockIdx.x == 0 && threadIdx.x == 0 && side->rows > 0) {     // the side run, if any
    const int32_t u = (int32_t)atomicAdd(counter, 1ull);
    side->u = u;
    run_len[u] = side->rows;
  }
  const int64_t tile = (int64_t)blockIdx.x * kBlock * kCompactPer;
  int mine = 0;
#pragma unroll
  for (int j = 0; j < kCompactPer; ++j) {
    const int64_t h = tile + (int64_t)j * kBlock + threadIdx.x;
    mine += (h < nslots && tkeys[h] != kHashEmpty) ? 1 : 0;
  }
  s_pre[threadIdx.x] = mine;
  __syncthreads();
  for (int off = 1; off < kBlock; off <<= 1) {           // inclusive Hillis-Steele scan in LDS
    const int v = threadIdx.x >= off ? s_pre[threadIdx.x - off] : 0;
    __syncthreads();
    s_pre[threadIdx.x] += v;
    __syncthreads();
  }
  if (threadIdx.x == kBlock - 1) s_base = s_pre[kBlock - 1] ? atomicAdd(counter, (unsigned long long)s_pre[kBlock - 1]) : 0;
  __syncthreads();
  int64_t u = (int64_t)s_base + s_pre[threadIdx.x] - mine;
#pragma unroll
  for (int j = 0; j < kCompactPer; ++j) {
    const int64_t h = tile + (int64_t)j * kBlock + threadIdx.x;
    if (h < nslots && tkeys[h] != kHashEmpty) {
      tidx[h] = (int32_t)u;
      run_len[u] = tcount[h];
      ++u;
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_hash_scatter(const int64_t* __restrict__ keys, int64_t n,
                                                         const int32_t* __restrict__ row_slot,
                                                         const int32_t* __restrict__ tidx,
                                                         const int64_t* __restrict__ starts,
                                                         int32_t* __restrict__ cursor, int64_t* __restrict__ perm,
                                                         int64_t* __restrict__ sk, const SideRun* __restrict__ side) {
  const int64_t nthr = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += nthr) {
    const int32_t s = row_slot[i];
    const int32_t u = s < 0 ? side->u : tidx[s];        // every row lands in a run: n positions in all
    const int64_t pos = starts[u] + atomicAdd(&cursor[u], 1);
    perm[pos] = i;
    sk[pos] = keys[i];
  }
}

// One lane per run: insertion sort of the run's row indices (runs of 2..kOrderMax rows).
__global__ __launch_bounds__(kBlock) void k_hash_order(const int64_t* __restrict__ starts,
                                                       const int32_t* __restrict__ run_len,
                                                       const unsigned long long* __restrict__ m_dev,
                                                       int64_t* __restrict__ perm) {
  const int64_t m = (int64_t)*m_dev;
  const int64_t nthr = (int64_t)gridDim.x * kBlock;
  for (int64_t u = (int64_t)blockIdx.x * kBlock + threadIdx.x; u < m; u += nthr) {
    const int L = run_len[u];
    if (L < 2 || L > kOrderMax) continue;
    int64_t* p = perm + starts[u];
    for (int a = 1; a < L; ++a) {
      const int64_t x = p[a];
      int b = a - 1;
      while (b >= 0 && p[b] > x) {
        p[b + 1] = p[b];
        --b;
      }
      p[b + 1] = x;
    }
  }
}

int64_t table_slots(int64_t n) {
  int64_t t = 1024;
  while (t < 2 * n) t <<= 1;
  return t;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t scan_temp_bytes(int64_t n) {
  size_t b = 0;
  (void)rocprim::exclusive_scan(nullptr, b, (const int32_t*)nullptr, (int64_t*)nullptr, (int64_t)0,
                                (size_t)(n < 1 ? 1 : n), rocprim::plus<int64_t>(), (hipStream_t)0);
  return b;
}

// The scratch layout (every part 256-byte aligned): table keys; then the zero-initialised block
// (slot counts, run lengths, run cursors, the side run: ONE memset); slot -> run, the row -> slot
// map, run starts, perm, sorted keys, scan temp.
struct Layout {
  size_t tkeys, tcount, run_len, cursor, side, zero_end, tidx, row_slot, starts, perm, sk, temp, total, temp_bytes;
  int64_t t;
};

Layout layout(int64_t n) {
  Layout L;
  L.t = table_slots(n);
  size_t o = 0;
  L.tkeys = o;    o += align256((size_t)L.t * 8);
  L.tcount = o;   o += align256((size_t)L.t * 4);
  L.run_len = o;  o += align256((size_t)n * 4);
  L.cursor = o;   o += align256((size_t)n * 4);
  L.side = o;     o += 256;
  L.zero_end = o;
  L.tidx = o;     o += align256((size_t)L.t * 4);
  L.row_slot = o; o += align256((size_t)n * 4);
  L.starts = o;   o += align256((size_t)n * 8);
  L.perm = o;     o += align256((size_t)n * 8);
  L.sk = o;       o += align256((size_t)n * 8);
  L.temp_bytes = scan_temp_bytes(n);
  L.temp = o;     o += align256(L.temp_bytes);
  L.total = o;
  return L;
}
}  // namespace

}  // namespace mp4x

using namespace mp4x;

extern "C" size_t mp4x_hash_rbk_scratch_bytes(int64_t n) { return layout(n < 0 ? 0 : n).total; }

// Does the hash path serve (dtype, op)?  1 / 0.  (Every reduction of the segmented reduce except
// the FIRST rule, which needs the rank order of arbitrarily long runs.)
extern "C" int mp4x_hash_rbk_supported(int dtype, int op) {
  if (op == MP4X_FIRST) return 0;
  const bool isint = dtype == MP4X_I64 || dtype == MP4X_I32 || dtype == MP4X_I16 || dtype == MP4X_I8 ||
                     dtype == MP4X_U8;
  const bool isflt = dtype == MP4X_F64 || dtype == MP4X_F32 || dtype == MP4X_BF16 || dtype == MP4X_F16;
  if (!isint && !isflt) return 0;
  if (op == MP4X_SUM || op == MP4X_MAX || op == MP4X_MIN || op == MP4X_PROD) return 1;
  return isint && (op == MP4X_BAND || op == MP4X_BOR || op == MP4X_BXOR) ? 1 : 0;
}

// keys[n], vals[n][dim] -> out_keys[m] (table order), out_vals[m][dim], out_count[m] (optional);
// m_flag[0] = m, written on the device (stream-ordered; m_flag[1] is zeroed).  out_* must hold
// n rows.
extern "C" int mp4x_hash_reduce_by_key(int dtype, int op, const int64_t* keys, int64_t n, const void* vals, int64_t dim,
                                       void* scratch, size_t scratch_bytes, int64_t* out_keys, void* out_vals,
                                       int32_t* out_count, int64_t* m_flag, void* stream) {
  if (!mp4x_hash_rbk_supported(dtype, op) || n < 0 || dim <= 0 || n >= (1ll << 30)) return MP4X_E_UNSUPPORTED;
  const Layout L = layout(n);
  if (scratch_bytes < L.total || ((uintptr_t)scratch & 255) || ((uintptr_t)m_flag & 7)) return MP4X_E_BADARG;
  hipStream_t st = (hipStream_t)stream;
  char* p = (char*)scratch;
  auto* tkeys = (unsigned long long*)(p + L.tkeys);
  auto* tcount = (int32_t*)(p + L.tcount);
  auto* tidx = (int32_t*)(p + L.tidx);
  auto* row_slot = (int32_t*)(p + L.row_slot);
  auto* run_len = (int32_t*)(p + L.run_len);
  auto* cursor = (int32_t*)(p + L.cursor);
  auto* starts = (int64_t*)(p + L.starts);
  auto* perm = (int64_t*)(p + L.perm);
  auto* sk = (int64_t*)(p + L.sk);
  auto* counter = (unsigned long long*)m_flag;            // m_flag[0]: the run counter IS m
  auto* side = (SideRun*)(p + L.side);
  if (hipError_t e = hipMemsetAsync(tkeys, 0xFF, (size_t)L.t * 8, st)) return (int)e;
  if (hipError_t e = hipMemsetAsync(p + L.tcount, 0, L.zero_end - L.tcount, st)) return (int)e;  // counts .. side
  if (hipError_t e = hipMemsetAsync(m_flag, 0, 16, st)) return (int)e;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_hash_insert, dim3(grid_for(n, 1)), dim3(kBlock), 0, st, keys, n, tkeys, tcount,
                     (uint64_t)(L.t - 1), row_slot, side);
  const int64_t tile = (int64_t)kBlock * kCompactPer;
  hipLaunchKernelGGL(k_hash_compact, dim3((unsigned)((L.t + tile - 1) / tile)), dim3(kBlock), 0, st,
                     (const unsigned long long*)tkeys, (const int32_t*)tcount, L.t, tidx, run_len, counter, side);
  size_t tb = L.temp_bytes;
  if (hipError_t e = rocprim::exclusive_scan(p + L.temp, tb, (const int32_t*)run_len, starts, (int64_t)0, (size_t)n,
                                             rocprim::plus<int64_t>(), st))
    return (int)e;
  hipLaunchKernelGGL(k_hash_scatter, dim3(grid_for(n, 1)), dim3(kBlock), 0, st, keys, n, (const int32_t*)row_slot,
                     (const int32_t*)tidx, (const int64_t*)starts, cursor, perm, sk, (const SideRun*)side);
  hipLaunchKernelGGL(k_hash_order, dim3(grid_for(n, 1)), dim3(kBlock), 0, st, (const int64_t*)starts,
                     (const int32_t*)run_len, (const unsigned long long*)counter, perm);
  if (int e = (int)hipGetLastError()) return e;
  return mp4x_segment_reduce_rows(dtype, op, sk, perm, starts, m_flag, n, n, vals, dim, out_keys, out_vals, out_count,
                                  stream);
}
