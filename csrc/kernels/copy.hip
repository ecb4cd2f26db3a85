// K3 — multi-segment copy and row gather (gfx950).
//
// Reference hot loops: the `System.arraycopy` of segments in threadCopy /
// threadArrayAllCopy / threadMerge (/root/reference/src/main/java/com/fenbi/mp4j/operand/DoubleOperand.java:375,392,413)
// and the per-segment serialisation of ArrayMetaData messages.  On the GPU a ragged
// segment table (allgatherv / gatherv unpacking, padded reduce-scatter staging) becomes ONE
// launch: blockIdx.y selects the segment, the x-dimension grid-strides over its bytes with
// 16-byte vector moves when source, destination and length allow it.
#include "common.hpp"

namespace mp4x {

__global__ __launch_bounds__(kBlock) void k_segment_copy(char* __restrict__ dst, const char* __restrict__ src,
                                                         const int64_t* __restrict__ table, int nseg) {
  const int s = blockIdx.y;
  const int64_t doff = table[s], soff = table[nseg + s], len = table[2 * nseg + s];
  char* d = dst + doff;
  const char* sp = src + soff;
  const int64_t nthr = (int64_t)gridDim.x * kBlock;
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if ((((uintptr_t)d | (uintptr_t)sp) & 15) == 0) {
    const int64_t nv = len >> 4;
    for (int64_t i = tid; i < nv; i += nthr)
      reinterpret_cast<u32x4*>(d)[i] = reinterpret_cast<const u32x4*>(sp)[i];
    for (int64_t i = (nv << 4) + tid; i < len; i += nthr) d[i] = sp[i];
  } else if ((((uintptr_t)d | (uintptr_t)sp) & 3) == 0) {
    const int64_t nv = len >> 2;
    for (int64_t i = tid; i < nv; i += nthr) reinterpret_cast<uint32_t*>(d)[i] = reinterpret_cast<const uint32_t*>(sp)[i];
    for (int64_t i = (nv << 2) + tid; i < len; i += nthr) d[i] = sp[i];
  } else {
    for (int64_t i = tid; i < len; i += nthr) d[i] = sp[i];
  }
}

// Lane groups: a row of V 16-byte vectors is moved by G = min(64, pow2 >= V) lanes, so a
// wave moves 64/G rows at once (256-B rows: 4 rows / wave-instruction, every lane busy).
__global__ __launch_bounds__(kBlock) void k_gather_rows_vec(u32x4* __restrict__ out, const u32x4* __restrict__ in,
                                                            const int64_t* __restrict__ idx, int64_t nrows, int64_t V,
                                                            int G) {
  const int lane = threadIdx.x & 63;
  const int grp = lane / G, sub = lane % G, R = 64 / G;
  const int64_t wave = wave_id();
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t r0 = wave * R; r0 < nrows; r0 += nwaves * R) {
    const int64_t r = r0 + grp;
    if (r >= nrows) continue;
    const u32x4* s = in + idx[r] * V;
    u32x4* d = out + r * V;
    for (int64_t v = sub; v < V; v += G) __builtin_nontemporal_store(s[v], d + v);
  }
}

// One wave64 per row; lanes move 16-byte words (fallback for unaligned / odd-sized rows).
__global__ __launch_bounds__(kBlock) void k_gather_rows(char* __restrict__ out, const char* __restrict__ in,
                                                        const int64_t* __restrict__ idx, int64_t nrows,
                                                        int64_t row_bytes) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = wave_id();
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  const bool vec = ((row_bytes & 15) == 0) && ((((uintptr_t)out | (uintptr_t)in) & 15) == 0);
  for (int64_t r = wave; r < nrows; r += nwaves) {
    const char* s = in + idx[r] * row_bytes;
    char* d = out + r * row_bytes;
    if (vec) {
      const int64_t nv = row_bytes >> 4;
      for (int64_t i = lane; i < nv; i += 64) reinterpret_cast<u32x4*>(d)[i] = reinterpret_cast<const u32x4*>(s)[i];
    } else {
      for (int64_t i = lane; i < row_bytes; i += 64) d[i] = s[i];
    }
  }
}

// Sparse exchanges (mp4x/parallel/sparse.py): the ragged all-to-all-v / all-gather-v of the map
// collectives stage a rank's rows and keys in its IPC buffer as two regions, rows (V 16-byte
// vectors each) and keys as 16-byte {key, 0} vectors, so one copy-plan kernel moves both with
// 16-byte pulls whatever the row counts, and the received rows land contiguous (no unpack pass).
// Stage: one grid-stride over the n * V row vectors then the n key vectors (no index division).
__global__ __launch_bounds__(kBlock) void k_stage_split(const int64_t* __restrict__ keys, const u32x4* __restrict__ vals,
                                                        int64_t n, int64_t V, u32x4* __restrict__ dv,
                                                        u32x4* __restrict__ dk) {
  const int64_t nv = n * V, total = nv + n;
  const int64_t nthr = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total; i += nthr) {
    if (i < nv) {
      dv[i] = vals[i];
    } else {
      const uint64_t k = (uint64_t)keys[i - nv];
      dk[i - nv] = u32x4{(uint32_t)k, (uint32_t)(k >> 32), 0u, 0u};
    }
  }
}

// The received {key, 0} vectors -> int64 keys.
__global__ __launch_bounds__(kBlock) void k_keys_from16(const u32x4* __restrict__ k16, int64_t n,
                                                        int64_t* __restrict__ keys) {
  const int64_t nthr = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += nthr) {
    const u32x4 x = k16[i];
    keys[i] = (int64_t)(((uint64_t)x[1] << 32) | x[0]);
  }
}

}  // namespace mp4x

using namespace mp4x;

// keys[n] (int64) + vals[n][row_bytes] (row_bytes a multiple of 16, 16-byte aligned; NULL when
// row_bytes == 0) -> dst_vals[n][row_bytes] + dst_keys16[n][16].
extern "C" int mp4x_stage_split(const int64_t* keys, const void* vals, int64_t n, int64_t row_bytes, void* dst_vals,
                                void* dst_keys16, void* stream) {
  if (n <= 0) return 0;
  if ((row_bytes & 15) || row_bytes < 0 || ((uintptr_t)keys & 7) || !keys || !dst_keys16 ||
      ((uintptr_t)dst_keys16 & 15) || (row_bytes && (!vals || !dst_vals || (((uintptr_t)vals | (uintptr_t)dst_vals) & 15))))
    return MP4X_E_BADARG;
  const int64_t V = row_bytes / 16;
  hipLaunchKernelGGL(k_stage_split, dim3(grid_for(n * (V + 1), 2)), dim3(kBlock), 0, (hipStream_t)stream, keys,
                     (const u32x4*)vals, n, V, (u32x4*)dst_vals, (u32x4*)dst_keys16);
  return (int)hipGetLastError();
}

extern "C" int mp4x_keys_from16(const void* keys16, int64_t n, int64_t* keys, void* stream) {
  if (n <= 0) return 0;
  if (!keys16 || !keys || ((uintptr_t)keys16 & 15) || ((uintptr_t)keys & 7)) return MP4X_E_BADARG;
  hipLaunchKernelGGL(k_keys_from16, dim3(grid_for(n, 2)), dim3(kBlock), 0, (hipStream_t)stream,
                     (const u32x4*)keys16, n, keys);
  return (int)hipGetLastError();
}

extern "C" int mp4x_segment_copy(void* dst, const void* src, const int64_t* dev_table, int nseg, int64_t max_len,
                                 void* stream) {
  if (nseg <= 0 || max_len <= 0) return 0;
  if (nseg > 65535) return MP4X_E_BADARG;
  int gx = grid_for((max_len + 15) / 16, 2);
  int64_t cap = (kMaxGrid + nseg - 1) / nseg;
  if (gx > cap) gx = (int)(cap < 1 ? 1 : cap);
  hipLaunchKernelGGL(k_segment_copy, dim3(gx, nseg), dim3(kBlock), 0, (hipStream_t)stream, (char*)dst,
                     (const char*)src, dev_table, nseg);
  return (int)hipGetLastError();
}

extern "C" int mp4x_gather_rows(void* out, const void* in, const int64_t* idx, int64_t nrows, int64_t row_bytes,
                                void* stream) {
  if (nrows <= 0 || row_bytes <= 0) return 0;
  if ((row_bytes & 15) == 0 && ((((uintptr_t)out | (uintptr_t)in) & 15) == 0)) {
    const int64_t V = row_bytes / 16;
    int G = 1;
    while (G < V && G < 64) G <<= 1;
    const int64_t waves = (nrows * G + 63) / 64;
    int g = grid_for(waves * 64, 1);
    hipLaunchKernelGGL(k_gather_rows_vec, dim3(g), dim3(kBlock), 0, (hipStream_t)stream, (u32x4*)out,
                       (const u32x4*)in, idx, nrows, V, G);
    return (int)hipGetLastError();
  }
  int g = grid_for(nrows * 64, 1);
  hipLaunchKernelGGL(k_gather_rows, dim3(g), dim3(kBlock), 0, (hipStream_t)stream, (char*)out, (const char*)in, idx,
                     nrows, row_bytes);
  return (int)hipGetLastError();
}
