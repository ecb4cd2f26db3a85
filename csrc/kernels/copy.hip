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

}  // namespace mp4x

using namespace mp4x;

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
