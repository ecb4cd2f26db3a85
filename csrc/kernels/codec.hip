// K6 — block-scaled fp8 (OCP e4m3, gfx950-native) wire codec for compressed collectives.
//
// The reference's only codec is lossless Deflate around every Kryo stream
// (/root/reference/src/main/java/com/fenbi/mp4j/operand/DoubleOperand.java:267-277).  Over
// xGMI a CPU-class entropy coder cannot keep up with the link, so the device path offers a
// lossy 4x (vs f32) codec whose kernels run far above link speed:
//
//   quant:          one wave64 per 256-element block, 4 elements per lane, wave-wide amax
//                   by shfl_xor, scale = amax / 448, v_cvt_pk_fp8_f32 packs 4 values per lane
//                   into one dword (a 256-B store per wave);
//   dequant_reduce: one wave per block, NIN fp8 chunks dequantised and summed in f32
//                   registers (the two-shot compressed allreduce's reduce step), optionally
//                   re-quantised in the same pass for the all-gather leg.
#include <hipcub/hipcub.hpp>

#include "fp8.hpp"

namespace mp4x {

// One wave per quant block; QU consecutive blocks per wave iteration so each lane keeps QU
// 16-byte loads in flight before the first amax reduction.
constexpr int QU = 4;

template <int DT>
__global__ __launch_bounds__(kBlock) void k_quant(const void* __restrict__ in, int64_t n, uint32_t* __restrict__ q,
                                                  float* __restrict__ scales) {
  const int lane = threadIdx.x & 63;
  const int64_t nblk = (n + kQBlock - 1) / kQBlock;
  const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t b0 = wave * QU; b0 < nblk; b0 += nwaves * QU) {
    float x[QU][4];
#pragma unroll
    for (int u = 0; u < QU; ++u)
      if (b0 + u < nblk) load4<DT>(in, (b0 + u) * kQBlock + lane * 4, n, x[u]);
#pragma unroll
    for (int u = 0; u < QU; ++u)
      if (b0 + u < nblk) quant_block(x[u], q, scales, b0 + u, lane);
  }
}

template <int NIN> struct QIn { const uint32_t* q[NIN]; const float* s[NIN]; };

template <int DT, int NIN>
__global__ __launch_bounds__(kBlock) void k_dequant_reduce(void* __restrict__ out, QIn<NIN> in, int64_t n,
                                                           int accumulate, uint32_t* __restrict__ q_out,
                                                           float* __restrict__ s_out) {
  const int lane = threadIdx.x & 63;
  const int64_t nblk = (n + kQBlock - 1) / kQBlock;
  const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t b = wave; b < nblk; b += nwaves) {
    const int64_t e = b * kQBlock + lane * 4;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (accumulate && out) load4<DT>(out, e, n, acc);
    uint32_t w[NIN];
    float s[NIN];
#pragma unroll
    for (int k = 0; k < NIN; ++k) {   // issue every load first: NIN independent requests in flight
      w[k] = __builtin_nontemporal_load(in.q[k] + b * 64 + lane);
      s[k] = in.s[k][b];
    }
#pragma unroll
    for (int k = 0; k < NIN; ++k) fp8_fma_acc(w[k], s[k], acc);
    if (out) store4<DT>(out, e, n, acc);
    if (q_out) quant_block(acc, q_out, s_out, b, lane);
  }
}

template <int DT>
static int launch_quant(const void* in, int64_t n, uint32_t* q, float* s, hipStream_t st) {
  int64_t nblk = (n + kQBlock - 1) / kQBlock;
  int g = grid_for(nblk * 64, 1);
  hipLaunchKernelGGL(k_quant<DT>, dim3(g), dim3(kBlock), 0, st, in, n, q, s);
  return (int)hipGetLastError();
}

template <int DT, int NIN>
static int launch_dr(void* out, const uint8_t* const* qs, const float* const* ss, int64_t n, int acc, uint8_t* qo,
                     float* so, hipStream_t st) {
  QIn<NIN> in;
  for (int k = 0; k < NIN; ++k) {
    in.q[k] = reinterpret_cast<const uint32_t*>(qs[k]);
    in.s[k] = ss[k];
  }
  int64_t nblk = (n + kQBlock - 1) / kQBlock;
  int g = grid_for(nblk * 64, 1);
  hipLaunchKernelGGL((k_dequant_reduce<DT, NIN>), dim3(g), dim3(kBlock), 0, st, out, in, n, acc,
                     reinterpret_cast<uint32_t*>(qo), so);
  return (int)hipGetLastError();
}

template <int DT>
static int dr_dt(void* out, const uint8_t* const* qs, const float* const* ss, int nin, int64_t n, int acc,
                 uint8_t* qo, float* so, hipStream_t st) {
  switch (nin) {
    case 1: return launch_dr<DT, 1>(out, qs, ss, n, acc, qo, so, st);
    case 2: return launch_dr<DT, 2>(out, qs, ss, n, acc, qo, so, st);
    case 3: return launch_dr<DT, 3>(out, qs, ss, n, acc, qo, so, st);
    case 4: return launch_dr<DT, 4>(out, qs, ss, n, acc, qo, so, st);
    case 5: return launch_dr<DT, 5>(out, qs, ss, n, acc, qo, so, st);
    case 6: return launch_dr<DT, 6>(out, qs, ss, n, acc, qo, so, st);
    case 7: return launch_dr<DT, 7>(out, qs, ss, n, acc, qo, so, st);
    case 8: return launch_dr<DT, 8>(out, qs, ss, n, acc, qo, so, st);
    default: return MP4X_E_BADARG;
  }
}


// ---------------------------------------------------------------- K6b lossless zero suppression
// The reference's compress=true is lossless Deflate.  For device tensors the lossless codec is
// zero suppression, the case where it pays on accelerator data (sparse / masked gradients,
// histograms).  Per 256-element block:
//   masks  4 x uint64 (ballot of "word != 0", one per 64-lane slice)
//   counts int32 non-zero words  ->  exclusive scan (hipCUB) -> offsets
//   vals   the non-zero words, compacted in order
// "Zero" means all bits zero, so -0.0, NaN payloads and every integer pattern round-trip
// exactly.  Blocks never straddle chunks: a chunk table (elem_start, elem_len, blk_start)
// maps block b to its chunk (binary search), so p destination chunks encode in ONE pass and
// their value runs come out contiguous per chunk for a ragged all-to-all.
constexpr int kZsBlock = 256;

struct ZsChunk {
  int64_t base, len;   // element start / remaining elements of this block inside its chunk
};

__device__ __forceinline__ ZsChunk zs_locate(const int64_t* __restrict__ table, int nchunk, int64_t b) {
  const int64_t* es = table;
  const int64_t* el = table + nchunk;
  const int64_t* bs = table + 2 * nchunk;       // nchunk + 1 entries
  int lo = 0, hi = nchunk - 1;
  while (lo < hi) {                              // last j with bs[j] <= b
    const int mid = (lo + hi + 1) >> 1;
    if (bs[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const int64_t lb = b - bs[lo];
  return {es[lo] + lb * kZsBlock, el[lo] - lb * kZsBlock};
}

// Lane l owns the 4 consecutive words 4l..4l+3 of a block (one 16-B load for 4-byte words),
// so mask word k holds bit l = "word 4l+k is non-zero".  The compaction stays in element
// order: words before (l, k) = sum_k' popc(mask_k' & lanes<l) + non-zeros of lane l before k.
template <typename W>
__device__ __forceinline__ void zs_load4(const W* __restrict__ in, int64_t base, int64_t len, int lane, W (&v)[4]) {
  const int64_t e = (int64_t)lane * 4;
  const W* p = in + base + e;
  if (e + 3 < len && (((uintptr_t)p) % (4 * sizeof(W))) == 0) {
    if constexpr (sizeof(W) == 8) {
      const u32x4 t0 = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
      const u32x4 t1 = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p) + 1);
      __builtin_memcpy(v, &t0, 16);
      __builtin_memcpy(v + 2, &t1, 16);
    } else if constexpr (sizeof(W) == 4) {
      const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
      __builtin_memcpy(v, &t, 16);
    } else if constexpr (sizeof(W) == 2) {
      const uint2 t = *reinterpret_cast<const uint2*>(p);
      __builtin_memcpy(v, &t, 8);
    } else {
      const uint32_t t = *reinterpret_cast<const uint32_t*>(p);
      __builtin_memcpy(v, &t, 4);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = (e + k < len) ? p[k] : (W)0;
  }
}

template <typename W>
__device__ __forceinline__ void zs_store4(W* __restrict__ out, int64_t base, int64_t len, int lane, const W (&v)[4]) {
  const int64_t e = (int64_t)lane * 4;
  W* p = out + base + e;
  if (e + 3 < len && (((uintptr_t)p) % (4 * sizeof(W))) == 0) {
    if constexpr (sizeof(W) == 8) {
      u32x4 t0, t1;
      __builtin_memcpy(&t0, v, 16);
      __builtin_memcpy(&t1, v + 2, 16);
      __builtin_nontemporal_store(t0, reinterpret_cast<u32x4*>(p));
      __builtin_nontemporal_store(t1, reinterpret_cast<u32x4*>(p) + 1);
    } else if constexpr (sizeof(W) == 4) {
      u32x4 t;
      __builtin_memcpy(&t, v, 16);
      __builtin_nontemporal_store(t, reinterpret_cast<u32x4*>(p));
    } else if constexpr (sizeof(W) == 2) {
      uint2 t;
      __builtin_memcpy(&t, v, 8);
      *reinterpret_cast<uint2*>(p) = t;
    } else {
      uint32_t t;
      __builtin_memcpy(&t, v, 4);
      *reinterpret_cast<uint32_t*>(p) = t;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (e + k < len) p[k] = v[k];
  }
}

// The chunk table is staged in LDS (binary searches then cost LDS latency, not L2 round
// trips), and each wave keeps ZU consecutive blocks in flight per iteration.
constexpr int kZsMaxLdsChunks = 256;
constexpr int ZU = 4;        // blocks in flight per wave: mask pass
constexpr int ZU2 = 4;       // compaction / expansion (LDS-staged, ZU2 * 256 words per wave)

// Always LDS (nchunk <= kZsMaxLdsChunks, checked on the host): a pointer that could be either
// LDS or global compiles to flat loads, whose s_waitcnt also drains every outstanding global
// load — that serialised the unrolled data loads (measured 2.2-3.6 TB/s before the fix).
__device__ __forceinline__ const int64_t* zs_table_lds(const int64_t* __restrict__ table, int nchunk,
                                                       int64_t* lds) {
  for (int i = threadIdx.x; i < 3 * nchunk + 1; i += kBlock) lds[i] = table[i];
  __syncthreads();
  return lds;
}

template <typename W>
__global__ __launch_bounds__(kBlock) void k_zs_mask(const W* __restrict__ in, const int64_t* __restrict__ table,
                                                    int nchunk, int64_t nblk, uint64_t* __restrict__ masks,
                                                    int32_t* __restrict__ counts) {
  __shared__ int64_t lt_tab[3 * kZsMaxLdsChunks + 1];
  const int64_t* tab = zs_table_lds(table, nchunk, lt_tab);
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t b0 = wave * ZU; b0 < nblk; b0 += nwaves * ZU) {
    ZsChunk c[ZU];
#pragma unroll
    for (int u = 0; u < ZU; ++u) c[u] = (b0 + u < nblk) ? zs_locate(tab, nchunk, b0 + u) : ZsChunk{0, 0};
    W v[ZU][4];
#pragma unroll
    for (int u = 0; u < ZU; ++u) zs_load4<W>(in, c[u].base, c[u].len, lane, v[u]);   // ZU loads in flight
#pragma unroll
    for (int u = 0; u < ZU; ++u) {
      if (b0 + u >= nblk) break;
      int cnt = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t m = __ballot(v[u][k] != (W)0);
        if (lane == 0) masks[(b0 + u) * 4 + k] = m;
        cnt += __popcll(m);
      }
      if (lane == 0) counts[b0 + u] = cnt;
    }
  }
}

// Compaction and expansion stage each wave's ZU consecutive blocks through LDS.  Their
// non-zero words form ONE contiguous range [offs[b0], offs[b0 + ZU]) of vals.  Global traffic
// on that side is therefore coalesced full-line stores or loads. Per-lane scattered 4-byte
// accesses would become one partial-line transaction each (measured 3.0 / 2.5 TB/s before).
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

template <typename W, int ZU>
__global__ __launch_bounds__(kBlock) void k_zs_compact(const W* __restrict__ in, const int64_t* __restrict__ table,
                                                       int nchunk, int64_t nblk, const int64_t* __restrict__ offs,
                                                       W* __restrict__ vals) {
  __shared__ int64_t lt_tab[3 * kZsMaxLdsChunks + 1];
  __shared__ W stage[kBlock / 64][ZU * kZsBlock];
  const int64_t* tab = zs_table_lds(table, nchunk, lt_tab);
  const int lane = threadIdx.x & 63;
  W* st = stage[threadIdx.x >> 6];
  const uint64_t lt = (1ull << lane) - 1;
  const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t b0 = wave * ZU; b0 < nblk; b0 += nwaves * ZU) {
    ZsChunk c[ZU];
#pragma unroll
    for (int u = 0; u < ZU; ++u) c[u] = (b0 + u < nblk) ? zs_locate(tab, nchunk, b0 + u) : ZsChunk{0, 0};
    W v[ZU][4];
    int64_t pos[ZU];
    const int64_t bend = (b0 + ZU < nblk) ? b0 + ZU : nblk;
#pragma unroll
    for (int u = 0; u < ZU; ++u) {
      zs_load4<W>(in, c[u].base, c[u].len, lane, v[u]);
      pos[u] = (b0 + u < nblk) ? offs[b0 + u] : 0;
    }
    const int64_t base = offs[b0];
    int total = (int)(offs[bend] - base);
    MP4X_DASSERT(total >= 0 && total <= ZU * kZsBlock);
    total = total < 0 ? 0 : (total > ZU * kZsBlock ? ZU * kZsBlock : total);   // never past the stage
#pragma unroll
    for (int u = 0; u < ZU; ++u) {
      if (b0 + u >= nblk) break;
      int q = (int)(pos[u] - base);
#pragma unroll
      for (int k = 0; k < 4; ++k) q += __popcll(__ballot(v[u][k] != (W)0) & lt);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (v[u][k] != (W)0) st[q++] = v[u][k];
    }
    wave_lds_sync();
    for (int i = lane; i < total; i += 64) vals[base + i] = st[i];
    wave_lds_sync();
  }
}

template <typename W, int ZU>
__global__ __launch_bounds__(kBlock) void k_zs_expand(const uint64_t* __restrict__ masks,
                                                      const int64_t* __restrict__ offs, const W* __restrict__ vals,
                                                      const int64_t* __restrict__ table, int nchunk, int64_t nblk,
                                                      W* __restrict__ out) {
  __shared__ int64_t lt_tab[3 * kZsMaxLdsChunks + 1];
  __shared__ W stage[kBlock / 64][ZU * kZsBlock];
  const int64_t* tab = zs_table_lds(table, nchunk, lt_tab);
  const int lane = threadIdx.x & 63;
  W* st = stage[threadIdx.x >> 6];
  const uint64_t lt = (1ull << lane) - 1;
  const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t b0 = wave * ZU; b0 < nblk; b0 += nwaves * ZU) {
    ZsChunk c[ZU];
#pragma unroll
    for (int u = 0; u < ZU; ++u) c[u] = (b0 + u < nblk) ? zs_locate(tab, nchunk, b0 + u) : ZsChunk{0, 0};
    const int64_t bend = (b0 + ZU < nblk) ? b0 + ZU : nblk;
    const int64_t base = offs[b0];
    int total = (int)(offs[bend] - base);
    MP4X_DASSERT(total >= 0 && total <= ZU * kZsBlock);
    total = total < 0 ? 0 : (total > ZU * kZsBlock ? ZU * kZsBlock : total);   // never past the stage
    uint64_t m[ZU][4];
    int64_t pos[ZU];
#pragma unroll
    for (int u = 0; u < ZU; ++u) {
      if (b0 + u < nblk) {
        pos[u] = offs[b0 + u];
#pragma unroll
        for (int k = 0; k < 4; ++k) m[u][k] = masks[(b0 + u) * 4 + k];
      }
    }
    for (int i = lane; i < total; i += 64) st[i] = vals[base + i];     // coalesced
    wave_lds_sync();
    W v[ZU][4] = {};
#pragma unroll
    for (int u = 0; u < ZU; ++u) {
      if (b0 + u >= nblk) break;
      int q = (int)(pos[u] - base);
#pragma unroll
      for (int k = 0; k < 4; ++k) q += __popcll(m[u][k] & lt);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[u][k] = ((m[u][k] >> lane) & 1) ? st[q++] : (W)0;
    }
#pragma unroll
    for (int u = 0; u < ZU; ++u) zs_store4<W>(out, c[u].base, c[u].len, lane, v[u]);
    wave_lds_sync();
  }
}

__global__ void k_zs_total(const int64_t* __restrict__ offs, const int32_t* __restrict__ counts, int64_t nblk,
                           int64_t* __restrict__ total) {
  *total = nblk ? offs[nblk - 1] + counts[nblk - 1] : 0;
}

template <typename W>
static int zs_encode_t(const void* in, const int64_t* table, int nchunk, int64_t nblk, uint64_t* masks,
                       int32_t* counts, int64_t* offs, void* vals, void* temp, size_t temp_bytes, hipStream_t st) {
  const int g = grid_for((nblk + ZU - 1) / ZU * 64, 1);
  hipLaunchKernelGGL(k_zs_mask<W>, dim3(g), dim3(kBlock), 0, st, (const W*)in, table, nchunk, nblk, masks, counts);
  int e = (int)hipGetLastError();
  if (e) return e;
  e = (int)hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, counts, offs, (int)nblk, st);
  if (e) return e;
  hipLaunchKernelGGL(k_zs_total, dim3(1), dim3(1), 0, st, offs, counts, nblk, offs + nblk);
  const int g2 = grid_for((nblk + ZU2 - 1) / ZU2 * 64, 1);
  hipLaunchKernelGGL((k_zs_compact<W, ZU2>), dim3(g2), dim3(kBlock), 0, st, (const W*)in, table, nchunk, nblk, offs,
                     (W*)vals);
  return (int)hipGetLastError();
}

template <typename W>
static int zs_decode_t(const uint64_t* masks, const int32_t* counts, const void* vals, const int64_t* table,
                       int nchunk, int64_t nblk, void* out, int64_t* offs, void* temp, size_t temp_bytes,
                       hipStream_t st) {
  int e = (int)hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, counts, offs, (int)nblk, st);
  if (e) return e;
  // offs[nblk] (= total words) bounds the last wave's staged range: it must be written here too
  hipLaunchKernelGGL(k_zs_total, dim3(1), dim3(1), 0, st, offs, counts, nblk, offs + nblk);
  const int g = grid_for((nblk + ZU2 - 1) / ZU2 * 64, 1);
  hipLaunchKernelGGL((k_zs_expand<W, ZU2>), dim3(g), dim3(kBlock), 0, st, masks, offs, (const W*)vals, table, nchunk,
                     nblk, (W*)out);
  return (int)hipGetLastError();
}

}  // namespace mp4x

using namespace mp4x;

extern "C" int mp4x_quant_fp8(int dtype_in, const void* in, int64_t n, uint8_t* q, float* scales, void* stream) {
  if (n <= 0) return 0;
  if (((uintptr_t)q & 3) || ((uintptr_t)in & 15)) return MP4X_E_BADARG;
  hipStream_t st = (hipStream_t)stream;
  uint32_t* qq = reinterpret_cast<uint32_t*>(q);
  switch (dtype_in) {
    case MP4X_F32: return launch_quant<MP4X_F32>(in, n, qq, scales, st);
    case MP4X_BF16: return launch_quant<MP4X_BF16>(in, n, qq, scales, st);
    case MP4X_F16: return launch_quant<MP4X_F16>(in, n, qq, scales, st);
    default: return MP4X_E_UNSUPPORTED;
  }
}

extern "C" int mp4x_dequant_reduce_fp8(int dtype_out, void* out, const uint8_t* const* qs, const float* const* scales,
                                       int nin, int64_t n, int accumulate, uint8_t* q_out, float* s_out, void* stream) {
  if (n <= 0) return 0;
  if (nin < 1 || nin > MP4X_MAX_NIN) return MP4X_E_BADARG;
  hipStream_t st = (hipStream_t)stream;
  switch (dtype_out) {
    case MP4X_F32: return dr_dt<MP4X_F32>(out, qs, scales, nin, n, accumulate, q_out, s_out, st);
    case MP4X_BF16: return dr_dt<MP4X_BF16>(out, qs, scales, nin, n, accumulate, q_out, s_out, st);
    case MP4X_F16: return dr_dt<MP4X_F16>(out, qs, scales, nin, n, accumulate, q_out, s_out, st);
    default: return MP4X_E_UNSUPPORTED;
  }
}

extern "C" int mp4x_dequant_fp8(int dtype_out, void* out, const uint8_t* q, const float* scales, int64_t n,
                                void* stream) {
  const uint8_t* qs[1] = {q};
  const float* ss[1] = {scales};
  return mp4x_dequant_reduce_fp8(dtype_out, out, qs, ss, 1, n, 0, nullptr, nullptr, stream);
}

extern "C" size_t mp4x_zs_temp_bytes(int64_t nblk) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const int32_t*)nullptr, (int64_t*)nullptr,
                                         (int)(nblk < 1 ? 1 : nblk), (hipStream_t)0);
  return bytes;
}

// table (device int64): elem_start[nchunk], elem_len[nchunk], blk_start[nchunk + 1] (blk_start[j]
// = sum of ceil(elem_len[i] / 256) for i < j).  offs needs nblk + 1 entries; offs[nblk] = total
// non-zero words.  vals must hold the worst case (every word non-zero).
extern "C" int mp4x_zs_encode(int elem_bytes, const void* in, const int64_t* table, int nchunk, int64_t nblk,
                              uint64_t* masks, int32_t* counts, int64_t* offs, void* vals, void* temp,
                              size_t temp_bytes, void* stream) {
  if (nblk <= 0) return 0;
  if (nchunk <= 0 || nchunk > kZsMaxLdsChunks) return MP4X_E_BADARG;
  hipStream_t st = (hipStream_t)stream;
  switch (elem_bytes) {
    case 1: return zs_encode_t<uint8_t>(in, table, nchunk, nblk, masks, counts, offs, vals, temp, temp_bytes, st);
    case 2: return zs_encode_t<uint16_t>(in, table, nchunk, nblk, masks, counts, offs, vals, temp, temp_bytes, st);
    case 4: return zs_encode_t<uint32_t>(in, table, nchunk, nblk, masks, counts, offs, vals, temp, temp_bytes, st);
    case 8: return zs_encode_t<uint64_t>(in, table, nchunk, nblk, masks, counts, offs, vals, temp, temp_bytes, st);
    default: return MP4X_E_UNSUPPORTED;
  }
}

extern "C" int mp4x_zs_decode(int elem_bytes, const uint64_t* masks, const int32_t* counts, const void* vals,
                              const int64_t* table, int nchunk, int64_t nblk, void* out, int64_t* offs, void* temp,
                              size_t temp_bytes, void* stream) {
  if (nblk <= 0) return 0;
  if (nchunk <= 0 || nchunk > kZsMaxLdsChunks) return MP4X_E_BADARG;
  hipStream_t st = (hipStream_t)stream;
  switch (elem_bytes) {
    case 1: return zs_decode_t<uint8_t>(masks, counts, vals, table, nchunk, nblk, out, offs, temp, temp_bytes, st);
    case 2: return zs_decode_t<uint16_t>(masks, counts, vals, table, nchunk, nblk, out, offs, temp, temp_bytes, st);
    case 4: return zs_decode_t<uint32_t>(masks, counts, vals, table, nchunk, nblk, out, offs, temp, temp_bytes, st);
    case 8: return zs_decode_t<uint64_t>(masks, counts, vals, table, nchunk, nblk, out, offs, temp, temp_bytes, st);
    default: return MP4X_E_UNSUPPORTED;
  }
}
