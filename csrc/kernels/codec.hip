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
#include <cstring>
#include <rocprim/device/device_scan.hpp>   // 64-bit scan sizes (no (int) narrowing)
#include <stdlib.h>

#include "fp8.hpp"

namespace mp4x {

// One wave per quant block; QU consecutive blocks per wave iteration so each lane keeps QU
// 16-byte loads in flight before the first amax reduction.
constexpr int QU = 4;

template <int DT, int QU>
__global__ __launch_bounds__(kBlock) void k_quant(const void* __restrict__ in, int64_t n, uint32_t* __restrict__ q,
                                                  float* __restrict__ scales) {
  const int lane = threadIdx.x & 63;
  const int64_t nblk = (n + kQBlock - 1) / kQBlock;
  const int64_t wave = wave_id();
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

// DU consecutive quant blocks per wave iteration: DU * NIN independent loads in flight.
template <int DT, int NIN, int DU = 1>
__global__ __launch_bounds__(kBlock) void k_dequant_reduce(void* __restrict__ out, QIn<NIN> in, int64_t n,
                                                           int accumulate, uint32_t* __restrict__ q_out,
                                                           float* __restrict__ s_out) {
  const int lane = threadIdx.x & 63;
  const int64_t nblk = (n + kQBlock - 1) / kQBlock;
  const int64_t wave = wave_id();
  const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t b0 = wave * DU; b0 < nblk; b0 += nwaves * DU) {
    uint32_t w[DU][NIN];
    float s[DU][NIN];
#pragma unroll
    for (int d = 0; d < DU; ++d)
#pragma unroll
      for (int k = 0; k < NIN; ++k) {   // issue every load first: DU * NIN requests in flight
        const int64_t b = b0 + d < nblk ? b0 + d : nblk - 1;
        w[d][k] = __builtin_nontemporal_load(in.q[k] + b * 64 + lane);
        s[d][k] = in.s[k][b];
      }
#pragma unroll
    for (int d = 0; d < DU; ++d) {
      const int64_t b = b0 + d;
      if (b >= nblk) break;
      const int64_t e = b * kQBlock + lane * 4;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      if (accumulate && out) load4<DT>(out, e, n, acc);
#pragma unroll
      for (int k = 0; k < NIN; ++k) fp8_fma_acc(w[d][k], s[d][k], acc);
      if (out) store4<DT>(out, e, n, acc);
      if (q_out) quant_block(acc, q_out, s_out, b, lane);
    }
  }
}

// Streaming codec kernels launch their whole grid (one wave iteration each, up to 2^20 blocks)
// instead of grid_for's kMaxGrid cap with a grid-stride loop: measured 5.55 -> 6.14 TB/s for the
// quantise of 1 GiB f32 (profiles/r6/codec/grid_ab.jsonl).
static int g_codec_grid = 1;      // 0 = grid_for's capped grid-stride form (A/B)
static int g_dq_unroll = 0;       // A/B: quant blocks per wave iteration of the dequant-reduce (0 = by NIN)

static int codec_grid(int64_t threads, int per_wave_iter_blocks) {
  if (!g_codec_grid) return grid_for(threads, 1);
  int64_t g = (threads + kBlock - 1) / kBlock / per_wave_iter_blocks;
  if (g < 1) g = 1;
  if (g > (1 << 20)) g = 1 << 20;
  return (int)g;
}

template <int DT>
static int launch_quant(const void* in, int64_t n, uint32_t* q, float* s, hipStream_t st) {
  int64_t nblk = (n + kQBlock - 1) / kQBlock;
  const int g = codec_grid(nblk * 64, QU);        // a wave takes QU quant blocks per iteration
  hipLaunchKernelGGL((k_quant<DT, QU>), dim3(g), dim3(kBlock), 0, st, in, n, q, s);
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
  const int g = grid_for(nblk * 64, 1);
  // quant blocks per wave iteration: more loads in flight for the multi-input reduce (NIN = 8:
  // 0.91 -> 0.61 ms for 8 x 256 Mi elements, 3.5 -> 5.3 TB/s), one for the single-input dequant
  // (more costs it 15 %; profiles/r6/codec/grid_ab.jsonl)
  const int du = g_dq_unroll ? g_dq_unroll : (NIN >= 4 ? 4 : (NIN >= 2 ? 2 : 1));
  if (du == 2)
    hipLaunchKernelGGL((k_dequant_reduce<DT, NIN, 2>), dim3(g), dim3(kBlock), 0, st, out, in, n, acc,
                       reinterpret_cast<uint32_t*>(qo), so);
  else if (du == 4)
    hipLaunchKernelGGL((k_dequant_reduce<DT, NIN, 4>), dim3(g), dim3(kBlock), 0, st, out, in, n, acc,
                       reinterpret_cast<uint32_t*>(qo), so);
  else
    hipLaunchKernelGGL((k_dequant_reduce<DT, NIN, 1>), dim3(g), dim3(kBlock), 0, st, out, in, n, acc,
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
//   counts int32 non-zero words  ->  exclusive scan (rocPRIM) -> offsets
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
  const int64_t wave = wave_id();
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
  const int64_t wave = wave_id();
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

// Single-pass encode (replaces mask -> scan -> compact, which read the input twice): every
// wave takes the next tile of ZU blocks from an atomic ticket, computes masks and counts,
// publishes its tile total, and finds its exclusive prefix by DECOUPLED LOOK-BACK over the
// predecessors' status words (64 predecessors per step, one per lane); then it stages its
// non-zero words through LDS and stores them as one coalesced run.  Status word = 2-bit flag
// (1 = tile total, 2 = inclusive prefix) + 62-bit value, written with ONE relaxed agent-scope
// 64-bit atomic (the data is the flag: no fence, cdna guide G16 R2).  Tickets are handed out
// in order, so every predecessor a wave waits on is already running and never waits on a
// later tile: progress is guaranteed.  The output is identical to the three-kernel form.
constexpr uint64_t kZsAgg = 1ull << 62, kZsInc = 2ull << 62, kZsVal = (1ull << 62) - 1;

__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Workgroup tiles: 8 waves x ZU blocks (8192 words at ZU = 4).  Wave totals combine in LDS;
// ONE decoupled look-back per tile reads 512 predecessor status words per step (one per
// thread), so the inclusive-prefix frontier advances 512 tiles per memory round trip.
constexpr int kZsEncThreads = 512;
constexpr int kZsEncWaves = kZsEncThreads / 64;

template <typename W, int ZU>
__global__ __launch_bounds__(kZsEncThreads) void k_zs_encode1(const W* __restrict__ in,
                                                              const int64_t* __restrict__ table, int nchunk,
                                                              int64_t nblk, int64_t ntiles,
                                                              uint64_t* __restrict__ masks,
                                                              int32_t* __restrict__ counts,
                                                              int64_t* __restrict__ offs, W* __restrict__ vals,
                                                              uint64_t* __restrict__ status,
                                                              uint32_t* __restrict__ ticket) {
  __shared__ int64_t lt_tab[3 * kZsMaxLdsChunks + 1];
  __shared__ W stage[kZsEncWaves][ZU * kZsBlock];
  __shared__ int64_t s_wave[kZsEncWaves];       // wave totals -> exclusive prefixes in the tile
  __shared__ int64_t s_red[kZsEncWaves];        // look-back partial sums per wave
  __shared__ uint64_t s_inc[kZsEncWaves], s_inv[kZsEncWaves];
  __shared__ int64_t s_tile, s_excl;
  __shared__ int s_done;
  for (int i = threadIdx.x; i < 3 * nchunk + 1; i += kZsEncThreads) lt_tab[i] = table[i];
  __syncthreads();
  const int64_t* tab = lt_tab;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  W* st = stage[wv];
  const uint64_t lt = (1ull << lane) - 1;
  for (;;) {
    if (threadIdx.x == 0) s_tile = (int64_t)atomicAdd(ticket, 1u);
    __syncthreads();
    const int64_t t = s_tile;
    if (t >= ntiles) break;
    const int64_t b0 = (t * kZsEncWaves + wv) * ZU;   // this wave's first block
    ZsChunk c[ZU];
#pragma unroll
    for (int u = 0; u < ZU; ++u) c[u] = (b0 + u < nblk) ? zs_locate(tab, nchunk, b0 + u) : ZsChunk{0, 0};
    W v[ZU][4];
#pragma unroll
    for (int u = 0; u < ZU; ++u) zs_load4<W>(in, c[u].base, c[u].len, lane, v[u]);   // ZU loads in flight
    uint64_t mk[ZU][4];
    int cnt[ZU];
    int agg = 0;
#pragma unroll
    for (int u = 0; u < ZU; ++u) {
      cnt[u] = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        mk[u][k] = (b0 + u < nblk) ? __ballot(v[u][k] != (W)0) : 0ull;
        cnt[u] += __popcll(mk[u][k]);
      }
      agg += cnt[u];
    }
    if (lane == 0) s_wave[wv] = agg;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t run = 0;
      for (int w = 0; w < kZsEncWaves; ++w) {
        const int64_t x = s_wave[w];
        s_wave[w] = run;
        run += x;
      }
      s_excl = run;                                     // tile total until the look-back
      __hip_atomic_store(&status[t], (t == 0 ? kZsInc : kZsAgg) | (uint64_t)run, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const int64_t tile_total = s_excl;
    int64_t excl = 0;
    if (t > 0) {                                        // workgroup-wide decoupled look-back
      int64_t j = t - 1;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        const int64_t idx = j - threadIdx.x;
        const uint64_t sw = idx >= 0 ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : kZsInc;
        const uint32_t flag = (uint32_t)(sw >> 62);
        const uint64_t inc = __ballot(flag == 2), inv = __ballot(flag == 0);
        if (lane == 0) {
          s_inc[wv] = inc;
          s_inv[wv] = inv;
        }
        __syncthreads();
        int first = kZsEncThreads;                      // nearest inclusive (thread index)
        for (int w = 0; w < kZsEncWaves; ++w)
          if (s_inc[w]) {
            first = w * 64 + __ffsll((long long)s_inc[w]) - 1;
            break;
          }
        bool wait = false;                              // any unpublished word at or before `first`
        for (int w = 0; w < kZsEncWaves && w * 64 <= first; ++w) {
          const int hi = first - w * 64;                // lanes 0..hi of wave w are needed
          const uint64_t need = hi >= 63 ? ~0ull : ((2ull << hi) - 1);
          if (s_inv[w] & need) wait = true;
        }
        if (wait) {
          // one thread decides the give-up (10 s: never hang) so every wave leaves together
          if (threadIdx.x == 0) s_done = __builtin_amdgcn_s_memrealtime() - t0 > 1000000000ull;
          __syncthreads();                              // also: s_inc / s_inv are rewritten next pass
          if (s_done) break;
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        const int64_t part = wave_sum_i64((int)threadIdx.x <= first ? (int64_t)(sw & kZsVal) : 0);
        if (lane == 0) s_red[wv] = part;
        __syncthreads();
        for (int w = 0; w < kZsEncWaves; ++w) excl += s_red[w];
        __syncthreads();
        if (first < kZsEncThreads) break;
        j -= kZsEncThreads;                             // 512 tile totals: look further back
      }
      if (threadIdx.x == 0)
        __hip_atomic_store(&status[t], kZsInc | (uint64_t)(excl + tile_total), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    int64_t pos = excl + s_wave[wv];                    // this wave's first word in vals
    const int64_t wbase = pos;
#pragma unroll
    for (int u = 0; u < ZU; ++u) {
      if (b0 + u >= nblk) break;
      if (lane == 0) {
        counts[b0 + u] = cnt[u];
        offs[b0 + u] = pos;
#pragma unroll
        for (int k = 0; k < 4; ++k) masks[(b0 + u) * 4 + k] = mk[u][k];
      }
      int q = (int)(pos - wbase);
#pragma unroll
      for (int k = 0; k < 4; ++k) q += __popcll(mk[u][k] & lt);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (v[u][k] != (W)0) st[q++] = v[u][k];
      pos += cnt[u];
    }
    if (b0 < nblk && b0 + ZU >= nblk && lane == 0) offs[nblk] = pos;   // the last block's wave
    wave_lds_sync();
    for (int i = lane; i < agg; i += 64) vals[wbase + i] = st[i];
    __syncthreads();                                    // stage / s_wave reused by the next tile
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
  const int64_t wave = wave_id();
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

static int64_t zs_tiles(int64_t nblk) { return (nblk + ZU2 * kZsEncWaves - 1) / (ZU2 * kZsEncWaves); }
static size_t zs_status_bytes(int64_t nblk) { return (size_t)(zs_tiles(nblk) + 2) * sizeof(uint64_t); }

template <typename W>
static int zs_encode_t(const void* in, const int64_t* table, int nchunk, int64_t nblk, uint64_t* masks,
                       int32_t* counts, int64_t* offs, void* vals, void* temp, size_t temp_bytes, hipStream_t st) {
  const int64_t ntiles = zs_tiles(nblk);
  if (temp_bytes < zs_status_bytes(nblk)) return MP4X_E_BADARG;
  uint64_t* status = (uint64_t*)temp;
  uint32_t* ticket = (uint32_t*)(status + ntiles);
  int e = (int)hipMemsetAsync(temp, 0, zs_status_bytes(nblk), st);    // re-initialised every call
  if (e) return e;
  // enough workgroups to fill the chip (4 x 512 threads per CU); each loops over tickets
  const int g = (int)(ntiles < 1024 ? ntiles : 1024);
  hipLaunchKernelGGL((k_zs_encode1<W, ZU2>), dim3(g), dim3(kZsEncThreads), 0, st, (const W*)in, table, nchunk, nblk,
                     ntiles, masks, counts, offs, (W*)vals, status, ticket);
  return (int)hipGetLastError();
}

// The three-kernel form (mask pass, rocPRIM scan, compaction): the default (see zs_twopass) and
// the reference the single-pass kernel is tested against.
template <typename W>
static int zs_encode_twopass_t(const void* in, const int64_t* table, int nchunk, int64_t nblk, uint64_t* masks,
                               int32_t* counts, int64_t* offs, void* vals, void* temp, size_t temp_bytes,
                               hipStream_t st) {
  const int g = grid_for((nblk + ZU - 1) / ZU * 64, 1);
  hipLaunchKernelGGL(k_zs_mask<W>, dim3(g), dim3(kBlock), 0, st, (const W*)in, table, nchunk, nblk, masks, counts);
  int e = (int)hipGetLastError();
  if (e) return e;
  e = (int)rocprim::exclusive_scan(temp, temp_bytes, counts, offs, (int64_t)0, (size_t)nblk, rocprim::plus<int64_t>(),
                                   st);
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
  int e = (int)rocprim::exclusive_scan(temp, temp_bytes, counts, offs, (int64_t)0, (size_t)nblk,
                                       rocprim::plus<int64_t>(), st);
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

extern "C" void mp4x_set_codec_grid(int full) { g_codec_grid = full; }
extern "C" void mp4x_set_dq_unroll(int du) { g_dq_unroll = du; }

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
  (void)rocprim::exclusive_scan(nullptr, bytes, (const int32_t*)nullptr, (int64_t*)nullptr, (int64_t)0,
                                (size_t)(nblk < 1 ? 1 : nblk), rocprim::plus<int64_t>(), (hipStream_t)0);
  const size_t sb = zs_status_bytes(nblk < 1 ? 1 : nblk);      // single-pass encode: tile status words
  return bytes > sb ? bytes : sb;
}

static int g_zs_twopass = -1;

// Default: the three-kernel form.  Measured on MI355X, 256 MiB f32 (profiles/r1/kbench9.json):
// 0.213 ms against 0.324 ms for the single-pass kernel — every workgroup serialises ticket ->
// loads -> look-back per tile, so the second read the single pass saves costs less than the
// latency it exposes.  MP4X_ZS_ONEPASS=1 selects the single pass.
static int zs_twopass() {
  if (g_zs_twopass < 0) {
    const char* e = getenv("MP4X_ZS_ONEPASS");
    g_zs_twopass = (e && e[0] == '1') ? 0 : 1;
  }
  return g_zs_twopass;
}

// A/B switch: 1 = mask + scan + compact (two reads of the input), 0 = single-pass encode
extern "C" int mp4x_zs_set_twopass(int on) {
  g_zs_twopass = on ? 1 : 0;
  return 0;
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
  if (zs_twopass()) {
    switch (elem_bytes) {
      case 1: return zs_encode_twopass_t<uint8_t>(in, table, nchunk, nblk, masks, counts, offs, vals, temp, temp_bytes, st);
      case 2: return zs_encode_twopass_t<uint16_t>(in, table, nchunk, nblk, masks, counts, offs, vals, temp, temp_bytes, st);
      case 4: return zs_encode_twopass_t<uint32_t>(in, table, nchunk, nblk, masks, counts, offs, vals, temp, temp_bytes, st);
      case 8: return zs_encode_twopass_t<uint64_t>(in, table, nchunk, nblk, masks, counts, offs, vals, temp, temp_bytes, st);
      default: return MP4X_E_UNSUPPORTED;
    }
  }
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
