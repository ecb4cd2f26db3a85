// Direct reduce-scatter over ragged per-rank ranges (see ipc_common.hpp for the protocol).
//
// The first half of the two-shot as a collective of its own (reduceScatterArray counts), in
// 16-byte vectors of the staged buffers or of registered tensors: rank r reads [lo_r, hi_r)
// from ALL p buffers at once and reduces in registers — the fused peer-load + reduce of the
// reference's ring reduce-scatter (ProcessCommSlave.java:1329-1373), for every
// operator of the table.
#include "ipc_common.hpp"

namespace mp4x {

// Per-call launch options of the reduce-scatter (passed by value to the kernel; no host state
// survives a call).
struct RsOpts {
  const u32x4* src;   // fused staging source, nullptr = pre-staged / zero-copy
  Segs segs;          // every rank's segment (vector offsets), used when src != nullptr
};

// src != nullptr: fused staging — block b copies, for EVERY rank's segment k, the vectors block b
// of rank k will read from this buffer (segment-relative grid stride), then meets the peers.
template <int DT, int OP, int NR>
__global__ __launch_bounds__(kIpcThreads) void k_ipc_reduce_range(IpcPtrs P, Signal* self, int rank, int64_t lo,
                                                                   int64_t hi, u32x4* __restrict__ out,
                                                                   uint32_t epoch, const uint32_t* epoch_dev,
                                                                   RsOpts o, int op) {
  constexpr int p = NR;
  MP4X_DASSERT(rank >= 0 && rank < NR && lo <= hi);
  epoch = resolve_epoch(epoch, epoch_dev);
  const int64_t stride = (int64_t)gridDim.x * kIpcThreads;
  if (o.src) {
    u32x4* mine = reinterpret_cast<u32x4*>(const_cast<void*>(P.data[rank]));
    const int64_t off0 = (int64_t)blockIdx.x * kIpcThreads + threadIdx.x;
#pragma unroll
    for (int k = 0; k < NR; ++k)
      for (int64_t v = o.segs.lo[k] + off0; v < o.segs.hi[k]; v += stride) mine[v] = o.src[v];
  }
  if (!block_barrier(P, 0, rank, p, epoch, self)) return;
  for (int64_t v = lo + (int64_t)blockIdx.x * kIpcThreads + threadIdx.x; v < hi; v += stride)
    out[v - lo] = reduce_vec<DT, OP, NR>(P, v, 1.0f, op);
  block_barrier(P, 2, rank, p, epoch, self);
}

static int launch_rs(int dtype, int op, const IpcPtrs& P, Signal* self, int rank, int p, int64_t lo, int64_t hi,
                     void* out, uint32_t epoch, const uint32_t* edev, int blocks, hipStream_t st, const RsOpts& o) {
  return with_dtype(dtype, [&](auto dtc) {
    constexpr int DT = decltype(dtc)::value;
    return with_op<DT>(op, [&](auto opc) {
      constexpr int OP = decltype(opc)::value;
      return with_nr(p, [&](auto nrc) {
        constexpr int NR = decltype(nrc)::value;
        hipLaunchKernelGGL((k_ipc_reduce_range<DT, OP, NR>), dim3(blocks), dim3(kIpcThreads), 0, st, P, self, rank,
                           lo, hi, (u32x4*)out, epoch, edev, o, op);
        return (int)hipGetLastError();
      });
    });
  });
}

}  // namespace mp4x

using namespace mp4x;

// Reduce-scatter over staged buffers: out (16-B aligned) receives vectors [vec_lo, vec_hi) of
// the op-reduction of all p buffers.  Every rank stages its WHOLE range before the call.
extern "C" int mp4x_ipc_reduce_scatter(int dtype, int op, void* const* data_ptrs, void* const* signal_ptrs, int rank,
                                       int p, int64_t vec_lo, int64_t vec_hi, void* out, uint32_t epoch, int blocks,
                                       const uint32_t* epoch_dev, void* stream) {
  IpcPtrs P;
  if (int e = ipc_prepare(data_ptrs, signal_ptrs, rank, p, &P)) return e;
  if (vec_lo < 0 || vec_hi < vec_lo || ((uintptr_t)out & 15)) return MP4X_E_BADARG;
  const RsOpts o{nullptr, Segs{}};
  return launch_rs(dtype, op, P, (Signal*)signal_ptrs[rank], rank, p, vec_lo, vec_hi, out, epoch, epoch_dev,
                   ipc_blocks(blocks, vec_hi - vec_lo), (hipStream_t)stream, o);
}

// Reduce-scatter with fused staging: `src` (16-B aligned) holds this rank's whole range laid out
// like the buffer (vector offsets seg_lo/seg_hi per rank, relative to src and to the buffer);
// this rank's reduced segment goes straight to `out` (16-B aligned) at out[v - lo].  One launch.
// Every refusal of mp4x_ipc_reduce_scatter_from (the latency fast path runs it before its epoch
// moves): alignment, rank range, segment bounds, and the (dtype, op) pair.
extern "C" int mp4x_ipc_reduce_scatter_from_check(int dtype, int op, int rank, int p, const int64_t* seg_lo,
                                                  const int64_t* seg_hi, const void* src, const void* out) {
  if (!src || ((uintptr_t)src & 15) || ((uintptr_t)out & 15)) return MP4X_E_BADARG;
  if (p < 2 || p > kIpcMaxRanks || rank < 0 || rank >= p) return MP4X_E_BADARG;
  for (int k = 0; k < p; ++k)
    if (seg_lo[k] < 0 || seg_hi[k] < seg_lo[k]) return MP4X_E_BADARG;
  return op_supported(dtype, op);
}

extern "C" int mp4x_ipc_reduce_scatter_from(int dtype, int op, void* const* data_ptrs, void* const* signal_ptrs,
                                            int rank, int p, const int64_t* seg_lo, const int64_t* seg_hi,
                                            const void* src, void* out, uint32_t epoch, int blocks,
                                            const uint32_t* epoch_dev, void* stream) {
  if (int e = mp4x_ipc_reduce_scatter_from_check(dtype, op, rank, p, seg_lo, seg_hi, src, out)) return e;
  IpcPtrs P;
  if (int e = ipc_prepare(data_ptrs, signal_ptrs, rank, p, &P)) return e;
  RsOpts o;
  o.src = (const u32x4*)src;
  for (int k = 0; k < kIpcMaxRanks; ++k) {
    o.segs.lo[k] = k < p ? seg_lo[k] : 0;
    o.segs.hi[k] = k < p ? seg_hi[k] : 0;
  }
  const int64_t lo = o.segs.lo[rank], hi = o.segs.hi[rank];
  return launch_rs(dtype, op, P, (Signal*)signal_ptrs[rank], rank, p, lo, hi, out, epoch, epoch_dev,
                   ipc_blocks(blocks, hi - lo), (hipStream_t)stream, o);
}

extern "C" int mp4x_ipc_occupancy_rs(int dtype, int op, int p, int* blocks_per_cu) {
  int m = 1 << 30;
  int e = with_dtype(dtype, [&](auto dtc) {
    constexpr int DT = decltype(dtc)::value;
    return with_op<DT>(op, [&](auto opc) {
      constexpr int OP = decltype(opc)::value;
      return with_nr(p, [&](auto nrc) {
        occ_min(k_ipc_reduce_range<DT, OP, decltype(nrc)::value>, &m);
        return 0;
      });
    });
  });
  *blocks_per_cu = m == (1 << 30) ? 0 : m;
  return e;
}
