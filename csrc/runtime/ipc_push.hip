// Zero-copy PUSH two-shot allreduce (see ipc_common.hpp for the protocol).
//
// The two-shot with every xGMI transfer a WRITE (posted: no request/response round trip per
// line, the protocol RCCL's ring primitives use) instead of a read.  Data pointers are the
// registered caller tensors; scr[k] is rank k's receive scratch of p-1 chunk slots (slot of
// sender q: q < k ? q : q - 1).
//   phase 1: rank r writes its chunk k (k != r) into slot(r) of rank k's scratch;
//   mid barrier (every write released at system scope before the flag);
//   phase 2: rank r reduces chunk r in RANK ORDER from its own tensor and the p-1 LOCAL slots,
//            stores the result into its tensor and writes it into chunk r of every peer's tensor;
//   end barrier.
// Block b of every rank touches the same chunk-relative offsets in every phase, so the per-block
// barriers order every write against the reads and writes of the same offsets on the peers.
#include "ipc_common.hpp"

namespace mp4x {

struct ScrPtrs {
  void* s[kIpcMaxRanks];
};

template <int DT, int OP, int NR>
__global__ __launch_bounds__(kIpcThreads) void k_ipc_twoshot_push(IpcPtrs P, ScrPtrs S, Signal* self, int rank,
                                                                   int64_t nvec, uint32_t epoch,
                                                                   const uint32_t* epoch_dev, float scale, int op) {
  constexpr int p = NR;
  MP4X_DASSERT(rank >= 0 && rank < NR && blockIdx.x < kIpcMaxBlocks);
  epoch = resolve_epoch(epoch, epoch_dev);
  const int64_t chunk = (nvec + p - 1) / p;
  const int64_t stride = (int64_t)gridDim.x * kIpcThreads;
  const int64_t off0 = (int64_t)blockIdx.x * kIpcThreads + threadIdx.x;
  u32x4* mine = reinterpret_cast<u32x4*>(const_cast<void*>(P.data[rank]));
  const u32x4* myscr = reinterpret_cast<const u32x4*>(S.s[rank]);
  if (!block_barrier(P, 0, rank, p, epoch, self)) return;
  for (int64_t v = off0; v < chunk; v += stride) {
    u32x4 x[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) {                 // local reads of every outgoing chunk
      const int64_t idx = (int64_t)k * chunk + v;
      if (k != rank && idx < nvec) x[k] = mine[idx];
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {                 // p-1 posted remote writes, every link at once
      const int64_t idx = (int64_t)k * chunk + v;
      if (k != rank && idx < nvec)
        reinterpret_cast<u32x4*>(S.s[k])[(int64_t)(rank < k ? rank : rank - 1) * chunk + v] = x[k];
    }
  }
  if (!block_barrier(P, 1, rank, p, epoch, self)) return;
  const int64_t b = (int64_t)rank * chunk;
  const int64_t e = b + chunk < nvec ? b + chunk : nvec;
  for (int64_t v = off0; b + v < e; v += stride) {
    u32x4 r[NR];
#pragma unroll
    for (int q = 0; q < NR; ++q)                   // all local: own chunk + p-1 scratch slots
      r[q] = q == rank ? mine[b + v] : myscr[(int64_t)(q < rank ? q : q - 1) * chunk + v];
    const u32x4 o = fold_any<DT, OP, NR>(r, scale, op);   // rank order: deterministic, = the pull form
    mine[b + v] = o;
#pragma unroll
    for (int k = 0; k < NR; ++k)                   // the all-gather half, pushed to every peer
      if (k != rank) reinterpret_cast<u32x4*>(const_cast<void*>(P.data[k]))[b + v] = o;
  }
  block_barrier(P, 2, rank, p, epoch, self);
}

}  // namespace mp4x

using namespace mp4x;

// Zero-copy PUSH two-shot (see k_ipc_twoshot_push): data_ptrs = every rank's registered tensor
// (this rank's own included; the result replaces it), scratch_ptrs = every rank's receive
// scratch of at least (p - 1) * ceil(nbytes / 16 / p) 16-byte vectors.  Any operator of the
// reference table valid for dtype.
extern "C" int mp4x_ipc_allreduce_push(int dtype, int op, void* const* data_ptrs, void* const* scratch_ptrs,
                                       void* const* signal_ptrs, int rank, int p, int64_t nbytes, uint32_t epoch,
                                       int blocks, const uint32_t* epoch_dev, float scale, void* stream) {
  if ((nbytes & 15) || nbytes <= 0) return MP4X_E_BADARG;
  if (scale != 1.0f && !float_dtype(dtype)) return MP4X_E_BADARG;
  IpcPtrs P;
  if (int e = ipc_prepare(data_ptrs, signal_ptrs, rank, p, &P)) return e;
  ScrPtrs S;
  for (int k = 0; k < kIpcMaxRanks; ++k) {
    S.s[k] = k < p ? scratch_ptrs[k] : nullptr;
    if (k < p && (((uintptr_t)S.s[k] & 15) || !S.s[k])) return MP4X_E_BADARG;
  }
  const int64_t nvec = nbytes / 16;
  if (blocks <= 0) {
    const int64_t chunk = (nvec + p - 1) / p;
    int64_t b = (chunk + kIpcThreads - 1) / kIpcThreads;
    blocks = (int)(b < 1 ? 1 : (b > kIpcMaxBlocks ? kIpcMaxBlocks : b));
  }
  if (blocks > kIpcMaxBlocks) blocks = kIpcMaxBlocks;
  Signal* self = (Signal*)signal_ptrs[rank];
  hipStream_t st = (hipStream_t)stream;
  return with_dtype(dtype, [&](auto dtc) {
    constexpr int DT = decltype(dtc)::value;
    return with_op<DT>(op, [&](auto opc) {
      constexpr int OP = decltype(opc)::value;
      return with_nr(p, [&](auto nrc) {
        constexpr int NR = decltype(nrc)::value;
        hipLaunchKernelGGL((k_ipc_twoshot_push<DT, OP, NR>), dim3(blocks), dim3(kIpcThreads), 0, st, P, S, self,
                           rank, nvec, epoch, epoch_dev, scale, op);
        return (int)hipGetLastError();
      });
    });
  });
}

extern "C" int mp4x_ipc_occupancy_push(int dtype, int op, int p, int* blocks_per_cu) {
  int m = 1 << 30;
  int e = with_dtype(dtype, [&](auto dtc) {
    constexpr int DT = decltype(dtc)::value;
    return with_op<DT>(op, [&](auto opc) {
      constexpr int OP = decltype(opc)::value;
      return with_nr(p, [&](auto nrc) {
        occ_min(k_ipc_twoshot_push<DT, OP, decltype(nrc)::value>, &m);
        return 0;
      });
    });
  });
  *blocks_per_cu = m == (1 << 30) ? 0 : m;
  return e;
}
