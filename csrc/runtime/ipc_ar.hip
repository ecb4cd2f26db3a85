// One-shot / two-shot allreduce over IPC-mapped peer buffers (see ipc_common.hpp for the
// protocol).  Every (dtype, op) pair of the reference's operator table runs here; the hot pairs
// with a compile-time combine, the others through the runtime-op kernel (kOpRt).
#include "ipc_common.hpp"

namespace mp4x {

// src != nullptr: the kernel stages its own input (fused copy-in, one launch instead of a
// memcpy + kernel): block b copies exactly the vectors block b of every peer will read, then
// meets them at the start barrier (whose release fence publishes the copies).
//
// slot_vecs > 0 (the latency tier, staged and fused): the staging area is one of TWO slots at
// vector offset slot_base + (epoch & 1) * slot_vecs, chosen by the epoch's parity (consecutive
// epochs alternate parity, next_epoch), and the kernel has NO end barrier — one cross-rank round
// trip per call instead of two.  Safe: this rank writes a slot again only two calls later, after
// the start barrier of the call in between, which every peer reaches only once it has finished
// reading this call's slot (kernels of one communicator complete in order: the stream-order
// guard, order.hip); the other kernel families stage below slot_base; a peer one call ahead at
// the start barrier is accepted there (only here: block_barrier's accept_ahead).
template <int DT, int OP, int NR>
__global__ __launch_bounds__(kIpcThreads) void k_ipc_oneshot(IpcPtrs P, Signal* self, int rank, int64_t nvec,
                                                              u32x4* __restrict__ out, uint32_t epoch,
                                                              const uint32_t* epoch_dev,
                                                              const u32x4* __restrict__ src, float scale, int op,
                                                              int64_t slot_base, int64_t slot_vecs) {
  constexpr int p = NR;
  epoch = resolve_epoch(epoch, epoch_dev);
  const int64_t so = slot_vecs > 0 ? slot_base + (int64_t)(epoch & 1u) * slot_vecs : 0;
  const int64_t stride = (int64_t)gridDim.x * kIpcThreads;
  if (src) {
    u32x4* mine = reinterpret_cast<u32x4*>(const_cast<void*>(P.data[rank])) + so;
    for (int64_t v = (int64_t)blockIdx.x * kIpcThreads + threadIdx.x; v < nvec; v += stride) mine[v] = src[v];
  }
  if (!block_barrier(P, 0, rank, p, epoch, self, slot_vecs > 0)) return;
  for (int64_t v = (int64_t)blockIdx.x * kIpcThreads + threadIdx.x; v < nvec; v += stride)
    out[v] = reduce_vec<DT, OP, NR>(P, v + so, scale, op);
  if (slot_vecs <= 0) block_barrier(P, 2, rank, p, epoch, self);
}

// two-shot: direct reduce-scatter into own buffer chunk `rank`, then direct all-gather.
template <int DT, int OP, int NR>
__global__ __launch_bounds__(kIpcThreads) void k_ipc_twoshot(IpcPtrs P, Signal* self, int rank, int64_t nvec,
                                                              u32x4* __restrict__ out, uint32_t epoch,
                                                              const uint32_t* epoch_dev,
                                                              const u32x4* __restrict__ src, float scale, int op,
                                                              int64_t slot_base, int64_t slot_vecs) {
  constexpr int p = NR;
  MP4X_DASSERT(rank >= 0 && rank < NR && blockIdx.x < kIpcMaxBlocks);
  epoch = resolve_epoch(epoch, epoch_dev);
  // slotted (staged, fused copy-in, one piece): the same double-buffered slots as the one-shot,
  // so the end barrier goes — the all-gather's reads of a slot finish before the reader's next
  // call starts, and this rank writes that slot again only two calls later (k_ipc_oneshot)
  const int64_t so = slot_vecs > 0 ? slot_base + (int64_t)(epoch & 1u) * slot_vecs : 0;
  const int64_t chunk = (nvec + p - 1) / p;
  const int64_t stride = (int64_t)gridDim.x * kIpcThreads;
  const int64_t off0 = (int64_t)blockIdx.x * kIpcThreads + threadIdx.x;
  u32x4* mine = reinterpret_cast<u32x4*>(const_cast<void*>(P.data[rank])) + so;
  if (src) {   // fused copy-in: block b stages the chunk offsets block b of every peer reads
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int64_t b = (int64_t)k * chunk;
      const int64_t e = b + chunk < nvec ? b + chunk : nvec;
      for (int64_t v = b + off0; v < e; v += stride) mine[v] = src[v];
    }
  }
  if (!block_barrier(P, 0, rank, p, epoch, self, slot_vecs > 0)) return;
  {
    const int64_t b = (int64_t)rank * chunk;
    const int64_t e = b + chunk < nvec ? b + chunk : nvec;
    // zero-copy form: `out` IS this rank's registered buffer (== mine), one store per vector
    const bool zc = out == mine;
    for (int64_t v = b + off0; v < e; v += stride) {
      u32x4 o = reduce_vec<DT, OP, NR>(P, v + so, scale, op);
      mine[v] = o;
      if (!zc) out[v] = o;
    }
  }
  if (!block_barrier(P, 1, rank, p, epoch, self)) return;
  // all-gather: every thread pulls the same chunk offset from ALL p-1 peers at once, so all
  // xGMI links stream concurrently (peer after peer would leave one link busy at a time).
  // k is a compile-time index: no dynamic indexing of the kernarg pointer table.
  for (int64_t v = off0; v < chunk; v += stride) {
    u32x4 x[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int64_t idx = (int64_t)k * chunk + v;
      if (k != rank && idx < nvec) x[k] = reinterpret_cast<const u32x4*>(P.data[k])[so + idx];
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int64_t idx = (int64_t)k * chunk + v;
      if (k != rank && idx < nvec) out[idx] = x[k];
    }
  }
  if (slot_vecs <= 0) block_barrier(P, 2, rank, p, epoch, self);
}

}  // namespace mp4x

using namespace mp4x;

// algo 0 = one-shot, 1 = two-shot.  data_ptrs / signal_ptrs: p entries (own rank included,
// peers as mapped by mp4x_ipc_open_handle).  nbytes must be a multiple of 16.
// epoch_dev == NULL: `epoch` (host counter) is used.  epoch_dev != NULL: graph-capturable form,
// the kernel reads the epoch from device memory (bump it with mp4x_ipc_bump_epoch first).
// src != NULL: this rank's input (16-byte aligned) is copied into its own buffer INSIDE the
// kernel (fused copy-in: one launch per call); NULL: already staged, or zero-copy (the data
// pointers are the registered caller tensors and out == data_ptrs[rank]).  scale != 1: the
// reduced value is multiplied by it before it is stored (fused average; float dtypes only).
// op: any operator of the reference table valid for dtype (MP4X_E_UNSUPPORTED otherwise).
// slot_base / slot_vecs (16-byte vectors; one- and two-shot): the double-buffered slots (see
// k_ipc_oneshot); 0 = the single-buffer form with its end barrier.  A slotted call needs src (the
// fused copy-in: the staging target depends on the device-side epoch) and nbytes <= a slot.
namespace {
// Everything mp4x_ipc_allreduce_ex2 refuses, checked without launching: the fast path
// (mp4x_ipc_fast_allreduce) runs it BEFORE its epoch moves, so a refused call leaves this rank's
// epoch where its peers expect it; after it only a HIP launch error remains.
int ar_check(int algo, int dtype, int op, int rank, int p, int64_t nbytes, const void* src, const void* out,
             float scale, int64_t slot_base, int64_t slot_vecs) {
  if ((nbytes & 15) || nbytes <= 0 || algo < 0 || algo > 1) return MP4X_E_BADARG;
  if (slot_vecs > 0 && (!src || nbytes / 16 > slot_vecs || slot_base < 0)) return MP4X_E_BADARG;
  if (((uintptr_t)out & 15) || ((uintptr_t)src & 15)) return MP4X_E_BADARG;
  if (scale != 1.0f && !float_dtype(dtype)) return MP4X_E_BADARG;
  if (p < 2 || p > kIpcMaxRanks || rank < 0 || rank >= p) return MP4X_E_BADARG;
  return op_supported(dtype, op);
}
}  // namespace

extern "C" int mp4x_ipc_allreduce_ex2(int algo, int dtype, int op, void* const* data_ptrs, void* const* signal_ptrs,
                                      int rank, int p, int64_t nbytes, const void* src, void* out, uint32_t epoch,
                                      int blocks, const uint32_t* epoch_dev, float scale, void* stream,
                                      int64_t slot_base, int64_t slot_vecs) {
  if (int e = ar_check(algo, dtype, op, rank, p, nbytes, src, out, scale, slot_base, slot_vecs)) return e;
  IpcPtrs P;
  if (int e = ipc_prepare(data_ptrs, signal_ptrs, rank, p, &P)) return e;
  const int64_t nvec = nbytes / 16;
  if (blocks <= 0) {
    int64_t b = (nvec + kIpcThreads - 1) / kIpcThreads;
    // one-shot (latency tier): up to 128 blocks; two-shot: up to one block per CU so large
    // messages keep enough remote requests in flight on every link
    const int64_t cap = algo == 0 ? 128 : kIpcMaxBlocks;
    blocks = (int)(b < 1 ? 1 : (b > cap ? cap : b));
  }
  if (blocks > kIpcMaxBlocks) blocks = kIpcMaxBlocks;
  Signal* self = (Signal*)signal_ptrs[rank];
  hipStream_t st = (hipStream_t)stream;
  const u32x4* srcv = (const u32x4*)src;
  u32x4* outv = (u32x4*)out;
  return with_dtype(dtype, [&](auto dtc) {
    constexpr int DT = decltype(dtc)::value;
    return with_op<DT>(op, [&](auto opc) {
      constexpr int OP = decltype(opc)::value;
      return with_nr(p, [&](auto nrc) {
        constexpr int NR = decltype(nrc)::value;
        if (algo == 0)
          hipLaunchKernelGGL((k_ipc_oneshot<DT, OP, NR>), dim3(blocks), dim3(kIpcThreads), 0, st, P, self, rank,
                             nvec, outv, epoch, epoch_dev, srcv, scale, op, slot_base, slot_vecs);
        else
          hipLaunchKernelGGL((k_ipc_twoshot<DT, OP, NR>), dim3(blocks), dim3(kIpcThreads), 0, st, P, self, rank,
                             nvec, outv, epoch, epoch_dev, srcv, scale, op, slot_base, slot_vecs);
        return (int)hipGetLastError();
      });
    });
  });
}

// The latency tier's whole per-call host path in ONE native call (VERDICT r4 Next #5: 4.7 us of a
// 10 us 4 KiB allreduce was interpreter time above the bare launch).  The Python entry
// (ProcessCommSlave.allreduceArray) looks its call shape up in the engine's memo and hands over
// the memoised launch; everything the Python path did per call happens here:
//   * the fail-stop check: every IPC instance's pinned host error word (an earlier collective
//     that timed out fails the next call: MP4X_E_FAILED_EARLIER, the caller raises);
//   * the capture check: a stream being captured needs the device-epoch form (MP4X_E_CAPTURING);
//   * every argument refusal of the launcher (MP4X_E_BADARG / MP4X_E_UNSUPPORTED);
//   * the communicator's stream order (order.hip: a call on another stream than the previous
//     one first waits for it);
//   * the epoch bump, in the instance's epoch box (the same word IpcAllreduce.epoch reads);
//   * the launch (mp4x_ipc_allreduce_ex: fused copy-in, in place, fused scale).
// Every refusal comes BEFORE the epoch moves (1001-1004: nothing happened, the caller may take
// the full path).  A launch that fails AFTER it (a HIP error) leaves this rank at the same epoch
// as its peers, whose kernels of this call then time out at their start barrier: that is
// consistent, so the epoch is NOT rolled back; instead the instance's own host error word gets
// code 5, and this rank's next call fails at once (raise_if_failed) instead of waiting for them.
struct FastAr {
  const uint32_t* herr[8];   // pinned host error words of the engine's instances (nullptr ends the list)
  uint32_t* epoch;           // the instance's epoch box
  void* const* data_ptrs;    // every rank's staging buffer
  void* const* signal_ptrs;  // every rank's signal block
  int32_t rank, p;
  int64_t slot_base, slot_vecs;   // the double-buffered slots of the one- / two-shot (0: none)
  StreamOrder* order;        // the communicator's stream-order guard (nullptr: none)
  uint32_t* own_err;         // this instance's pinned host error word (launch failures: code 5)
};

constexpr uint32_t kLaunchFailedErr = 5u;

namespace {
// The first check of every fast path: an earlier collective of any of the engine's instances
// timed out (fail the call: MP4X_E_FAILED_EARLIER).  Host memory only.
int fast_prologue(const FastAr* s) {
  for (int i = 0; i < 8 && s->herr[i]; ++i)
    if (__atomic_load_n(s->herr[i], __ATOMIC_RELAXED)) return MP4X_E_FAILED_EARLIER;
  return 0;
}

// After the argument checks (host only, so a refused call never touches HIP): the stream is being
// captured (the device-epoch form is needed: MP4X_E_CAPTURING), else order the stream after the
// communicator's previous launch and move the epoch box.  A failing stream join is a HIP error
// before the epoch moved.
int fast_begin(const FastAr* s, void* stream, uint32_t* e) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing((hipStream_t)stream, &cs) != hipSuccess) {
    (void)hipGetLastError();
    return MP4X_E_CAPTURING;
  }
  if (cs != hipStreamCaptureStatusNone) return MP4X_E_CAPTURING;
  if (int rc = mp4x_order_enter(s->order, stream)) return rc;
  *e = next_epoch(*s->epoch);
  *s->epoch = *e;
  return 0;
}

// After the epoch moved: a failed launch marks the instance (see FastAr).
int fast_end(const FastAr* s, int rc) {
  if (rc && s->own_err) __atomic_store_n(s->own_err, kLaunchFailedErr, __ATOMIC_RELAXED);
  return rc;
}
}  // namespace

extern "C" int mp4x_ipc_fast_allreduce(const FastAr* s, int algo, int dtype, int op, void* buf, int64_t nbytes,
                                       int blocks, float scale, void* stream) {
  if (int e = fast_prologue(s)) return e;
  const bool slotted = (algo == 0 || algo == 1) && s->slot_vecs > 0 && nbytes > 0 && nbytes / 16 <= s->slot_vecs;
  const int64_t sb = slotted ? s->slot_base : 0, sv = slotted ? s->slot_vecs : 0;
  if (int e = ar_check(algo, dtype, op, s->rank, s->p, nbytes, buf, buf, scale, sb, sv)) return e;
  uint32_t e = 0;
  if (int rc = fast_begin(s, stream, &e)) return rc;
  return fast_end(s, mp4x_ipc_allreduce_ex2(algo, dtype, op, s->data_ptrs, s->signal_ptrs, s->rank, s->p, nbytes, buf,
                                            buf, e, blocks, nullptr, scale, stream, sb, sv));
}

extern "C" int mp4x_ipc_copy_plan(void* const* data_ptrs, void* const* signal_ptrs, int rank, int p,
                                  const int64_t* stage, int nstage, const int64_t* pull, int npull, const void* src,
                                  void* out, int64_t grid_len, int64_t buf_vecs, uint32_t epoch, int blocks,
                                  const uint32_t* epoch_dev, void* stream);
extern "C" int mp4x_ipc_copy_plan_check(int rank, int p, const int64_t* stage, int nstage, const int64_t* pull,
                                        int npull, const void* src, const void* out, int64_t buf_vecs);

// The same one-call path for a memoised copy plan (the latency tier of broadcast / gather /
// scatter / all-gather, csrc/runtime/ipc.hip k_ipc_copy_plan): error words, capture check, every
// refusal of the launcher — all before the epoch moves — then the stream order, the epoch bump
// and the launch.  src_off / out_off: byte offsets of the plan's source / output from `base` (the
// caller's tensor), or -1 for none.
extern "C" int mp4x_ipc_fast_plan(const FastAr* s, const int64_t* stage, int nstage, const int64_t* pull, int npull,
                                  int64_t src_off, int64_t out_off, void* base, int64_t grid_len, int64_t buf_vecs,
                                  int blocks, void* stream) {
  if (int e = fast_prologue(s)) return e;
  char* b = static_cast<char*>(base);
  const void* src = src_off >= 0 ? b + src_off : nullptr;
  void* out = out_off >= 0 ? b + out_off : nullptr;
  if (!b) return MP4X_E_BADARG;
  if (int e = mp4x_ipc_copy_plan_check(s->rank, s->p, stage, nstage, pull, npull, src, out, buf_vecs)) return e;
  uint32_t e = 0;
  if (int rc = fast_begin(s, stream, &e)) return rc;
  return fast_end(s, mp4x_ipc_copy_plan(s->data_ptrs, s->signal_ptrs, s->rank, s->p, stage, nstage, pull, npull, src,
                                        out, grid_len, buf_vecs, e, blocks, nullptr, stream));
}

extern "C" int mp4x_ipc_reduce_scatter_from(int dtype, int op, void* const* data_ptrs, void* const* signal_ptrs,
                                            int rank, int p, const int64_t* seg_lo, const int64_t* seg_hi,
                                            const void* src, void* out, uint32_t epoch, int blocks,
                                            const uint32_t* epoch_dev, void* stream);
extern "C" int mp4x_ipc_reduce_scatter_from_check(int dtype, int op, int rank, int p, const int64_t* seg_lo,
                                                  const int64_t* seg_hi, const void* src, const void* out);

// The same one-call path for a memoised fused reduce-scatter (csrc/runtime/ipc_rs.hip: the
// kernel stages this rank's range and writes its segment in place).  seg_lo / seg_hi: p segment
// bounds in 16-byte vectors from the range start; src_off / out_off: byte offsets from `base`.
extern "C" int mp4x_ipc_fast_rs(const FastAr* s, int dtype, int op, const int64_t* seg_lo, const int64_t* seg_hi,
                                int64_t src_off, int64_t out_off, void* base, int blocks, void* stream) {
  if (int e = fast_prologue(s)) return e;
  char* b = static_cast<char*>(base);
  if (!b || src_off < 0 || out_off < 0) return MP4X_E_BADARG;
  if (int e = mp4x_ipc_reduce_scatter_from_check(dtype, op, s->rank, s->p, seg_lo, seg_hi, b + src_off, b + out_off))
    return e;
  uint32_t e = 0;
  if (int rc = fast_begin(s, stream, &e)) return rc;
  return fast_end(s, mp4x_ipc_reduce_scatter_from(dtype, op, s->data_ptrs, s->signal_ptrs, s->rank, s->p, seg_lo,
                                                  seg_hi, b + src_off, b + out_off, e, blocks, nullptr, stream));
}

extern "C" int mp4x_ipc_allreduce_ex(int algo, int dtype, int op, void* const* data_ptrs, void* const* signal_ptrs,
                                     int rank, int p, int64_t nbytes, const void* src, void* out, uint32_t epoch,
                                     int blocks, const uint32_t* epoch_dev, float scale, void* stream) {
  return mp4x_ipc_allreduce_ex2(algo, dtype, op, data_ptrs, signal_ptrs, rank, p, nbytes, src, out, epoch, blocks,
                                epoch_dev, scale, stream, 0, 0);
}

// The pre-staged form (no fused copy-in, no scale).
extern "C" int mp4x_ipc_allreduce(int algo, int dtype, int op, void* const* data_ptrs, void* const* signal_ptrs,
                                  int rank, int p, int64_t nbytes, void* out, uint32_t epoch, int blocks,
                                  const uint32_t* epoch_dev, void* stream) {
  return mp4x_ipc_allreduce_ex(algo, dtype, op, data_ptrs, signal_ptrs, rank, p, nbytes, nullptr, out, epoch, blocks,
                               epoch_dev, 1.0f, stream);
}

// Does the IPC allreduce have a kernel for (dtype, op)?  1 / 0.
extern "C" int mp4x_ipc_op_supported(int dtype, int op) {
  return with_dtype(dtype, [&](auto dtc) {
    constexpr int DT = decltype(dtc)::value;
    return with_op<DT>(op, [&](auto) { return 1; }) == 1 ? 1 : 0;
  }) == 1 ? 1 : 0;
}

// Blocks per CU the occupancy API admits for the kernel a call of (algo, dtype, op, p) launches
// (the shared-GPU co-residency budget, mp4x/parallel/occupancy.py).
extern "C" int mp4x_ipc_occupancy_ar(int algo, int dtype, int op, int p, int* blocks_per_cu) {
  int m = 1 << 30;
  int e = with_dtype(dtype, [&](auto dtc) {
    constexpr int DT = decltype(dtc)::value;
    return with_op<DT>(op, [&](auto opc) {
      constexpr int OP = decltype(opc)::value;
      return with_nr(p, [&](auto nrc) {
        constexpr int NR = decltype(nrc)::value;
        if (algo == 0) occ_min(k_ipc_oneshot<DT, OP, NR>, &m);
        else occ_min(k_ipc_twoshot<DT, OP, NR>, &m);
        return 0;
      });
    });
  });
  *blocks_per_cu = m == (1 << 30) ? 0 : m;
  return e;
}
