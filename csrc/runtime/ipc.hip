// Custom xGMI allreduce over IPC-mapped peer buffers (gfx950, one process per GPU).
//
// RCCL moves large messages well; for small and medium messages its ring/tree protocol
// overheads dominate.  These kernels read peer HBM directly through xGMI mappings
// (hipIpcOpenMemHandle) so every one of the 7 links of an MI355X is used at once:
//
//   one-shot : each rank reads all p buffers and reduces in registers (1 hop, p*S read/rank)
//   two-shot : direct reduce-scatter (rank r reduces chunk r from all p buffers into its own
//              buffer) + direct all-gather (rank r pulls chunk c from rank c); 2(p-1)/p*S
//              remote bytes per rank — the bandwidth-optimal full-mesh schedule.
//
// Reference analogue: the fused recv+reduce of the ring reduce-scatter
// (/root/reference/src/main/java/com/fenbi/mp4j/operand/DoubleOperand.java:196) and the
// small-message RPC allreduce (ProcessCommSlave.java:1776-1926) — here as one kernel.
//
// Synchronisation (cdna guide §6 G16, system scope because peers are other GPUs):
//  * every rank owns a Signal block in fine-grained, UNCACHED memory; flags are epochs
//    (monotonic per call, never reset) stored by the signalling lane with a relaxed
//    system-scope atomic store into the PEER's slot, after every wave of the block drained
//    its stores (s_waitcnt vmcnt(0)) + __syncthreads + a system-scope release fence;
//  * waiting lanes poll their own slots with relaxed system-scope loads + s_sleep, then a
//    system-scope acquire;  barriers are per BLOCK: block b of every rank touches exactly
//    the same element offsets, so block b only has to meet block b of the peers;
//  * every spin is bounded (s_memrealtime, 100 MHz): on timeout the block records an
//    error word and exits instead of hanging the GPU;
//  * the STAGED forms' data buffers are uncached as well, so remote reads never see stale L2
//    lines;
//  * the ZERO-COPY forms read and write the peers' own tensors (coarse-grained hipMalloc or
//    memAlloc/VMM memory, L2-cached on their home GPU).  What they rely on: (a) every remote
//    WRITE of a call is followed by the writer's system-scope release (L2 write-back) before
//    its barrier flag, and (b) every block of the home GPU passes a system-scope ACQUIRE after
//    that barrier (block_barrier below: `buffer_inv sc0 sc1`, run by blocks on every XCD), so
//    the lines of its own tensor it cached before the peers' writes (phase 1 reads) are
//    invalidated before the kernel ends — the next kernel reads the peers' values from memory.
//    This is the protocol argument, not an architectural guarantee for every topology: the
//    collective self-test (device_engine._ipc_self_test -> selftest_zero_copy) runs every form
//    TWICE on the same tensor at mesh creation (the second call reduces the first call's
//    results in place, so a stale line would show as a wrong element), autotune repeats that
//    probe per candidate, and tests/test_multigpu_gpu.py runs it across real GPUs.
#include <hip/hip_runtime.h>
#include <cstdlib>

#include "../kernels/common.hpp"
#include "../kernels/fp8.hpp"

namespace mp4x {

constexpr int kIpcMaxRanks = 8;
constexpr int kIpcMaxBlocks = 256;
constexpr int kIpcThreads = 512;
// Epoch tag of the zero-copy protocol (peers' registered tensors instead of the staging
// buffers).  Host epochs live in the low 31 bits; a rank that runs the staged protocol while a
// peer runs the zero-copy one sees the other tag in its flag slot and fails at once instead of
// reading the wrong buffers (registration is collective, but the choice is made per rank).
constexpr uint32_t kZcTag = 0x80000000u;
// The zero-copy PUSH two-shot (k_ipc_twoshot_push) carries a second tag bit; host epochs live in
// the low 30 bits, and a flag whose low bits match but whose tag differs fails the call at once.
constexpr uint32_t kPushTag = 0x40000000u;
constexpr uint32_t kTagMask = kZcTag | kPushTag;

struct alignas(128) Signal {
  uint32_t start[kIpcMaxBlocks][kIpcMaxRanks];
  uint32_t mid[kIpcMaxBlocks][kIpcMaxRanks];
  uint32_t end[kIpcMaxBlocks][kIpcMaxRanks];
  uint32_t error;
  // host-visible copy of `error`: device address of a pinned, mapped host word (0 = none), set
  // once at setup (mp4x_ipc_set_host_error); written on a barrier timeout so the host can fail
  // the NEXT call without any device synchronisation.  Only the owning rank reads this field.
  uint64_t host_err;
};

// Spin bound of every barrier wait, in s_memrealtime ticks (100 MHz); mp4x_ipc_set_spin.
__device__ uint64_t g_ipc_spin_ticks = 1000000000ull;   // 10 s

struct IpcPtrs {
  const void* data[kIpcMaxRanks];   // every rank's data buffer (own one included)
  Signal* sig[kIpcMaxRanks];        // every rank's signal block
};

__device__ __forceinline__ bool block_barrier(uint32_t (*slots)[kIpcMaxRanks] /*Signal::start etc*/,
                                              const IpcPtrs& P, int which, int rank, int p, uint32_t epoch,
                                              Signal* self) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave drains its stores
  __syncthreads();
  __shared__ int s_fail;
  if (threadIdx.x == 0) s_fail = 0;
  __syncthreads();
  const int t = threadIdx.x;
  if (t < p) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");      // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    Signal* peer = P.sig[t];
    uint32_t* slot = which == 0 ? &peer->start[blockIdx.x][rank]
                   : which == 1 ? &peer->mid[blockIdx.x][rank] : &peer->end[blockIdx.x][rank];
    __hip_atomic_store(slot, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = which == 0 ? &self->start[blockIdx.x][t]
                   : which == 1 ? &self->mid[blockIdx.x][t] : &self->end[blockIdx.x][t];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t spin = g_ipc_spin_ticks;
    uint32_t seen;
    while ((seen = __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) != epoch) {
      __builtin_amdgcn_s_sleep(2);
      const bool other_protocol = seen != epoch && ((seen ^ epoch) & ~kTagMask) == 0;
      if (other_protocol || __builtin_amdgcn_s_memrealtime() - t0 > spin) {
        const uint32_t code = other_protocol ? 4u : 1u + (uint32_t)which;
        __hip_atomic_store(&self->error, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        uint32_t* host = reinterpret_cast<uint32_t*>(
            __hip_atomic_load(&self->host_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        if (host) __hip_atomic_store(host, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s_fail = 1;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  (void)slots;
  return s_fail == 0;
}

// NR (rank count) is a template parameter: the NR remote loads are issued unconditionally
// and back to back (no per-load branch, cdna guide §5 trap (c)).
// ``scale`` multiplies the reduced value before the store (the fused 1/p average of a DP
// gradient allreduce); float dtypes only, 1.0 = plain reduction (a wave-uniform branch).
template <int DT, int OP, int NR>
__device__ __forceinline__ u32x4 reduce_vec(const IpcPtrs& P, int64_t v, float scale = 1.0f) {
  using E = Elem<DT>;
  using S = typename E::S;
  using A = typename E::A;
  constexpr int W = 16 / sizeof(S);
  u32x4 r[NR];
#pragma unroll
  for (int k = 0; k < NR; ++k) r[k] = reinterpret_cast<const u32x4*>(P.data[k])[v];   // NR loads in flight
  S s[W];
  __builtin_memcpy(s, &r[0], 16);
  A acc[W];
#pragma unroll
  for (int j = 0; j < W; ++j) acc[j] = E::load(s[j]);
#pragma unroll
  for (int k = 1; k < NR; ++k) {
    S x[W];
    __builtin_memcpy(x, &r[k], 16);
#pragma unroll
    for (int j = 0; j < W; ++j) acc[j] = combine<DT, OP>(acc[j], E::load(x[j]));
  }
  if constexpr (is_float_dt<DT>()) {
    if (scale != 1.0f) {
#pragma unroll
      for (int j = 0; j < W; ++j) acc[j] = acc[j] * (A)scale;
    }
  }
#pragma unroll
  for (int j = 0; j < W; ++j) s[j] = E::store(acc[j]);
  u32x4 o;
  __builtin_memcpy(&o, s, 16);
  return o;
}

// one-shot: out[v] = op over all ranks' data[v]
__device__ __forceinline__ uint32_t resolve_epoch(uint32_t epoch, const uint32_t* epoch_dev) {
  // graph mode: the epoch lives in device memory and is bumped by k_ipc_bump_epoch, the
  // preceding node of the same graph, so every replay gets a fresh, rank-consistent epoch
  // (the protocol tag of a host-passed epoch is kept in graph mode too)
  return epoch_dev ? (__hip_atomic_load(epoch_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) | (epoch & kTagMask))
                   : epoch;
}

__global__ void k_ipc_bump_epoch(uint32_t* epoch_dev) {
  uint32_t e = (*epoch_dev + 1) & ~kTagMask;
  *epoch_dev = e ? e : 1;
}

// src != nullptr: the kernel stages its own input (fused copy-in, one launch instead of a
// memcpy + kernel): block b copies exactly the vectors block b of every peer will read, then
// meets them at the start barrier (whose release fence publishes the copies).
template <int DT, int OP, int NR>
__global__ __launch_bounds__(kIpcThreads) void k_ipc_oneshot(IpcPtrs P, Signal* self, int rank, int64_t nvec,
                                                              u32x4* __restrict__ out, uint32_t epoch,
                                                              const uint32_t* epoch_dev,
                                                              const u32x4* __restrict__ src, float scale) {
  constexpr int p = NR;
  epoch = resolve_epoch(epoch, epoch_dev);
  const int64_t stride = (int64_t)gridDim.x * kIpcThreads;
  if (src) {
    u32x4* mine = reinterpret_cast<u32x4*>(const_cast<void*>(P.data[rank]));
    for (int64_t v = (int64_t)blockIdx.x * kIpcThreads + threadIdx.x; v < nvec; v += stride) mine[v] = src[v];
  }
  if (!block_barrier(nullptr, P, 0, rank, p, epoch, self)) return;
  for (int64_t v = (int64_t)blockIdx.x * kIpcThreads + threadIdx.x; v < nvec; v += stride)
    out[v] = reduce_vec<DT, OP, NR>(P, v, scale);
  block_barrier(nullptr, P, 2, rank, p, epoch, self);
}

// two-shot: direct reduce-scatter into own buffer chunk `rank`, then direct all-gather.
template <int DT, int OP, int NR>
__global__ __launch_bounds__(kIpcThreads) void k_ipc_twoshot(IpcPtrs P, Signal* self, int rank, int64_t nvec,
                                                              u32x4* __restrict__ out, uint32_t epoch,
                                                              const uint32_t* epoch_dev,
                                                              const u32x4* __restrict__ src, float scale) {
  constexpr int p = NR;
  MP4X_DASSERT(rank >= 0 && rank < NR && blockIdx.x < kIpcMaxBlocks);
  epoch = resolve_epoch(epoch, epoch_dev);
  const int64_t chunk = (nvec + p - 1) / p;
  const int64_t stride = (int64_t)gridDim.x * kIpcThreads;
  const int64_t off0 = (int64_t)blockIdx.x * kIpcThreads + threadIdx.x;
  u32x4* mine = reinterpret_cast<u32x4*>(const_cast<void*>(P.data[rank]));
  if (src) {   // fused copy-in: block b stages the chunk offsets block b of every peer reads
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int64_t b = (int64_t)k * chunk;
      const int64_t e = b + chunk < nvec ? b + chunk : nvec;
      for (int64_t v = b + off0; v < e; v += stride) mine[v] = src[v];
    }
  }
  if (!block_barrier(nullptr, P, 0, rank, p, epoch, self)) return;
  {
    const int64_t b = (int64_t)rank * chunk;
    const int64_t e = b + chunk < nvec ? b + chunk : nvec;
    // zero-copy form: `out` IS this rank's registered buffer (== mine), one store per vector
    const bool zc = out == mine;
    for (int64_t v = b + off0; v < e; v += stride) {
      u32x4 o = reduce_vec<DT, OP, NR>(P, v, scale);
      mine[v] = o;
      if (!zc) out[v] = o;
    }
  }
  if (!block_barrier(nullptr, P, 1, rank, p, epoch, self)) return;
  // all-gather: every thread pulls the same chunk offset from ALL p-1 peers at once, so all
  // xGMI links stream concurrently (peer after peer would leave one link busy at a time).
  // k is a compile-time index: no dynamic indexing of the kernarg pointer table.
  for (int64_t v = off0; v < chunk; v += stride) {
    u32x4 x[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int64_t idx = (int64_t)k * chunk + v;
      if (k != rank && idx < nvec) x[k] = reinterpret_cast<const u32x4*>(P.data[k])[idx];
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int64_t idx = (int64_t)k * chunk + v;
      if (k != rank && idx < nvec) out[idx] = x[k];
    }
  }
  block_barrier(nullptr, P, 2, rank, p, epoch, self);
}

// ---------------------------------------------------------------- zero-copy PUSH two-shot
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
struct ScrPtrs {
  void* s[kIpcMaxRanks];
};

template <int DT, int OP, int NR>
__global__ __launch_bounds__(kIpcThreads) void k_ipc_twoshot_push(IpcPtrs P, ScrPtrs S, Signal* self, int rank,
                                                                   int64_t nvec, uint32_t epoch,
                                                                   const uint32_t* epoch_dev, float scale) {
  using E = Elem<DT>;
  using St = typename E::S;
  using A = typename E::A;
  constexpr int W = 16 / sizeof(St);
  constexpr int p = NR;
  MP4X_DASSERT(rank >= 0 && rank < NR && blockIdx.x < kIpcMaxBlocks);
  epoch = resolve_epoch(epoch, epoch_dev);
  const int64_t chunk = (nvec + p - 1) / p;
  const int64_t stride = (int64_t)gridDim.x * kIpcThreads;
  const int64_t off0 = (int64_t)blockIdx.x * kIpcThreads + threadIdx.x;
  u32x4* mine = reinterpret_cast<u32x4*>(const_cast<void*>(P.data[rank]));
  const u32x4* myscr = reinterpret_cast<const u32x4*>(S.s[rank]);
  if (!block_barrier(nullptr, P, 0, rank, p, epoch, self)) return;
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
  if (!block_barrier(nullptr, P, 1, rank, p, epoch, self)) return;
  const int64_t b = (int64_t)rank * chunk;
  const int64_t e = b + chunk < nvec ? b + chunk : nvec;
  for (int64_t v = off0; b + v < e; v += stride) {
    u32x4 r[NR];
#pragma unroll
    for (int q = 0; q < NR; ++q)                   // all local: own chunk + p-1 scratch slots
      r[q] = q == rank ? mine[b + v] : myscr[(int64_t)(q < rank ? q : q - 1) * chunk + v];
    St s0[W];
    __builtin_memcpy(s0, &r[0], 16);
    A acc[W];
#pragma unroll
    for (int j = 0; j < W; ++j) acc[j] = E::load(s0[j]);
#pragma unroll
    for (int q = 1; q < NR; ++q) {                 // rank order: deterministic, = the pull form
      St xq[W];
      __builtin_memcpy(xq, &r[q], 16);
#pragma unroll
      for (int j = 0; j < W; ++j) acc[j] = combine<DT, OP>(acc[j], E::load(xq[j]));
    }
    if constexpr (is_float_dt<DT>()) {
      if (scale != 1.0f) {
#pragma unroll
        for (int j = 0; j < W; ++j) acc[j] = acc[j] * (A)scale;
      }
    }
#pragma unroll
    for (int j = 0; j < W; ++j) s0[j] = E::store(acc[j]);
    u32x4 o;
    __builtin_memcpy(&o, s0, 16);
    mine[b + v] = o;
#pragma unroll
    for (int k = 0; k < NR; ++k)                   // the all-gather half, pushed to every peer
      if (k != rank) reinterpret_cast<u32x4*>(const_cast<void*>(P.data[k]))[b + v] = o;
  }
  block_barrier(nullptr, P, 2, rank, p, epoch, self);
}

template <int DT, int OP>
static int push_nr(const IpcPtrs& P, const ScrPtrs& S, Signal* self, int rank, int p, int64_t nvec, uint32_t epoch,
                   int blocks, const uint32_t* edev, float scale, hipStream_t st) {
#define MP4X_PUSH_CASE(N)                                                                                     \
  case N:                                                                                                     \
    hipLaunchKernelGGL((k_ipc_twoshot_push<DT, OP, N>), dim3(blocks), dim3(kIpcThreads), 0, st, P, S, self,    \
                       rank, nvec, epoch, edev, scale);                                                       \
    return (int)hipGetLastError();
  switch (p) {
    MP4X_PUSH_CASE(2) MP4X_PUSH_CASE(3) MP4X_PUSH_CASE(4) MP4X_PUSH_CASE(5) MP4X_PUSH_CASE(6) MP4X_PUSH_CASE(7)
    MP4X_PUSH_CASE(8)
    default: return MP4X_E_BADARG;
  }
#undef MP4X_PUSH_CASE
}

template <int DT>
static int push_dt(int op, const IpcPtrs& P, const ScrPtrs& S, Signal* self, int rank, int p, int64_t nvec,
                   uint32_t epoch, int blocks, const uint32_t* edev, float scale, hipStream_t st) {
  switch (op) {
    case MP4X_SUM: return push_nr<DT, MP4X_SUM>(P, S, self, rank, p, nvec, epoch, blocks, edev, scale, st);
    case MP4X_MAX:
      if constexpr (is_float_dt<DT>() && DT != MP4X_F64)
        return push_nr<DT, MP4X_MAX>(P, S, self, rank, p, nvec, epoch, blocks, edev, scale, st);
      return MP4X_E_UNSUPPORTED;
    case MP4X_MIN:
      if constexpr (is_float_dt<DT>() && DT != MP4X_F64)
        return push_nr<DT, MP4X_MIN>(P, S, self, rank, p, nvec, epoch, blocks, edev, scale, st);
      return MP4X_E_UNSUPPORTED;
    default: return MP4X_E_UNSUPPORTED;
  }
}

// ---------------------------------------------------------------- direct reduce-scatter / all-gather
// The two halves of the two-shot as collectives of their own, over RAGGED per-rank ranges
// (reduceScatterArray counts / allgatherArray froms-tos), in 16-byte vectors of the staged
// buffers.  Reduce-scatter: rank r reads [lo_r, hi_r) from ALL p buffers at once and reduces
// in registers (the fused peer-load + reduce of SURVEY C7).  All-gather: rank r pulls every
// peer's segment, the same offset from all p-1 peers per step, so all links stream at once.
struct Segs {
  int64_t lo[kIpcMaxRanks];
  int64_t hi[kIpcMaxRanks];
};

// src != nullptr: fused staging — block b copies, for EVERY rank's segment k, the vectors block b
// of rank k will read from this buffer (segment-relative grid stride), then meets the peers.
template <int DT, int OP, int NR>
__global__ __launch_bounds__(kIpcThreads) void k_ipc_reduce_range(IpcPtrs P, Signal* self, int rank, int64_t lo,
                                                                   int64_t hi, u32x4* __restrict__ out,
                                                                   uint32_t epoch, const uint32_t* epoch_dev,
                                                                   const u32x4* __restrict__ src, Segs S) {
  constexpr int p = NR;
  MP4X_DASSERT(rank >= 0 && rank < NR && lo <= hi);
  epoch = resolve_epoch(epoch, epoch_dev);
  const int64_t stride = (int64_t)gridDim.x * kIpcThreads;
  if (src) {
    u32x4* mine = reinterpret_cast<u32x4*>(const_cast<void*>(P.data[rank]));
    const int64_t off0 = (int64_t)blockIdx.x * kIpcThreads + threadIdx.x;
#pragma unroll
    for (int k = 0; k < NR; ++k)
      for (int64_t v = S.lo[k] + off0; v < S.hi[k]; v += stride) mine[v] = src[v];
  }
  if (!block_barrier(nullptr, P, 0, rank, p, epoch, self)) return;
  for (int64_t v = lo + (int64_t)blockIdx.x * kIpcThreads + threadIdx.x; v < hi; v += stride)
    out[v - lo] = reduce_vec<DT, OP, NR>(P, v);
  block_barrier(nullptr, P, 2, rank, p, epoch, self);
}

template <int NR>
__global__ __launch_bounds__(kIpcThreads) void k_ipc_gather(IpcPtrs P, Signal* self, int rank, Segs S,
                                                             int64_t maxlen, u32x4* __restrict__ out, uint32_t epoch,
                                                             const uint32_t* epoch_dev) {
  constexpr int p = NR;
  MP4X_DASSERT(rank >= 0 && rank < NR);
  epoch = resolve_epoch(epoch, epoch_dev);
  if (!block_barrier(nullptr, P, 0, rank, p, epoch, self)) return;
  const int64_t stride = (int64_t)gridDim.x * kIpcThreads;
  for (int64_t v = (int64_t)blockIdx.x * kIpcThreads + threadIdx.x; v < maxlen; v += stride) {
    u32x4 x[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k)
      if (k != rank && S.lo[k] + v < S.hi[k]) x[k] = reinterpret_cast<const u32x4*>(P.data[k])[S.lo[k] + v];
#pragma unroll
    for (int k = 0; k < NR; ++k)
      if (k != rank && S.lo[k] + v < S.hi[k]) out[S.lo[k] + v] = x[k];
  }
  block_barrier(nullptr, P, 2, rank, p, epoch, self);
}

// ---------------------------------------------------------------- copy plans (bcast / scatter / gather)
// The data-movement collectives as ONE kernel per call: a plan of up to kIpcMaxRanks "stage"
// items (this rank's input -> its own buffer, fused copy-in) and up to kIpcMaxRanks "pull" items
// (a peer's buffer -> this rank's output, over xGMI, all pulls interleaved so every link
// streams).  Every item is walked with the same grid-stride relative index on every rank, so
// the vectors block b stages are exactly the vectors block b of the peers pull: per-block
// barriers suffice, as in the two-shot.  Units: 16-byte vectors.
struct CopyItem {
  int64_t src_off, dst_off, len;
  int64_t peer;          // pull: source rank; stage: unused
};
struct CopyPlan {
  CopyItem stage[kIpcMaxRanks];
  CopyItem pull[kIpcMaxRanks];
  int nstage, npull;
};

__global__ __launch_bounds__(kIpcThreads) void k_ipc_copy_plan(IpcPtrs P, Signal* self, int rank, int p,
                                                                CopyPlan plan, const u32x4* __restrict__ src,
                                                                u32x4* __restrict__ out, uint32_t epoch,
                                                                const uint32_t* epoch_dev) {
  epoch = resolve_epoch(epoch, epoch_dev);
  const int64_t stride = (int64_t)gridDim.x * kIpcThreads;
  const int64_t off0 = (int64_t)blockIdx.x * kIpcThreads + threadIdx.x;
  u32x4* mine = reinterpret_cast<u32x4*>(const_cast<void*>(P.data[rank]));
  for (int i = 0; i < plan.nstage; ++i) {
    const CopyItem it = plan.stage[i];
    MP4X_DASSERT(it.len >= 0);
    for (int64_t v = off0; v < it.len; v += stride) mine[it.dst_off + v] = src[it.src_off + v];
  }
  if (!block_barrier(nullptr, P, 0, rank, p, epoch, self)) return;
  int64_t maxlen = 0;
  for (int i = 0; i < plan.npull; ++i) maxlen = plan.pull[i].len > maxlen ? plan.pull[i].len : maxlen;
  for (int64_t v = off0; v < maxlen; v += stride) {
    u32x4 x[kIpcMaxRanks];
#pragma unroll
    for (int i = 0; i < kIpcMaxRanks; ++i)           // every pull's vector in flight at once
      if (i < plan.npull && v < plan.pull[i].len)
        x[i] = reinterpret_cast<const u32x4*>(P.data[plan.pull[i].peer])[plan.pull[i].src_off + v];
#pragma unroll
    for (int i = 0; i < kIpcMaxRanks; ++i)
      if (i < plan.npull && v < plan.pull[i].len) out[plan.pull[i].dst_off + v] = x[i];
  }
  block_barrier(nullptr, P, 2, rank, p, epoch, self);
}

// ---------------------------------------------------------------- fused fp8 two-shot (K6 on xGMI)
// Compressed allreduce with the block-scaled e4m3 codec on the links, in ONE kernel per piece
// (the quantise of this rank's input into its own IPC buffer runs just before, stream-ordered):
//   RS: for every 256-element quant block of chunk `rank`, each wave pulls the block's 256 fp8
//       bytes + scale from ALL p buffers at once (every xGMI link busy), dequantises and sums in
//       f32 registers, re-quantises (wave amax -> scale) into its OWN buffer, and writes the
//       dequantised result of that re-quantised block to `out` (so this rank's chunk holds
//       exactly what the peers will decode);
//   AG: every wave pulls the same block offset of every peer's chunk at once, dequantises
//       straight into `out`.
// Versus the RCCL form (all-to-all + fused dequant-reduce-requant + all-gather + dequant) no
// landing buffers are written and read back, and p-1 scale messages disappear.  Layout of the
// buffers: q bytes [0, M) then f32 scales at `soff` bytes, one per quant block; block j of chunk
// k is global quant block k * cb + j.  Block b of every rank visits the same chunk-relative j
// values in both phases, so the per-block barriers are the two-shot's.
// Wide form: every lane moves 16 bytes (16 e4m3 values) per peer per step, so one wave covers
// FOUR quant blocks (lanes 16g..16g+15 hold block g) and a block's amax is a 16-lane reduction;
// the four scales a wave needs sit in one 16-byte span, so the scale load is one request per
// wave.  Per element the arithmetic (rank-ordered FMAs, amax, e4m3 rounding) is the K6 codec's,
// so the result stays bit-identical to quantise -> dequant-reduce-requant -> dequantise.
__device__ __forceinline__ float group16_max(float v) {
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));   // stays inside the 16-lane group
  return v;
}

// Output of one wave's 1024 dequantised values (4 consecutive quant blocks starting at
// global block b0): lane l holds values [16 l, 16 l + 16) — a 64-byte stride between lanes, so
// storing straight from registers would leave every store instruction 16 bytes per line.  The
// values go through a wave-private LDS tile (20-float lane pitch: 16-byte aligned, spread over
// the banks) and leave as 16-byte-per-lane CONTIGUOUS stores (1 KB of f32 per instruction).
constexpr int kFp8LdsPitch = 20;
template <int DT>
__device__ __forceinline__ void fp8_wave_store(float* tile, const float (&y)[16], int lane, void* out,
                                               int64_t b0, int64_t cb_end, int64_t n) {
#pragma unroll
  for (int d = 0; d < 4; ++d)
    *reinterpret_cast<float4*>(tile + lane * kFp8LdsPitch + d * 4) = make_float4(y[4 * d], y[4 * d + 1],
                                                                                  y[4 * d + 2], y[4 * d + 3]);
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the wave's LDS writes are done
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const int e = (d * 64 + lane) * 4;                  // value index inside the wave's 1024
    const float4 v = *reinterpret_cast<const float4*>(tile + (e >> 4) * kFp8LdsPitch + (e & 15));
    const int64_t blk = b0 + (e >> 8);
    if (blk < cb_end) {
      float x[4] = {v.x, v.y, v.z, v.w};
      store4<DT>(out, b0 * kQBlock + e, n, x);
    }
  }
  __builtin_amdgcn_wave_barrier();      // the tile is rewritten by this wave's next step
}

template <int DT, int NR>
__global__ __launch_bounds__(kIpcThreads) void k_ipc_fp8_twoshot(IpcPtrs P, Signal* self, int rank, int64_t cb,
                                                                  int64_t soff, void* __restrict__ out, int64_t n,
                                                                  uint32_t epoch, const uint32_t* epoch_dev,
                                                                  float scale) {
  constexpr int p = NR;
  MP4X_DASSERT(rank >= 0 && rank < NR && blockIdx.x < kIpcMaxBlocks);
  __shared__ __attribute__((aligned(16))) float s_tile[kIpcThreads * kFp8LdsPitch];
  epoch = resolve_epoch(epoch, epoch_dev);
  if (!block_barrier(nullptr, P, 0, rank, p, epoch, self)) return;
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;                 // quant block of this lane within the wave's 4
  const int sub = lane & 15;               // 16-byte slot inside the 256-byte block
  constexpr int kWaves = kIpcThreads / 64;
  float* tile = s_tile + (threadIdx.x >> 6) * 64 * kFp8LdsPitch;
  const int64_t w0 = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * kWaves;
  const int64_t nquad = (cb + 3) / 4;      // wave steps per chunk
  {
    u32x4* myq = reinterpret_cast<u32x4*>(const_cast<void*>(P.data[rank]));
    float* mys = reinterpret_cast<float*>(reinterpret_cast<char*>(myq) + soff);
    for (int64_t t = w0; t < nquad; t += nw) {
      const int64_t j = t * 4 + g;                       // chunk-relative quant block
      const bool live = j < cb;
      const int64_t b = (int64_t)rank * cb + (live ? j : 0);   // global quant block
      u32x4 w[NR];
      float sc[NR];
#pragma unroll
      for (int k = 0; k < NR; ++k) {                      // every peer's 16 bytes in flight at once
        const u32x4* q = reinterpret_cast<const u32x4*>(P.data[k]);
        w[k] = live ? q[b * 16 + sub] : u32x4{0u, 0u, 0u, 0u};
        sc[k] = live ? reinterpret_cast<const float*>(reinterpret_cast<const char*>(q) + soff)[b] : 0.0f;
      }
      float acc[4][4];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        acc[d][0] = acc[d][1] = acc[d][2] = acc[d][3] = 0.0f;
#pragma unroll
        for (int k = 0; k < NR; ++k) fp8_fma_acc(w[k][d], sc[k], acc[d]);   // rank order: deterministic
      }
      if (scale != 1.0f) {                                // fused average, before the re-quantisation
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[d][e] *= scale;
      }
      float m = 0.0f;
#pragma unroll
      for (int d = 0; d < 4; ++d)
        m = fmaxf(m, fmaxf(fmaxf(fabsf(acc[d][0]), fabsf(acc[d][1])), fmaxf(fabsf(acc[d][2]), fabsf(acc[d][3]))));
      m = group16_max(m);
      const float bscale = m > 0.0f ? m / kFp8Max : 1.0f;
      const float inv = 1.0f / bscale;
      u32x4 qq;
#pragma unroll
      for (int d = 0; d < 4; ++d) qq[d] = pack_fp8(acc[d], inv);
      if (live) {
        myq[b * 16 + sub] = qq;                           // read by the peers after the mid barrier
        if (sub == 0) mys[b] = bscale;
      }
      float y[16];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        float yy[4];
        unpack_fp8(qq[d], bscale, yy);
        y[4 * d] = yy[0]; y[4 * d + 1] = yy[1]; y[4 * d + 2] = yy[2]; y[4 * d + 3] = yy[3];
      }
      fp8_wave_store<DT>(tile, y, lane, out, (int64_t)rank * cb + t * 4, (int64_t)rank * cb + cb, n);
    }
  }
  if (!block_barrier(nullptr, P, 1, rank, p, epoch, self)) return;
  for (int64_t t = w0; t < nquad; t += nw) {
    const int64_t j = t * 4 + g;
    const bool live = j < cb;
    u32x4 w[NR];
    float sc[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      if (k == rank) continue;
      const u32x4* q = reinterpret_cast<const u32x4*>(P.data[k]);
      const int64_t b = (int64_t)k * cb + (live ? j : 0);
      w[k] = live ? q[b * 16 + sub] : u32x4{0u, 0u, 0u, 0u};
      sc[k] = live ? reinterpret_cast<const float*>(reinterpret_cast<const char*>(q) + soff)[b] : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      if (k == rank) continue;
      float y[16];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        float yy[4];
        unpack_fp8(w[k][d], sc[k], yy);
        y[4 * d] = yy[0]; y[4 * d + 1] = yy[1]; y[4 * d + 2] = yy[2]; y[4 * d + 3] = yy[3];
      }
      fp8_wave_store<DT>(tile, y, lane, out, (int64_t)k * cb + t * 4, (int64_t)k * cb + cb, n);
    }
  }
  block_barrier(nullptr, P, 2, rank, p, epoch, self);
}

// The r1 form (4 bytes per lane per peer, one wave per quant block), kept for A/B measurement
// (MP4X_FP8_NARROW=1); bit-identical results.
template <int DT, int NR>
__global__ __launch_bounds__(kIpcThreads) void k_ipc_fp8_twoshot_narrow(IpcPtrs P, Signal* self, int rank, int64_t cb,
                                                                  int64_t soff, void* __restrict__ out, int64_t n,
                                                                  uint32_t epoch, const uint32_t* epoch_dev,
                                                                  float scale) {
  constexpr int p = NR;
  MP4X_DASSERT(rank >= 0 && rank < NR && blockIdx.x < kIpcMaxBlocks);
  epoch = resolve_epoch(epoch, epoch_dev);
  if (!block_barrier(nullptr, P, 0, rank, p, epoch, self)) return;
  const int lane = threadIdx.x & 63;
  constexpr int kWaves = kIpcThreads / 64;
  const int64_t w0 = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * kWaves;
  {
    uint32_t* myq = reinterpret_cast<uint32_t*>(const_cast<void*>(P.data[rank]));
    float* mys = reinterpret_cast<float*>(reinterpret_cast<char*>(myq) + soff);
    for (int64_t j = w0; j < cb; j += nw) {
      const int64_t b = (int64_t)rank * cb + j;          // global quant block
      uint32_t w[NR];
      float sc[NR];
#pragma unroll
      for (int k = 0; k < NR; ++k) {                      // every peer's block in flight at once
        const uint32_t* q = reinterpret_cast<const uint32_t*>(P.data[k]);
        w[k] = q[b * 64 + lane];
        sc[k] = reinterpret_cast<const float*>(reinterpret_cast<const char*>(q) + soff)[b];
      }
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < NR; ++k) fp8_fma_acc(w[k], sc[k], acc);   // rank order: deterministic
      if (scale != 1.0f) {                                // fused average, before the re-quantisation
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] *= scale;
      }
      float m = fmaxf(fmaxf(fabsf(acc[0]), fabsf(acc[1])), fmaxf(fabsf(acc[2]), fabsf(acc[3])));
      m = wave_max(m);
      const float bscale = m > 0.0f ? m / kFp8Max : 1.0f;
      const uint32_t qq = pack_fp8(acc, 1.0f / bscale);
      myq[b * 64 + lane] = qq;                            // read by the peers after the mid barrier
      if (lane == 0) mys[b] = bscale;
      float y[4];
      unpack_fp8(qq, bscale, y);
      store4<DT>(out, b * kQBlock + lane * 4, n, y);
    }
  }
  if (!block_barrier(nullptr, P, 1, rank, p, epoch, self)) return;
  for (int64_t j = w0; j < cb; j += nw) {
    uint32_t w[NR];
    float sc[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      if (k == rank) continue;
      const uint32_t* q = reinterpret_cast<const uint32_t*>(P.data[k]);
      const int64_t b = (int64_t)k * cb + j;
      w[k] = q[b * 64 + lane];
      sc[k] = reinterpret_cast<const float*>(reinterpret_cast<const char*>(q) + soff)[b];
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      if (k == rank) continue;
      const int64_t b = (int64_t)k * cb + j;
      if (b * kQBlock >= n) continue;
      float y[4];
      unpack_fp8(w[k], sc[k], y);
      store4<DT>(out, b * kQBlock + lane * 4, n, y);
    }
  }
  block_barrier(nullptr, P, 2, rank, p, epoch, self);
}

template <int DT>
static int fp8_nr(const IpcPtrs& P, Signal* self, int rank, int p, int64_t cb, int64_t soff, void* out, int64_t n,
                  uint32_t epoch, const uint32_t* edev, float scale, int blocks, hipStream_t st, bool narrow) {
#define MP4X_FP8_CASE(N)                                                                                     \
  case N:                                                                                                    \
    if (narrow)                                                                                              \
      hipLaunchKernelGGL((k_ipc_fp8_twoshot_narrow<DT, N>), dim3(blocks), dim3(kIpcThreads), 0, st, P, self,   \
                         rank, cb, soff, out, n, epoch, edev, scale);                                        \
    else                                                                                                     \
      hipLaunchKernelGGL((k_ipc_fp8_twoshot<DT, N>), dim3(blocks), dim3(kIpcThreads), 0, st, P, self, rank,   \
                         cb, soff, out, n, epoch, edev, scale);                                              \
    return (int)hipGetLastError();
  switch (p) {
    MP4X_FP8_CASE(2) MP4X_FP8_CASE(3) MP4X_FP8_CASE(4) MP4X_FP8_CASE(5) MP4X_FP8_CASE(6) MP4X_FP8_CASE(7)
    MP4X_FP8_CASE(8)
    default: return MP4X_E_BADARG;
  }
#undef MP4X_FP8_CASE
}

// Per-call launch options of the one-/two-shot allreduce.
struct LaunchOpts {
  const uint32_t* edev;   // device epoch (graph mode) or nullptr
  const u32x4* src;       // fused copy-in source or nullptr (pre-staged / zero-copy)
  float scale;            // applied to the reduced value (1 = none)
};

template <int DT, int OP, int NR>
static int launch_nr(int algo, const IpcPtrs& P, Signal* self, int rank, int64_t nvec, void* out, uint32_t epoch,
                     int blocks, hipStream_t st, const LaunchOpts& o) {
  if (algo == 0)
    hipLaunchKernelGGL((k_ipc_oneshot<DT, OP, NR>), dim3(blocks), dim3(kIpcThreads), 0, st, P, self, rank, nvec,
                       (u32x4*)out, epoch, o.edev, o.src, o.scale);
  else
    hipLaunchKernelGGL((k_ipc_twoshot<DT, OP, NR>), dim3(blocks), dim3(kIpcThreads), 0, st, P, self, rank, nvec,
                       (u32x4*)out, epoch, o.edev, o.src, o.scale);
  return (int)hipGetLastError();
}

template <int DT, int OP>
static int launch_ipc(int algo, const IpcPtrs& P, Signal* self, int rank, int p, int64_t nvec, void* out,
                      uint32_t epoch, int blocks, hipStream_t st, const LaunchOpts& o) {
  switch (p) {
    case 2: return launch_nr<DT, OP, 2>(algo, P, self, rank, nvec, out, epoch, blocks, st, o);
    case 3: return launch_nr<DT, OP, 3>(algo, P, self, rank, nvec, out, epoch, blocks, st, o);
    case 4: return launch_nr<DT, OP, 4>(algo, P, self, rank, nvec, out, epoch, blocks, st, o);
    case 5: return launch_nr<DT, OP, 5>(algo, P, self, rank, nvec, out, epoch, blocks, st, o);
    case 6: return launch_nr<DT, OP, 6>(algo, P, self, rank, nvec, out, epoch, blocks, st, o);
    case 7: return launch_nr<DT, OP, 7>(algo, P, self, rank, nvec, out, epoch, blocks, st, o);
    case 8: return launch_nr<DT, OP, 8>(algo, P, self, rank, nvec, out, epoch, blocks, st, o);
    default: return MP4X_E_BADARG;
  }
}

// IPC path covers the common gradient / statistic reductions; other (dtype, op) pairs use
// the RCCL or a2a schedules.
template <int DT>
static int ipc_dt(int op, int algo, const IpcPtrs& P, Signal* self, int rank, int p, int64_t nvec, void* out,
                  uint32_t epoch, int blocks, hipStream_t st, const LaunchOpts& o) {
  switch (op) {
    case MP4X_SUM: return launch_ipc<DT, MP4X_SUM>(algo, P, self, rank, p, nvec, out, epoch, blocks, st, o);
    case MP4X_MAX:
      if constexpr (is_float_dt<DT>() && DT != MP4X_F64)
        return launch_ipc<DT, MP4X_MAX>(algo, P, self, rank, p, nvec, out, epoch, blocks, st, o);
      return MP4X_E_UNSUPPORTED;
    case MP4X_MIN:
      if constexpr (is_float_dt<DT>() && DT != MP4X_F64)
        return launch_ipc<DT, MP4X_MIN>(algo, P, self, rank, p, nvec, out, epoch, blocks, st, o);
      return MP4X_E_UNSUPPORTED;
    default: return MP4X_E_UNSUPPORTED;
  }
}

}  // namespace mp4x

using namespace mp4x;

extern "C" size_t mp4x_ipc_signal_bytes(void) { return sizeof(Signal); }

// Fine-grained, uncached device allocation (signal blocks and IPC data buffers), zeroed.
extern "C" int mp4x_ipc_alloc(size_t bytes, void** ptr) {
  hipError_t e = hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*ptr, 0, bytes);
  if (e != hipSuccess) return (int)e;
  return (int)hipDeviceSynchronize();
}

extern "C" int mp4x_ipc_free(void* ptr) { return (int)hipFree(ptr); }

// Staging data buffer of an IPC instance, zeroed: ``coarse`` = 0 -> fine-grained uncached (the
// default: peers' reads never meet a stale L2 line); 1 -> plain coarse-grained hipMalloc memory,
// L2-cached on its home GPU, kept coherent by the kernels' system-scope release / acquire at
// every barrier (the zero-copy protocol's argument).  MP4X_IPC_DATA_MEM selects it (A/B).
extern "C" int mp4x_ipc_alloc_data(size_t bytes, int coarse, void** ptr) {
  if (!coarse) return mp4x_ipc_alloc(bytes, ptr);
  hipError_t e = hipMalloc(ptr, bytes);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*ptr, 0, bytes);
  if (e != hipSuccess) return (int)e;
  return (int)hipDeviceSynchronize();
}

// Plain (coarse-grained) device allocation, the kind the PyTorch caching allocator makes: the
// self-test of the zero-copy protocol runs on memory like the caller tensors it will map.
extern "C" int mp4x_dev_alloc(size_t bytes, void** ptr) { return (int)hipMalloc(ptr, bytes); }

// Pinned host word the kernels can write (mapped, coherent): *host_ptr for the CPU,
// *dev_ptr for the kernels.  Zeroed.
extern "C" int mp4x_host_word_alloc(void** host_ptr, void** dev_ptr) {
  hipError_t e = hipHostMalloc(host_ptr, 64, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return (int)e;
  __builtin_memset(*host_ptr, 0, 64);
  return (int)hipHostGetDevicePointer(dev_ptr, *host_ptr, 0);
}

extern "C" int mp4x_host_word_free(void* host_ptr) { return (int)hipHostFree(host_ptr); }

// Register the host-visible error word of a signal block (device address from
// mp4x_host_word_alloc; nullptr to detach).
extern "C" int mp4x_ipc_set_host_error(void* signal, void* dev_word) {
  const uint64_t v = (uint64_t)(uintptr_t)dev_word;
  hipError_t e = hipMemcpy((char*)signal + offsetof(Signal, host_err), &v, sizeof(v), hipMemcpyHostToDevice);
  return (int)e;
}

// Barrier spin bound for every IPC kernel launched afterwards (process-wide), in seconds.
extern "C" int mp4x_ipc_set_spin(double seconds) {
  if (!(seconds > 0.0)) return MP4X_E_BADARG;
  const uint64_t ticks = (uint64_t)(seconds * 1.0e8);
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_ipc_spin_ticks), &ticks, sizeof(ticks), 0, hipMemcpyHostToDevice);
}

// PCI bus id of the current device: ranks compare them to detect a GPU shared by several
// ranks (single-GPU rehearsal), where the per-block barriers need every rank's blocks
// co-resident and the block count must shrink accordingly.
extern "C" int mp4x_device_pci_id(char* buf, int len) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  return (int)hipDeviceGetPCIBusId(buf, len, dev);
}

extern "C" int mp4x_ipc_handle_size(void) { return (int)sizeof(hipIpcMemHandle_t); }

// Base and size of the allocation that contains `ptr` (IPC handles name whole allocations:
// a caller tensor inside a caching-allocator segment is exported as (segment handle, offset)).
extern "C" int mp4x_mem_range(void* ptr, void** base, size_t* size) {
  hipDeviceptr_t b = nullptr;
  size_t sz = 0;
  hipError_t e = hipMemGetAddressRange(&b, &sz, (hipDeviceptr_t)ptr);
  *base = (void*)b;
  *size = sz;
  return (int)e;
}

extern "C" int mp4x_ipc_get_handle(void* ptr, void* handle_out) {
  return (int)hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle_out), ptr);
}

extern "C" int mp4x_ipc_open_handle(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

extern "C" int mp4x_ipc_close_handle(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

extern "C" int mp4x_memcpy_async(void* dst, const void* src, size_t bytes, void* stream) {
  return (int)hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
}

extern "C" int mp4x_ipc_read_error(void* signal, uint32_t* err) {
  return (int)hipMemcpy(err, (char*)signal + offsetof(Signal, error), 4, hipMemcpyDeviceToHost);
}

// The error word read on `stream` (a private non-blocking stream, so a poll from the collective
// watchdog thread never serialises with the caller's streams); clear != 0 resets it after the
// read, so one timed-out barrier is reported once instead of poisoning every later check.
extern "C" int mp4x_ipc_error_word(void* signal, uint32_t* err, int clear, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  char* w = (char*)signal + offsetof(Signal, error);
  hipError_t e = hipMemcpyAsync(err, w, 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && clear) e = hipMemsetAsync(w, 0, 4, st);
  if (e != hipSuccess) return (int)e;
  return (int)hipStreamSynchronize(st);
}

// algo 0 = one-shot, 1 = two-shot.  data_ptrs / signal_ptrs: p entries (own rank included,
// peers as mapped by mp4x_ipc_open_handle).  nbytes must be a multiple of 16; the caller has
// already placed this rank's input in data_ptrs[rank] (stream-ordered before this launch).
extern "C" int mp4x_ipc_bump_epoch(uint32_t* epoch_dev, void* stream) {
  hipLaunchKernelGGL(k_ipc_bump_epoch, dim3(1), dim3(1), 0, (hipStream_t)stream, epoch_dev);
  return (int)hipGetLastError();
}

// epoch_dev == NULL: `epoch` (host counter) is used.  epoch_dev != NULL: graph-capturable form,
// the kernel reads the epoch from device memory (bump it with mp4x_ipc_bump_epoch first).
// src != NULL: this rank's input (16-byte aligned) is copied into its own buffer INSIDE the
// kernel (fused copy-in: one launch per call); NULL: already staged, or zero-copy (the data
// pointers are the registered caller tensors and out == data_ptrs[rank]).  scale != 1: the
// reduced value is multiplied by it before it is stored (fused average; float dtypes only).
extern "C" int mp4x_ipc_allreduce_ex(int algo, int dtype, int op, void* const* data_ptrs, void* const* signal_ptrs,
                                     int rank, int p, int64_t nbytes, const void* src, void* out, uint32_t epoch,
                                     int blocks, const uint32_t* epoch_dev, float scale, void* stream) {
  if (p < 2 || p > kIpcMaxRanks || rank < 0 || rank >= p || (nbytes & 15) || nbytes <= 0) return MP4X_E_BADARG;
  if (((uintptr_t)out & 15) || ((uintptr_t)src & 15)) return MP4X_E_BADARG;
  if (scale != 1.0f && !(dtype == MP4X_F32 || dtype == MP4X_F64 || dtype == MP4X_BF16 || dtype == MP4X_F16))
    return MP4X_E_BADARG;
  IpcPtrs P;
  for (int k = 0; k < kIpcMaxRanks; ++k) {
    P.data[k] = k < p ? data_ptrs[k] : nullptr;
    P.sig[k] = k < p ? (Signal*)signal_ptrs[k] : nullptr;
    if (k < p && (((uintptr_t)P.data[k] & 15) || !P.sig[k])) return MP4X_E_BADARG;
  }
  int64_t nvec = nbytes / 16;
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
  const LaunchOpts o{epoch_dev, (const u32x4*)src, scale};
  // element count per 16-byte vector is encoded in the dtype; nvec is the vector count
  switch (dtype) {
    case MP4X_F64: return ipc_dt<MP4X_F64>(op, algo, P, self, rank, p, nvec, out, epoch, blocks, st, o);
    case MP4X_F32: return ipc_dt<MP4X_F32>(op, algo, P, self, rank, p, nvec, out, epoch, blocks, st, o);
    case MP4X_I64: return ipc_dt<MP4X_I64>(op, algo, P, self, rank, p, nvec, out, epoch, blocks, st, o);
    case MP4X_I32: return ipc_dt<MP4X_I32>(op, algo, P, self, rank, p, nvec, out, epoch, blocks, st, o);
    case MP4X_BF16: return ipc_dt<MP4X_BF16>(op, algo, P, self, rank, p, nvec, out, epoch, blocks, st, o);
    case MP4X_F16: return ipc_dt<MP4X_F16>(op, algo, P, self, rank, p, nvec, out, epoch, blocks, st, o);
    default: return MP4X_E_UNSUPPORTED;
  }
}

// The pre-staged form (no fused copy-in, no scale).
extern "C" int mp4x_ipc_allreduce(int algo, int dtype, int op, void* const* data_ptrs, void* const* signal_ptrs,
                                  int rank, int p, int64_t nbytes, void* out, uint32_t epoch, int blocks,
                                  const uint32_t* epoch_dev, void* stream) {
  return mp4x_ipc_allreduce_ex(algo, dtype, op, data_ptrs, signal_ptrs, rank, p, nbytes, nullptr, out, epoch, blocks,
                               epoch_dev, 1.0f, stream);
}

// Zero-copy PUSH two-shot (see k_ipc_twoshot_push): data_ptrs = every rank's registered tensor
// (this rank's own included; the result replaces it), scratch_ptrs = every rank's receive
// scratch of at least (p - 1) * ceil(nbytes / 16 / p) 16-byte vectors.
extern "C" int mp4x_ipc_allreduce_push(int dtype, int op, void* const* data_ptrs, void* const* scratch_ptrs,
                                       void* const* signal_ptrs, int rank, int p, int64_t nbytes, uint32_t epoch,
                                       int blocks, const uint32_t* epoch_dev, float scale, void* stream) {
  if (p < 2 || p > kIpcMaxRanks || rank < 0 || rank >= p || (nbytes & 15) || nbytes <= 0) return MP4X_E_BADARG;
  if (scale != 1.0f && !(dtype == MP4X_F32 || dtype == MP4X_F64 || dtype == MP4X_BF16 || dtype == MP4X_F16))
    return MP4X_E_BADARG;
  IpcPtrs P;
  ScrPtrs S;
  for (int k = 0; k < kIpcMaxRanks; ++k) {
    P.data[k] = k < p ? data_ptrs[k] : nullptr;
    P.sig[k] = k < p ? (Signal*)signal_ptrs[k] : nullptr;
    S.s[k] = k < p ? scratch_ptrs[k] : nullptr;
    if (k < p && (((uintptr_t)P.data[k] & 15) || ((uintptr_t)S.s[k] & 15) || !P.sig[k] || !S.s[k]))
      return MP4X_E_BADARG;
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
  switch (dtype) {
    case MP4X_F64: return push_dt<MP4X_F64>(op, P, S, self, rank, p, nvec, epoch, blocks, epoch_dev, scale, st);
    case MP4X_F32: return push_dt<MP4X_F32>(op, P, S, self, rank, p, nvec, epoch, blocks, epoch_dev, scale, st);
    case MP4X_I64: return push_dt<MP4X_I64>(op, P, S, self, rank, p, nvec, epoch, blocks, epoch_dev, scale, st);
    case MP4X_I32: return push_dt<MP4X_I32>(op, P, S, self, rank, p, nvec, epoch, blocks, epoch_dev, scale, st);
    case MP4X_BF16: return push_dt<MP4X_BF16>(op, P, S, self, rank, p, nvec, epoch, blocks, epoch_dev, scale, st);
    case MP4X_F16: return push_dt<MP4X_F16>(op, P, S, self, rank, p, nvec, epoch, blocks, epoch_dev, scale, st);
    default: return MP4X_E_UNSUPPORTED;
  }
}

static int ipc_prepare(void* const* data_ptrs, void* const* signal_ptrs, int rank, int p, IpcPtrs* P) {
  if (p < 2 || p > kIpcMaxRanks || rank < 0 || rank >= p) return MP4X_E_BADARG;
  for (int k = 0; k < kIpcMaxRanks; ++k) {
    P->data[k] = k < p ? data_ptrs[k] : nullptr;
    P->sig[k] = k < p ? (Signal*)signal_ptrs[k] : nullptr;
    if (k < p && (((uintptr_t)P->data[k] & 15) || !P->sig[k])) return MP4X_E_BADARG;
  }
  return 0;
}

static int ipc_blocks(int blocks, int64_t nvec) {
  if (blocks <= 0) {
    int64_t b = (nvec + kIpcThreads - 1) / kIpcThreads;
    blocks = (int)(b < 1 ? 1 : (b > kIpcMaxBlocks ? kIpcMaxBlocks : b));
  }
  return blocks > kIpcMaxBlocks ? kIpcMaxBlocks : blocks;
}

static thread_local const void* g_rs_src = nullptr;   // fused RS staging source (nullptr: pre-staged)
static thread_local Segs g_rs_segs;

template <int DT, int OP>
static int rs_nr(const IpcPtrs& P, Signal* self, int rank, int p, int64_t lo, int64_t hi, void* out, uint32_t epoch,
                 const uint32_t* edev, int blocks, hipStream_t st) {
  const u32x4* src = (const u32x4*)g_rs_src;
  const Segs S = g_rs_segs;
#define MP4X_RS_CASE(N)                                                                                 \
  case N:                                                                                               \
    hipLaunchKernelGGL((k_ipc_reduce_range<DT, OP, N>), dim3(blocks), dim3(kIpcThreads), 0, st, P, self, \
                       rank, lo, hi, (u32x4*)out, epoch, edev, src, S);                                 \
    return (int)hipGetLastError();
  switch (p) {
    MP4X_RS_CASE(2) MP4X_RS_CASE(3) MP4X_RS_CASE(4) MP4X_RS_CASE(5) MP4X_RS_CASE(6) MP4X_RS_CASE(7) MP4X_RS_CASE(8)
    default: return MP4X_E_BADARG;
  }
#undef MP4X_RS_CASE
}

template <int DT>
static int rs_dt(int op, const IpcPtrs& P, Signal* self, int rank, int p, int64_t lo, int64_t hi, void* out,
                 uint32_t epoch, const uint32_t* edev, int blocks, hipStream_t st) {
  switch (op) {
    case MP4X_SUM: return rs_nr<DT, MP4X_SUM>(P, self, rank, p, lo, hi, out, epoch, edev, blocks, st);
    case MP4X_MAX:
      if constexpr (is_float_dt<DT>() && DT != MP4X_F64)
        return rs_nr<DT, MP4X_MAX>(P, self, rank, p, lo, hi, out, epoch, edev, blocks, st);
      return MP4X_E_UNSUPPORTED;
    case MP4X_MIN:
      if constexpr (is_float_dt<DT>() && DT != MP4X_F64)
        return rs_nr<DT, MP4X_MIN>(P, self, rank, p, lo, hi, out, epoch, edev, blocks, st);
      return MP4X_E_UNSUPPORTED;
    default: return MP4X_E_UNSUPPORTED;
  }
}

// Reduce-scatter over staged buffers: out (16-B aligned) receives vectors [vec_lo, vec_hi) of
// the op-reduction of all p buffers.  Every rank stages its WHOLE range before the call.
extern "C" int mp4x_ipc_reduce_scatter(int dtype, int op, void* const* data_ptrs, void* const* signal_ptrs, int rank,
                                       int p, int64_t vec_lo, int64_t vec_hi, void* out, uint32_t epoch, int blocks,
                                       const uint32_t* epoch_dev, void* stream) {
  IpcPtrs P;
  if (int e = ipc_prepare(data_ptrs, signal_ptrs, rank, p, &P)) return e;
  if (vec_lo < 0 || vec_hi < vec_lo || ((uintptr_t)out & 15)) return MP4X_E_BADARG;
  blocks = ipc_blocks(blocks, vec_hi - vec_lo);
  Signal* self = (Signal*)signal_ptrs[rank];
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case MP4X_F64: return rs_dt<MP4X_F64>(op, P, self, rank, p, vec_lo, vec_hi, out, epoch, epoch_dev, blocks, st);
    case MP4X_F32: return rs_dt<MP4X_F32>(op, P, self, rank, p, vec_lo, vec_hi, out, epoch, epoch_dev, blocks, st);
    case MP4X_I64: return rs_dt<MP4X_I64>(op, P, self, rank, p, vec_lo, vec_hi, out, epoch, epoch_dev, blocks, st);
    case MP4X_I32: return rs_dt<MP4X_I32>(op, P, self, rank, p, vec_lo, vec_hi, out, epoch, epoch_dev, blocks, st);
    case MP4X_BF16: return rs_dt<MP4X_BF16>(op, P, self, rank, p, vec_lo, vec_hi, out, epoch, epoch_dev, blocks, st);
    case MP4X_F16: return rs_dt<MP4X_F16>(op, P, self, rank, p, vec_lo, vec_hi, out, epoch, epoch_dev, blocks, st);
    default: return MP4X_E_UNSUPPORTED;
  }
}

// Reduce-scatter with fused staging: `src` (16-B aligned) holds this rank's whole range laid out
// like the buffer (vector offsets seg_lo/seg_hi per rank, relative to src and to the buffer);
// this rank's reduced segment goes straight to `out` (16-B aligned).  One launch, no copies.
extern "C" int mp4x_ipc_reduce_scatter_from(int dtype, int op, void* const* data_ptrs, void* const* signal_ptrs,
                                            int rank, int p, const int64_t* seg_lo, const int64_t* seg_hi,
                                            const void* src, void* out, uint32_t epoch, int blocks,
                                            const uint32_t* epoch_dev, void* stream) {
  if (!src || ((uintptr_t)src & 15) || p < 2 || p > kIpcMaxRanks || rank < 0 || rank >= p) return MP4X_E_BADARG;
  Segs S;
  for (int k = 0; k < kIpcMaxRanks; ++k) {
    S.lo[k] = k < p ? seg_lo[k] : 0;
    S.hi[k] = k < p ? seg_hi[k] : 0;
    if (k < p && (S.lo[k] < 0 || S.hi[k] < S.lo[k])) return MP4X_E_BADARG;
  }
  g_rs_src = src;
  g_rs_segs = S;
  // `out` receives vectors [lo, hi) at out[v - lo]
  int e = mp4x_ipc_reduce_scatter(dtype, op, data_ptrs, signal_ptrs, rank, p, S.lo[rank], S.hi[rank], out, epoch,
                                  blocks, epoch_dev, stream);
  g_rs_src = nullptr;
  return e;
}

// All-gather of ragged segments: seg_lo/seg_hi[p] (host arrays, 16-B vectors from the buffer
// base); every rank stages its own segment at its offset; out (the same layout, 16-B aligned)
// receives every peer's segment.
extern "C" int mp4x_ipc_allgather(void* const* data_ptrs, void* const* signal_ptrs, int rank, int p,
                                  const int64_t* seg_lo, const int64_t* seg_hi, void* out, uint32_t epoch, int blocks,
                                  const uint32_t* epoch_dev, void* stream) {
  IpcPtrs P;
  if (int e = ipc_prepare(data_ptrs, signal_ptrs, rank, p, &P)) return e;
  if ((uintptr_t)out & 15) return MP4X_E_BADARG;
  Segs S;
  int64_t maxlen = 0;
  for (int k = 0; k < kIpcMaxRanks; ++k) {
    S.lo[k] = k < p ? seg_lo[k] : 0;
    S.hi[k] = k < p ? seg_hi[k] : 0;
    if (k < p && (S.lo[k] < 0 || S.hi[k] < S.lo[k])) return MP4X_E_BADARG;
    if (S.hi[k] - S.lo[k] > maxlen) maxlen = S.hi[k] - S.lo[k];
  }
  blocks = ipc_blocks(blocks, maxlen);
  Signal* self = (Signal*)signal_ptrs[rank];
  hipStream_t st = (hipStream_t)stream;
#define MP4X_AG_CASE(N)                                                                                     \
  case N:                                                                                                   \
    hipLaunchKernelGGL((k_ipc_gather<N>), dim3(blocks), dim3(kIpcThreads), 0, st, P, self, rank, S, maxlen, \
                       (u32x4*)out, epoch, epoch_dev);                                                      \
    return (int)hipGetLastError();
  switch (p) {
    MP4X_AG_CASE(2) MP4X_AG_CASE(3) MP4X_AG_CASE(4) MP4X_AG_CASE(5) MP4X_AG_CASE(6) MP4X_AG_CASE(7) MP4X_AG_CASE(8)
    default: return MP4X_E_BADARG;
  }
#undef MP4X_AG_CASE
}

// Fused fp8 two-shot allreduce of one piece.  Every rank has already quantised its input into
// its own buffer (q bytes at 0, f32 scales at `soff`, p * cb quant blocks, blocks past the input
// zeroed); `out` (dtype = f32 / bf16 / f16, 16-B aligned) receives n elements.
extern "C" int mp4x_ipc_fp8_allreduce(int dtype, void* const* data_ptrs, void* const* signal_ptrs, int rank, int p,
                                      int64_t cb, int64_t soff, void* out, int64_t n, uint32_t epoch, int blocks,
                                      const uint32_t* epoch_dev, float scale, void* stream) {
  IpcPtrs P;
  if (int e = ipc_prepare(data_ptrs, signal_ptrs, rank, p, &P)) return e;
  if (cb <= 0 || n <= 0 || n > (int64_t)p * cb * kQBlock || (soff & 15) || ((uintptr_t)out & 15))
    return MP4X_E_BADARG;
  if (soff < (int64_t)p * cb * kQBlock) return MP4X_E_BADARG;     // scales after the q bytes
  static const bool narrow = getenv("MP4X_FP8_NARROW") && getenv("MP4X_FP8_NARROW")[0] == '1';
  if (blocks <= 0) {
    const int64_t waves = narrow ? cb : (cb + 3) / 4;               // one wave per 4 quant blocks
    int64_t b = (waves + kIpcThreads / 64 - 1) / (kIpcThreads / 64);
    blocks = (int)(b < 1 ? 1 : (b > kIpcMaxBlocks ? kIpcMaxBlocks : b));
  }
  if (blocks > kIpcMaxBlocks) blocks = kIpcMaxBlocks;
  Signal* self = (Signal*)signal_ptrs[rank];
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case MP4X_F32: return fp8_nr<MP4X_F32>(P, self, rank, p, cb, soff, out, n, epoch, epoch_dev, scale, blocks, st, narrow);
    case MP4X_BF16: return fp8_nr<MP4X_BF16>(P, self, rank, p, cb, soff, out, n, epoch, epoch_dev, scale, blocks, st, narrow);
    case MP4X_F16: return fp8_nr<MP4X_F16>(P, self, rank, p, cb, soff, out, n, epoch, epoch_dev, scale, blocks, st, narrow);
    default: return MP4X_E_UNSUPPORTED;
  }
}

extern "C" int mp4x_memset_async(void* dst, int value, size_t bytes, void* stream) {
  return (int)hipMemsetAsync(dst, value, bytes, (hipStream_t)stream);
}

// Copy plan (see k_ipc_copy_plan).  stage / pull: n x {src_off, dst_off, len, peer} int64
// quadruples in 16-byte vectors; `grid_len` (vectors) must be rank-independent — the largest
// item of any rank — so every rank launches the same grid.
extern "C" int mp4x_ipc_copy_plan(void* const* data_ptrs, void* const* signal_ptrs, int rank, int p,
                                  const int64_t* stage, int nstage, const int64_t* pull, int npull, const void* src,
                                  void* out, int64_t grid_len, int64_t buf_vecs, uint32_t epoch, int blocks,
                                  const uint32_t* epoch_dev, void* stream) {
  IpcPtrs P;
  if (int e = ipc_prepare(data_ptrs, signal_ptrs, rank, p, &P)) return e;
  if (nstage < 0 || nstage > kIpcMaxRanks || npull < 0 || npull > kIpcMaxRanks) return MP4X_E_BADARG;
  if ((nstage && (!src || ((uintptr_t)src & 15))) || (npull && (!out || ((uintptr_t)out & 15)))) return MP4X_E_BADARG;
  CopyPlan plan;
  plan.nstage = nstage;
  plan.npull = npull;
  for (int i = 0; i < kIpcMaxRanks; ++i) {
    plan.stage[i] = i < nstage ? CopyItem{stage[4 * i], stage[4 * i + 1], stage[4 * i + 2], 0} : CopyItem{0, 0, 0, 0};
    plan.pull[i] = i < npull ? CopyItem{pull[4 * i], pull[4 * i + 1], pull[4 * i + 2], pull[4 * i + 3]}
                             : CopyItem{0, 0, 0, 0};
    if (i < nstage && (plan.stage[i].len < 0 || plan.stage[i].dst_off < 0 ||
                       plan.stage[i].dst_off + plan.stage[i].len > buf_vecs))
      return MP4X_E_BADARG;                               // staging stays inside the own buffer
    if (i < npull && (plan.pull[i].len < 0 || plan.pull[i].peer < 0 || plan.pull[i].peer >= p ||
                      plan.pull[i].src_off < 0 || plan.pull[i].src_off + plan.pull[i].len > buf_vecs))
      return MP4X_E_BADARG;                               // pulls stay inside the peer's buffer
  }
  blocks = ipc_blocks(blocks, grid_len);
  hipLaunchKernelGGL(k_ipc_copy_plan, dim3(blocks), dim3(kIpcThreads), 0, (hipStream_t)stream, P,
                     (Signal*)signal_ptrs[rank], rank, p, plan, (const u32x4*)src, (u32x4*)out, epoch, epoch_dev);
  return (int)hipGetLastError();
}
