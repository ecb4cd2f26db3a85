// Shared device side of the custom xGMI collectives over IPC-mapped peer buffers (gfx950, one
// process per GPU).  The kernels live in per-family translation units so they compile in
// parallel: ipc_ar.hip (one-/two-shot allreduce), ipc_push.hip (zero-copy push two-shot),
// ipc_rs.hip (direct reduce-scatter), ipc.hip (all-gather, copy plans, fp8, host runtime).
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
// Reference analogue: the fused recv+reduce of the ring reduce-scatter, for EVERY operator of
// every primitive type (/root/reference/src/main/java/com/fenbi/mp4j/operator/Operators.java:29-353,
// hot loops DoubleOperand.java:196, ShortOperand.java:194, ByteOperand.java:193) and the
// small-message RPC allreduce (ProcessCommSlave.java:1776-1926) — here as one kernel.
//
// Operators: the gradient / statistic hot pairs (SUM of f64/f32/i64/i32/bf16/f16, MAX / MIN of
// f32/bf16/f16) have kernels of their own; every other valid (dtype, op) pair of the operator
// table — PROD, MAX / MIN of f64 and integers, BITS_AND / OR / XOR, the *_LOC packed words, int16
// and int8 — runs ONE runtime-op kernel per (dtype, rank count): the op is a kernel argument
// (wave-uniform, an SGPR), the NR remote loads are issued before one scalar branch per 16-byte
// vector selects the combine, so those pairs move exactly the bytes of the hot kernels.
//
// Synchronisation (cdna guide §6 G16, system scope because peers are other GPUs):
//  * every rank owns a Signal block in fine-grained, UNCACHED memory; flags are epochs
//    (monotonic per call, never reset) stored by the signalling lane with a relaxed
//    system-scope atomic store into the PEER's slot, after every wave of the block drained
//    its stores (s_waitcnt vmcnt(0)) + __syncthreads + a system-scope release fence;
//  * waiting lanes poll their own slots with relaxed system-scope loads + s_sleep, then a
//    system-scope acquire;  barriers are per BLOCK: block b of every rank touches exactly
//    the same element offsets, so block b only has to meet block b of the peers;
//  * every spin is bounded (s_memrealtime, 100 MHz) by the instance's Signal::spin_ticks, set
//    from the host: by default the fail-stop budget of the collective watchdog
//    (MP4X_WATCHDOG_TIMEOUT, 600 s — a straggling rank, e.g. one saving a checkpoint, is waited
//    for as the reference's blocking ring step waits, ProcessCommSlave.java:1355), a short
//    bound only while the mesh self-test and the autotune probes run.  On timeout the block
//    records an error word (device + pinned host copy) and exits instead of hanging the GPU;
//  * the STAGED forms' data buffers are uncached as well, so remote reads never see stale L2
//    lines;
//  * the ZERO-COPY forms read and write the peers' own tensors (coarse-grained hipMalloc or
//    memAlloc/VMM memory, L2-cached on their home GPU).  What they rely on: (a) every remote
//    WRITE of a call is followed by the writer's system-scope release (L2 write-back) before
//    its barrier flag, and (b) every block of the home GPU passes a system-scope ACQUIRE after
//    that barrier (block_barrier below: run by blocks on every XCD), so the lines of its own
//    tensor it cached before the peers' writes are invalidated before the kernel ends.  This is
//    the protocol argument, not an architectural guarantee for every topology: the collective
//    self-test (device_engine._ipc_self_test -> IpcAllreduce.selftest_zero_copy) runs the
//    zero-copy two-shot pull and push forms, the zero-copy copy plans and one memAlloc (VMM
//    imported) region TWICE on the same memory at mesh creation (the second call consumes the
//    first call's results, so a stale line would show as a wrong element) and drops the
//    zero-copy forms on every rank if any is wrong; autotune repeats that probe per candidate;
//    tests/test_multigpu_gpu.py runs them across real GPUs.  Until that module has run on a
//    multi-GPU node these forms are unverified across real xGMI (every builder run so far shared
//    one GPU).
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>

#include "../kernels/common.hpp"

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
// Op template value of the runtime-op kernels: the operator is the kernel argument `op`.
constexpr int kOpRt = -1;

struct alignas(128) Signal {
  uint32_t start[kIpcMaxBlocks][kIpcMaxRanks];
  uint32_t mid[kIpcMaxBlocks][kIpcMaxRanks];
  uint32_t end[kIpcMaxBlocks][kIpcMaxRanks];
  uint32_t error;
  // host-visible copy of `error`: device address of a pinned, mapped host word (0 = none), set
  // once at setup (mp4x_ipc_set_host_error); written on a barrier timeout so the host can fail
  // the call without any device synchronisation.  Only the owning rank reads this field.
  uint64_t host_err;
  // barrier spin bound of this instance's kernels, s_memrealtime ticks (100 MHz); 0 = the
  // built-in 600 s.  Set from the host (mp4x_ipc_set_spin); only the owning rank reads it.
  uint64_t spin_ticks;
  // DEBUG BUILD ONLY (MP4X_DEBUG; the release kernels never read it): kDbgNoRelease /
  // kDbgNoAcquire remove block_barrier's system-scope release / acquire, so a test can show that
  // the coherence probes detect a missing fence (tests/test_coherence_gpu.py).  mp4x_ipc_set_debug.
  uint32_t dbg_flags;
};

constexpr uint32_t kDbgNoRelease = 1u;
constexpr uint32_t kDbgNoAcquire = 2u;

// The two halves of every cross-agent hand-off of these kernels (MI355X_MICROARCH "inter-workgroup
// visibility": per-XCD L2s are not coherent with each other, a CU's L1 is never refreshed by
// another CU's stores).  Release: write back the dirty lines of this XCD's L2, and WAIT for the
// write-back before the flag store (an inline-asm wait: the compiler may drop its own after
// buffer_wbl2).  Acquire: invalidate this CU's L1 / the non-coherent L2 lines, and WAIT for the
// invalidate, which completes asynchronously — the block's other waves load right after the
// __syncthreads that follows, so without this wait they could still hit stale lines.
__device__ __forceinline__ void sys_release() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");        // system scope
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void sys_acquire() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");        // system scope
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The debug flags of `self` (0 in release builds: the fences are unconditional there).
__device__ __forceinline__ uint32_t dbg_flags_of(const Signal* self) {
#ifdef MP4X_DEBUG
  return __hip_atomic_load(&self->dbg_flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else
  (void)self;
  return 0u;
#endif
}

constexpr uint64_t kDefaultSpinTicks = 600ull * 100000000ull;   // 600 s at 100 MHz

// The per-communicator stream-order guard (csrc/runtime/order.hip, mp4x/parallel/order.py): the
// device-side total order of ONE communicator's collectives across the caller's streams.  Field
// order is the ctypes layout of mp4x.parallel.order.StreamOrder.
struct StreamOrder {
  void* last;            // hipStream_t of the communicator's previous launch (when have_last)
  void* ev;              // hipEvent_t, created at the first stream switch
  void* cap_stream;      // the stream of the current graph capture's launches (when cap_have)
  uint64_t cap_id;       // that capture's id
  uint64_t switches;     // stream switches joined so far (statistics, tests)
  int32_t have_last;
  int32_t cap_have;
  int32_t disabled;      // MP4X_TEST_NO_STREAM_ORDER=1: tests only (shows the guard has teeth)
  int32_t pad;
};
// 0, or MP4X_E_STREAM_SWITCH / a HIP error: see order.hip (mp4x_order_enter: the caller knows the
// stream is not being captured).
extern "C" int mp4x_order_enter(StreamOrder* o, void* stream);

struct IpcPtrs {
  const void* data[kIpcMaxRanks];   // every rank's data buffer (own one included)
  Signal* sig[kIpcMaxRanks];        // every rank's signal block
};

// Every rank's segment of a ragged collective, in 16-byte vectors.
struct Segs {
  int64_t lo[kIpcMaxRanks];
  int64_t hi[kIpcMaxRanks];
};

// Lane t's peer Signal block: a select chain over the kernel argument's pointers (held in SGPRs)
// instead of P.sig[t], whose per-lane index made every barrier a vector load from the kernarg
// segment before the flag store.
__device__ __forceinline__ uint64_t sgpr64(const void* v) {   // a wave-uniform pointer, in SGPRs
  const uint64_t x = reinterpret_cast<uint64_t>(v);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x >> 32));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

__device__ __forceinline__ Signal* sig_of(const IpcPtrs& P, int t) {
  uint64_t s = sgpr64(P.sig[0]);
#pragma unroll
  for (int k = 1; k < kIpcMaxRanks; ++k) {
    const uint64_t v = sgpr64(P.sig[k]);
    s = t == k ? v : s;
  }
  return reinterpret_cast<Signal*>(s);
}

// The epoch after `e` (low 30 bits; 0 is never used and the sequence wraps to 2, so consecutive
// epochs always alternate parity — the one-shot's double-buffered slots are chosen by it).  Host
// (IpcAllreduce._next_epoch, mp4x_ipc_fast_allreduce) and k_ipc_bump_epoch follow the same rule.
__host__ __device__ __forceinline__ uint32_t next_epoch(uint32_t e) {
  const uint32_t n = ((e & ~kTagMask) + 1u) & ~kTagMask;
  return n ? n : 2u;
}

// `which`: 0 start, 1 mid, 2 end.  `accept_ahead` (start barrier of the SLOTTED one- and two-shot
// only, k_ipc_oneshot / k_ipc_twoshot with slots): a peer may already be ONE call ahead — those
// kernels have no end barrier, so a peer that finished call e can store call e+1's start flag
// before this rank saw its flag of call e.  It can get no further (call e+1's start barrier needs
// this rank's arrival), and never ahead at a mid barrier.  A start flag holding the next epoch
// therefore means "arrived, and done with call e" — with ANY protocol tag: call e+1 may
// legitimately be a zero-copy call (a registered tensor) after a staged slotted call e.  Only a
// kernel without an end barrier can face a peer that is ahead, so every other kernel accepts its
// own epoch only.  Mismatch detection is one-sided in the slotted kernels: if a peer
// runs another protocol for call e itself (registrations differ across ranks), one side sees the
// other tag and fails at once (code 4), the other may take that peer's flag for "ahead".
__device__ __forceinline__ bool block_barrier(const IpcPtrs& P, int which, int rank, int p, uint32_t epoch,
                                              Signal* self, bool accept_ahead = false) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave drains its stores
  __syncthreads();
  __shared__ int s_fail;
  if (threadIdx.x == 0) s_fail = 0;
  __syncthreads();
  const int t = threadIdx.x;
  if (t < p) {
    const uint32_t dbg = dbg_flags_of(self);
    if (!(dbg & kDbgNoRelease)) sys_release();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    Signal* peer = sig_of(P, t);
    uint32_t* slot = which == 0 ? &peer->start[blockIdx.x][rank]
                   : which == 1 ? &peer->mid[blockIdx.x][rank] : &peer->end[blockIdx.x][rank];
    __hip_atomic_store(slot, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = which == 0 ? &self->start[blockIdx.x][t]
                   : which == 1 ? &self->mid[blockIdx.x][t] : &self->end[blockIdx.x][t];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    // the bound is read only by a lane that has to wait: the fast path (peers already there)
    // pays one uncached round trip, not two (r4 latency: +4 us per kernel when it was read first)
    uint64_t spin = 0;
    uint32_t seen;
    // (an epoch's low bits are never all ones: 0xFFFFFFFF never matches)
    const uint32_t ahead = accept_ahead ? next_epoch(epoch) : 0xFFFFFFFFu;
    while ((seen = __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) != epoch &&
           (seen & ~kTagMask) != ahead) {
      if (spin == 0) {
        spin = __hip_atomic_load(&self->spin_ticks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (spin == 0) spin = kDefaultSpinTicks;
      }
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
    if (!(dbg & kDbgNoAcquire)) sys_acquire();
  }
  __syncthreads();
  return s_fail == 0;
}

// Combine of NR 16-byte vectors (rank order: r[0] first, deterministic), then the optional
// fused scale (float dtypes, a wave-uniform branch; 1.0 = plain reduction).
template <int DT, int OP, int NR>
__device__ __forceinline__ u32x4 fold_vec(const u32x4 (&r)[NR], float scale) {
  using E = Elem<DT>;
  using S = typename E::S;
  using A = typename E::A;
  constexpr int W = 16 / sizeof(S);
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

// OP = kOpRt: the combine chosen by the kernel argument `op` (validated on the host against
// op_valid; one scalar branch per vector after the loads are in flight).
template <int DT, int OP, int NR>
__device__ __forceinline__ u32x4 fold_any(const u32x4 (&r)[NR], float scale, int op) {
  if constexpr (OP != kOpRt) {
    (void)op;
    return fold_vec<DT, OP, NR>(r, scale);
  } else {
    switch (op) {
#define MP4X_FOLD_CASE(X)                                   \
  case X:                                                   \
    if constexpr (op_valid<DT, X>()) return fold_vec<DT, X, NR>(r, scale); \
    break;
      MP4X_FOLD_CASE(MP4X_SUM) MP4X_FOLD_CASE(MP4X_MAX) MP4X_FOLD_CASE(MP4X_MIN) MP4X_FOLD_CASE(MP4X_PROD)
      MP4X_FOLD_CASE(MP4X_BAND) MP4X_FOLD_CASE(MP4X_BOR) MP4X_FOLD_CASE(MP4X_BXOR)
      MP4X_FOLD_CASE(MP4X_FMAXLOC) MP4X_FOLD_CASE(MP4X_FMINLOC) MP4X_FOLD_CASE(MP4X_IMAXLOC)
      MP4X_FOLD_CASE(MP4X_IMINLOC)
#undef MP4X_FOLD_CASE
      default: break;
    }
    return r[0];
  }
}

// NR (rank count) is a template parameter: the NR remote loads are issued unconditionally
// and back to back (no per-load branch, cdna guide §5 trap (c)).
template <int DT, int OP, int NR>
__device__ __forceinline__ u32x4 reduce_vec(const IpcPtrs& P, int64_t v, float scale, int op) {
  u32x4 r[NR];
#pragma unroll
  for (int k = 0; k < NR; ++k) r[k] = reinterpret_cast<const u32x4*>(P.data[k])[v];   // NR loads in flight
  return fold_any<DT, OP, NR>(r, scale, op);
}

__device__ __forceinline__ uint32_t resolve_epoch(uint32_t epoch, const uint32_t* epoch_dev) {
  // graph mode: the epoch lives in device memory and is bumped by k_ipc_bump_epoch, the
  // preceding node of the same graph, so every replay gets a fresh, rank-consistent epoch
  // (the protocol tag of a host-passed epoch is kept in graph mode too)
  return epoch_dev ? (__hip_atomic_load(epoch_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) | (epoch & kTagMask))
                   : epoch;
}

// ---------------------------------------------------------------- host-side dispatch
template <int V> using IntC = std::integral_constant<int, V>;

// (dtype, op) pairs with kernels of their own (compile-time op): the DP gradient / statistic path.
template <int DT> constexpr bool hot_sum() {
  return DT == MP4X_F64 || DT == MP4X_F32 || DT == MP4X_I64 || DT == MP4X_I32 || DT == MP4X_BF16 || DT == MP4X_F16;
}
template <int DT> constexpr bool hot_minmax() { return DT == MP4X_F32 || DT == MP4X_BF16 || DT == MP4X_F16; }

// Every reduction of the reference's operator table for DT (MP4X_FIRST is a sparse-merge rule,
// not a collective operator).
template <int DT> inline bool rt_op_ok(int op) {
  switch (op) {
    case MP4X_SUM: return op_valid<DT, MP4X_SUM>();
    case MP4X_MAX: return op_valid<DT, MP4X_MAX>();
    case MP4X_MIN: return op_valid<DT, MP4X_MIN>();
    case MP4X_PROD: return op_valid<DT, MP4X_PROD>();
    case MP4X_BAND: return op_valid<DT, MP4X_BAND>();
    case MP4X_BOR: return op_valid<DT, MP4X_BOR>();
    case MP4X_BXOR: return op_valid<DT, MP4X_BXOR>();
    case MP4X_FMAXLOC: return op_valid<DT, MP4X_FMAXLOC>();
    case MP4X_FMINLOC: return op_valid<DT, MP4X_FMINLOC>();
    case MP4X_IMAXLOC: return op_valid<DT, MP4X_IMAXLOC>();
    case MP4X_IMINLOC: return op_valid<DT, MP4X_IMINLOC>();
    default: return false;
  }
}

// f(IntC<DT>{}) for a runtime dtype code.
template <typename F> inline int with_dtype(int dtype, F&& f) {
  switch (dtype) {
    case MP4X_F64: return f(IntC<MP4X_F64>{});
    case MP4X_F32: return f(IntC<MP4X_F32>{});
    case MP4X_I64: return f(IntC<MP4X_I64>{});
    case MP4X_I32: return f(IntC<MP4X_I32>{});
    case MP4X_I16: return f(IntC<MP4X_I16>{});
    case MP4X_I8: return f(IntC<MP4X_I8>{});
    case MP4X_BF16: return f(IntC<MP4X_BF16>{});
    case MP4X_F16: return f(IntC<MP4X_F16>{});
    case MP4X_U8: return f(IntC<MP4X_U8>{});
    default: return MP4X_E_UNSUPPORTED;
  }
}

// f(IntC<OP>{}) with the kernel op of (DT, op): a hot pair's own op, else kOpRt.
template <int DT, typename F> inline int with_op(int op, F&& f) {
  if constexpr (hot_sum<DT>()) {
    if (op == MP4X_SUM) return f(IntC<MP4X_SUM>{});
  }
  if constexpr (hot_minmax<DT>()) {
    if (op == MP4X_MAX) return f(IntC<MP4X_MAX>{});
    if (op == MP4X_MIN) return f(IntC<MP4X_MIN>{});
  }
  if (!rt_op_ok<DT>(op)) return MP4X_E_UNSUPPORTED;
  return f(IntC<kOpRt>{});
}

// 0 when the IPC kernels reduce `op` over `dtype` (a hot pair or the runtime-op kernel), else
// MP4X_E_UNSUPPORTED — the refusal with_dtype / with_op would make at launch time.
inline int op_supported(int dtype, int op) {
  return with_dtype(dtype, [&](auto dtc) {
    constexpr int DT = decltype(dtc)::value;
    return with_op<DT>(op, [](auto) { return 0; });
  });
}

// f(IntC<NR>{}) for a rank count 2..8.
template <typename F> inline int with_nr(int p, F&& f) {
  switch (p) {
    case 2: return f(IntC<2>{});
    case 3: return f(IntC<3>{});
    case 4: return f(IntC<4>{});
    case 5: return f(IntC<5>{});
    case 6: return f(IntC<6>{});
    case 7: return f(IntC<7>{});
    case 8: return f(IntC<8>{});
    default: return MP4X_E_BADARG;
  }
}

// Blocks per CU the occupancy API admits for `kern` at kIpcThreads threads (min-folded into *m).
template <typename K> inline void occ_min(K kern, int* m) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, kIpcThreads, 0) != hipSuccess) {
    n = 0;
    (void)hipGetLastError();      // a failed query must not surface as PyTorch's next error
  }
  if (n < *m) *m = n;
}

inline int ipc_prepare(void* const* data_ptrs, void* const* signal_ptrs, int rank, int p, IpcPtrs* P) {
  if (p < 2 || p > kIpcMaxRanks || rank < 0 || rank >= p) return MP4X_E_BADARG;
  for (int k = 0; k < kIpcMaxRanks; ++k) {
    P->data[k] = k < p ? data_ptrs[k] : nullptr;
    P->sig[k] = k < p ? (Signal*)signal_ptrs[k] : nullptr;
    if (k < p && (((uintptr_t)P->data[k] & 15) || !P->sig[k])) return MP4X_E_BADARG;
  }
  return 0;
}

inline int ipc_blocks(int blocks, int64_t nvec) {
  if (blocks <= 0) {
    int64_t b = (nvec + kIpcThreads - 1) / kIpcThreads;
    blocks = (int)(b < 1 ? 1 : (b > kIpcMaxBlocks ? kIpcMaxBlocks : b));
  }
  return blocks > kIpcMaxBlocks ? kIpcMaxBlocks : blocks;
}

inline bool float_dtype(int dtype) {
  return dtype == MP4X_F32 || dtype == MP4X_F64 || dtype == MP4X_BF16 || dtype == MP4X_F16;
}

}  // namespace mp4x
