// Cross-XCD hand-off probe: do the IPC kernels' system-scope release / acquire (ipc_common.hpp
// sys_release / sys_acquire, the fences of every block_barrier) make a producer's plain stores
// visible to a consumer on ANOTHER XCD of the same GPU — and does the probe see it when they are
// left out?  ("the coherence probes have no teeth on the hardware the builder
// can reach".  On one MI355X the 8 XCDs have L2s that are not coherent with each other, so the
// failure the zero-copy protocol guards against across GPUs has a same-GPU analogue.)
//
// 16 workgroups, co-resident (16 of 256 CUs).  Block b < 8 produces region b; block 8 + k consumes
// region (k + 1) % 8 — blocks are dealt round-robin over the XCDs, so producer and consumer sit on
// different XCDs (each block reports its XCC id; the test checks).  Round i, the "two-call"
// stale-line probe of tests/test_multigpu_gpu.py:
//   consumer: reads the region (round i-1's data -> its L1 / L2 now hold those lines), tells the
//             producer it may write (ready = i);
//   producer: waits for ready = i, overwrites the region with round i's pattern (plain stores),
//             release (unless masked off), flag done = i;
//   consumer: polls done = i, acquire (unless masked off), reads the region again and counts the
//             vectors that still hold anything but round i's pattern.
// Every spin is bounded (s_memrealtime, 100 MHz): a timeout stops every block (out[32]).
// Region size 4 KiB: re-reads of that size are near-certain to be served from the stale lines
// (MI355X_MICROARCH "inter-workgroup visibility").
#include <hip/hip_runtime.h>

#include "ipc_common.hpp"

namespace mp4x {
namespace {

constexpr int kProbeBlocks = 16;
constexpr int kProbeThreads = 256;

__device__ __forceinline__ u32x4 probe_pattern(int round, int64_t v, int region) {
  u32x4 x;
  x[0] = (uint32_t)round;
  x[1] = (uint32_t)v;
  x[2] = (uint32_t)region;
  x[3] = (uint32_t)round * 2654435761u ^ (uint32_t)v;
  return x;
}

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  return x;
}

// Lane 0 waits for *flag == want (relaxed system-scope polls); false after `spin` ticks or when
// another block already gave up.
__device__ __forceinline__ bool wait_flag(uint32_t* flag, uint32_t want, uint64_t spin, uint32_t* abort_word) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != want) {
    __builtin_amdgcn_s_sleep(2);
    if (__builtin_amdgcn_s_memrealtime() - t0 > spin ||
        __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
      __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
  }
  return true;
}

// out[0..15]: stale vectors seen by block b (consumers only); out[16..31]: XCC id of block b;
// out[32]: 1 if any spin timed out.  flags: 8 regions x 64 words (ready at +0, done at +32: their
// own 128-byte lines), zero on entry.
__global__ __launch_bounds__(kProbeThreads) void k_xcd_probe(u32x4* data, uint32_t* flags, int64_t region_vecs,
                                                             int rounds, uint32_t mask, uint64_t spin, uint32_t* out) {
  const int b = blockIdx.x;
  const bool producer = b < 8;
  const int region = producer ? b : ((b - 8 + 1) & 7);
  u32x4* d = data + region * region_vecs;
  uint32_t* ready = flags + region * 64;
  uint32_t* done = flags + region * 64 + 32;
  uint32_t* abort_word = out + 32;
  __shared__ int s_ok;
  if (threadIdx.x == 0) out[16 + b] = xcc_id();
  uint32_t stale = 0, sink = 0;
  for (int i = 1; i <= rounds; ++i) {
    if (producer) {
      if (threadIdx.x == 0) s_ok = wait_flag(ready, (uint32_t)i, spin, abort_word);
      __syncthreads();
      if (!s_ok) break;
      for (int64_t v = threadIdx.x; v < region_vecs; v += blockDim.x) d[v] = probe_pattern(i, v, region);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        if (!(mask & kDbgNoRelease)) sys_release();
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(done, (uint32_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    } else {
      for (int64_t v = threadIdx.x; v < region_vecs; v += blockDim.x) sink ^= d[v][3];   // cache round i-1
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        __hip_atomic_store(ready, (uint32_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s_ok = wait_flag(done, (uint32_t)i, spin, abort_word);
        if (!(mask & kDbgNoAcquire)) sys_acquire();
      }
      __syncthreads();
      if (!s_ok) break;
      for (int64_t v = threadIdx.x; v < region_vecs; v += blockDim.x) {
        const u32x4 x = d[v];
        const u32x4 e = probe_pattern(i, v, region);
        stale += (x[0] != e[0] || x[1] != e[1] || x[2] != e[2] || x[3] != e[3]) ? 1u : 0u;
      }
      __syncthreads();
    }
  }
  if (stale) atomicAdd(out + b, stale);
  if (sink == 0xFFFFFFFFu && stale == 0xFFFFFFFFu) out[33] = sink;   // keeps the pre-reads alive
}

}  // namespace
}  // namespace mp4x

// Run the probe on caller-provided device buffers: `data` (8 * region_vecs 16-byte vectors, any
// contents), `flags` (512 u32, zeroed by this call), `out` (34 u32, zeroed by this call).  `mask`:
// kDbgNoRelease | kDbgNoAcquire leave the producer's release / the consumer's acquire out.
extern "C" int mp4x_xcd_probe(void* data, void* flags, void* out, int64_t region_vecs, int rounds, uint32_t mask,
                              double spin_s, void* stream) {
  using namespace mp4x;
  if (!data || !flags || !out || region_vecs <= 0 || rounds <= 0 || !(spin_s > 0.0)) return MP4X_E_BADARG;
  if (((uintptr_t)data & 15) || ((uintptr_t)flags & 127)) return MP4X_E_BADARG;
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(flags, 0, 512 * sizeof(uint32_t), st);
  if (e != hipSuccess) return (int)e;
  e = hipMemsetAsync(out, 0, 34 * sizeof(uint32_t), st);
  if (e != hipSuccess) return (int)e;
  const uint64_t spin = (uint64_t)(spin_s * 1.0e8);
  hipLaunchKernelGGL(k_xcd_probe, dim3(kProbeBlocks), dim3(kProbeThreads), 0, st, (u32x4*)data, (uint32_t*)flags,
                     region_vecs, rounds, mask, spin, (uint32_t*)out);
  return (int)hipGetLastError();
}

// The debug flags of an IPC instance's own Signal block (kDbgNoRelease / kDbgNoAcquire): read by
// block_barrier in the debug build (libmp4x_hip_debug.so) only; the release kernels ignore them.
extern "C" int mp4x_ipc_set_debug(void* signal, uint32_t flags) {
  using namespace mp4x;
  if (!signal) return MP4X_E_BADARG;
  return (int)hipMemcpy((char*)signal + offsetof(Signal, dbg_flags), &flags, sizeof(flags), hipMemcpyHostToDevice);
}

extern "C" int mp4x_debug_build(void) {
#ifdef MP4X_DEBUG
  return 1;
#else
  return 0;
#endif
}
