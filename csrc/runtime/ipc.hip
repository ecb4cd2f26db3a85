// All-gather, copy plans (broadcast / scatter / gather / ragged all-to-all) and the fused fp8
// two-shot over IPC-mapped peer buffers, plus the host runtime of the IPC mesh (allocation,
// handles, error words, spin bound).  Protocol: ipc_common.hpp.  The reducing families live in
// ipc_ar.hip (one-/two-shot), ipc_push.hip (zero-copy push) and ipc_rs.hip (reduce-scatter).
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdlib>

#include "ipc_common.hpp"
#include "../kernels/fp8.hpp"

namespace mp4x {

__global__ void k_ipc_bump_epoch(uint32_t* epoch_dev) {
  *epoch_dev = next_epoch(*epoch_dev);      // (wraps to 2: consecutive epochs alternate parity)
}

// ---------------------------------------------------------------- direct all-gather
// The second half of the two-shot as a collective of its own over RAGGED per-rank ranges
// (allgatherArray froms-tos): rank r pulls every peer's segment, the same offset from all p-1
// peers per step, so all links stream at once.
template <int NR>
__global__ __launch_bounds__(kIpcThreads) void k_ipc_gather(IpcPtrs P, Signal* self, int rank, Segs S,
                                                             int64_t maxlen, u32x4* __restrict__ out, uint32_t epoch,
                                                             const uint32_t* epoch_dev) {
  constexpr int p = NR;
  MP4X_DASSERT(rank >= 0 && rank < NR);
  epoch = resolve_epoch(epoch, epoch_dev);
  if (!block_barrier(P, 0, rank, p, epoch, self)) return;
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
  block_barrier(P, 2, rank, p, epoch, self);
}

// ---------------------------------------------------------------- copy plans (bcast / scatter / gather)
// The data-movement collectives as ONE kernel per call: a plan of up to kIpcMaxRanks "stage"
// items (this rank's input -> its own buffer, fused copy-in) and up to kPlanMaxPulls "pull" items
// (a peer's buffer -> this rank's output, over xGMI, all pulls interleaved so every link
// streams; two per peer: the sparse exchanges pull a row block and a key block from each).  Every item is walked with the same grid-stride relative index on every rank, so
// the vectors block b stages are exactly the vectors block b of the peers pull: per-block
// barriers suffice, as in the two-shot.  Units: 16-byte vectors.
struct CopyItem {
  int64_t src_off, dst_off, len;
  int64_t peer;          // pull: source rank; stage: unused
};
constexpr int kPlanMaxPulls = 2 * kIpcMaxRanks;
struct CopyPlan {
  CopyItem stage[kIpcMaxRanks];
  CopyItem pull[kPlanMaxPulls];
  int nstage, npull;
};

// NP: the pulls the kernel keeps in flight per vector step (kIpcMaxRanks, or kPlanMaxPulls for
// plans with more pulls than that: the wider form takes ~30 more VGPRs, so it only runs when needed).
template <int NP>
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
  if (!block_barrier(P, 0, rank, p, epoch, self)) return;
  int64_t maxlen = 0;
  for (int i = 0; i < plan.npull; ++i) maxlen = plan.pull[i].len > maxlen ? plan.pull[i].len : maxlen;
  for (int64_t v = off0; v < maxlen; v += stride) {
    u32x4 x[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i)                     // every pull's vector in flight at once
      if (i < plan.npull && v < plan.pull[i].len)
        x[i] = reinterpret_cast<const u32x4*>(P.data[plan.pull[i].peer])[plan.pull[i].src_off + v];
#pragma unroll
    for (int i = 0; i < NP; ++i)
      if (i < plan.npull && v < plan.pull[i].len) out[plan.pull[i].dst_off + v] = x[i];
  }
  block_barrier(P, 2, rank, p, epoch, self);
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
  if (!block_barrier(P, 0, rank, p, epoch, self)) return;
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
  if (!block_barrier(P, 1, rank, p, epoch, self)) return;
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
  block_barrier(P, 2, rank, p, epoch, self);
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
  if (!block_barrier(P, 0, rank, p, epoch, self)) return;
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
  if (!block_barrier(P, 1, rank, p, epoch, self)) return;
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
  block_barrier(P, 2, rank, p, epoch, self);
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

// Barrier spin bound of the kernels that use `signal` (this rank's own Signal block), in seconds.
// Stream-ordered on `stream` (kernels queued before it keep the previous bound).
extern "C" int mp4x_ipc_set_spin(void* signal, double seconds, void* stream) {
  if (!(seconds > 0.0) || !signal) return MP4X_E_BADARG;
  const uint64_t ticks = (uint64_t)(seconds * 1.0e8);   // the stream is synchronised below
  char* w = (char*)signal + offsetof(Signal, spin_ticks);
  hipError_t e = hipMemcpyAsync(w, &ticks, sizeof(ticks), hipMemcpyHostToDevice, (hipStream_t)stream);
  if (e != hipSuccess) return (int)e;
  return (int)hipStreamSynchronize((hipStream_t)stream);
}

// Bump the device epoch counter of a graph-capturable instance (stream-ordered: the next IPC
// kernel on `stream` reads the new epoch; see resolve_epoch).
extern "C" int mp4x_ipc_bump_epoch(uint32_t* epoch_dev, void* stream) {
  hipLaunchKernelGGL(k_ipc_bump_epoch, dim3(1), dim3(1), 0, (hipStream_t)stream, epoch_dev);
  return (int)hipGetLastError();
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
// Every refusal of mp4x_ipc_copy_plan (the latency fast path runs it before its epoch moves).
extern "C" int mp4x_ipc_copy_plan_check(int rank, int p, const int64_t* stage, int nstage, const int64_t* pull,
                                        int npull, const void* src, const void* out, int64_t buf_vecs) {
  if (p < 2 || p > kIpcMaxRanks || rank < 0 || rank >= p) return MP4X_E_BADARG;
  if (nstage < 0 || nstage > kIpcMaxRanks || npull < 0 || npull > kPlanMaxPulls) return MP4X_E_BADARG;
  if ((nstage && (!src || ((uintptr_t)src & 15))) || (npull && (!out || ((uintptr_t)out & 15)))) return MP4X_E_BADARG;
  for (int i = 0; i < nstage; ++i) {
    const int64_t* it = stage + 4 * i;                    // {src_off, dst_off, len, -}
    if (it[2] < 0 || it[1] < 0 || it[1] + it[2] > buf_vecs) return MP4X_E_BADARG;   // inside the own buffer
  }
  for (int i = 0; i < npull; ++i) {
    const int64_t* it = pull + 4 * i;                     // {src_off, dst_off, len, peer}
    if (it[2] < 0 || it[3] < 0 || it[3] >= p || it[0] < 0 || it[0] + it[2] > buf_vecs)
      return MP4X_E_BADARG;                               // pulls stay inside the peer's buffer
  }
  return 0;
}

extern "C" int mp4x_ipc_copy_plan(void* const* data_ptrs, void* const* signal_ptrs, int rank, int p,
                                  const int64_t* stage, int nstage, const int64_t* pull, int npull, const void* src,
                                  void* out, int64_t grid_len, int64_t buf_vecs, uint32_t epoch, int blocks,
                                  const uint32_t* epoch_dev, void* stream) {
  if (int e = mp4x_ipc_copy_plan_check(rank, p, stage, nstage, pull, npull, src, out, buf_vecs)) return e;
  IpcPtrs P;
  if (int e = ipc_prepare(data_ptrs, signal_ptrs, rank, p, &P)) return e;
  CopyPlan plan;
  plan.nstage = nstage;
  plan.npull = npull;
  for (int i = 0; i < kIpcMaxRanks; ++i)
    plan.stage[i] = i < nstage ? CopyItem{stage[4 * i], stage[4 * i + 1], stage[4 * i + 2], 0} : CopyItem{0, 0, 0, 0};
  for (int i = 0; i < kPlanMaxPulls; ++i)
    plan.pull[i] = i < npull ? CopyItem{pull[4 * i], pull[4 * i + 1], pull[4 * i + 2], pull[4 * i + 3]}
                             : CopyItem{0, 0, 0, 0};
  blocks = ipc_blocks(blocks, grid_len);
  if (npull <= kIpcMaxRanks)
    hipLaunchKernelGGL(k_ipc_copy_plan<kIpcMaxRanks>, dim3(blocks), dim3(kIpcThreads), 0, (hipStream_t)stream, P,
                       (Signal*)signal_ptrs[rank], rank, p, plan, (const u32x4*)src, (u32x4*)out, epoch, epoch_dev);
  else
    hipLaunchKernelGGL(k_ipc_copy_plan<kPlanMaxPulls>, dim3(blocks), dim3(kIpcThreads), 0, (hipStream_t)stream, P,
                       (Signal*)signal_ptrs[rank], rank, p, plan, (const u32x4*)src, (u32x4*)out, epoch, epoch_dev);
  return (int)hipGetLastError();
}


// Blocks per CU the occupancy API admits for the data-movement kernels (family 0 = the ragged
// all-gather k_ipc_gather<p>, 1 = the copy plan) and the fused fp8 two-shot (2 = wide, 3 = narrow;
// dtype = the output dtype): the shared-GPU co-residency budget (mp4x/parallel/occupancy.py).
extern "C" int mp4x_ipc_occupancy_misc(int family, int dtype, int p, int* blocks_per_cu) {
  int m = 1 << 30;
  int e = 0;
  if (family == 1) {
    occ_min(k_ipc_copy_plan<kIpcMaxRanks>, &m);       // the shared-GPU cap must hold for both forms
    occ_min(k_ipc_copy_plan<kPlanMaxPulls>, &m);
  } else {
    e = with_nr(p, [&](auto nrc) {
      constexpr int NR = decltype(nrc)::value;
      if (family == 0) {
        occ_min(k_ipc_gather<NR>, &m);
        return 0;
      }
      const bool narrow = family == 3;
      switch (dtype) {
        case MP4X_F32: narrow ? occ_min(k_ipc_fp8_twoshot_narrow<MP4X_F32, NR>, &m)
                              : occ_min(k_ipc_fp8_twoshot<MP4X_F32, NR>, &m); return 0;
        case MP4X_BF16: narrow ? occ_min(k_ipc_fp8_twoshot_narrow<MP4X_BF16, NR>, &m)
                               : occ_min(k_ipc_fp8_twoshot<MP4X_BF16, NR>, &m); return 0;
        case MP4X_F16: narrow ? occ_min(k_ipc_fp8_twoshot_narrow<MP4X_F16, NR>, &m)
                              : occ_min(k_ipc_fp8_twoshot<MP4X_F16, NR>, &m); return 0;
        default: return (int)MP4X_E_UNSUPPORTED;
      }
    });
  }
  *blocks_per_cu = m == (1 << 30) ? 0 : m;
  return e;
}
