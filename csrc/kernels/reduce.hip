// K1 / K1b / K2 — fused multi-input elementwise reduction (gfx950).
//
// Replaces the reference's per-element reduce-on-receive loop
// (/root/reference/src/main/java/com/fenbi/mp4j/operand/DoubleOperand.java:196, and the
// thread-level `threadReduce` loop :453) with ONE streaming pass over up to 8 inputs:
//
//   out[i] = op(...op(op(in0[i], in1[i]), in2[i])..., in_{nin-1}[i])
//
// Design for CDNA4:
//  * HBM-bound: every lane moves 16 B per input per iteration (global_load_dwordx4),
//    all NIN loads of an iteration are issued before the first use so each lane keeps
//    NIN x 2 loads in flight (2-way unrolled grid-stride loop);
//  * 256-thread workgroups (4 x wave64), grid capped at 256 CUs x 8 blocks and
//    grid-strided, so a 1 GB operand needs no giant launch;
//  * 16-bit floats accumulate in f32 across the whole fan-in and round once;
//  * operands with mismatched 16-byte alignment fall back to the scalar kernel.
#include "common.hpp"
#include <stdlib.h>

namespace mp4x {

template <int NIN> struct InPtrs { const void* p[NIN]; };

template <int DT, int OP, int NIN>
__global__ __launch_bounds__(kBlock) void k_reduce_vec(void* __restrict__ out_, InPtrs<NIN> ins,
                                                       int64_t nvec, int64_t n) {
  using E = Elem<DT>;
  using S = typename E::S;
  using A = typename E::A;
  constexpr int W = 16 / sizeof(S);
  const int64_t nthr = (int64_t)gridDim.x * kBlock;
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  u32x4* out = reinterpret_cast<u32x4*>(out_);

  for (int64_t v = tid; v < nvec; v += 2 * nthr) {
    const int64_t v1 = v + nthr;
    const bool two = v1 < nvec;
    u32x4 r0[NIN], r1[NIN];
#pragma unroll
    for (int k = 0; k < NIN; ++k) {
      r0[k] = reinterpret_cast<const u32x4*>(ins.p[k])[v];
      if (two) r1[k] = reinterpret_cast<const u32x4*>(ins.p[k])[v1];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      u32x4* r = u ? r1 : r0;
      S acc_s[W];
      __builtin_memcpy(acc_s, &r[0], 16);
      A acc[W];
#pragma unroll
      for (int j = 0; j < W; ++j) acc[j] = E::load(acc_s[j]);
#pragma unroll
      for (int k = 1; k < NIN; ++k) {
        S x[W];
        __builtin_memcpy(x, &r[k], 16);
#pragma unroll
        for (int j = 0; j < W; ++j) acc[j] = combine<DT, OP>(acc[j], E::load(x[j]));
      }
#pragma unroll
      for (int j = 0; j < W; ++j) acc_s[j] = E::store(acc[j]);
      u32x4 o;
      __builtin_memcpy(&o, acc_s, 16);
      out[u ? v1 : v] = o;
    }
  }
  // scalar tail (< W elements)
  const int64_t base = nvec * W;
  if (tid < n - base) {
    const int64_t i = base + tid;
    A acc = E::load(reinterpret_cast<const S*>(ins.p[0])[i]);
#pragma unroll
    for (int k = 1; k < NIN; ++k) acc = combine<DT, OP>(acc, E::load(reinterpret_cast<const S*>(ins.p[k])[i]));
    reinterpret_cast<S*>(out_)[i] = E::store(acc);
  }
}

// Tile variant: block b owns vectors [b*kBlock*U, (b+1)*kBlock*U); lane t handles
// b*kBlock*U + t + k*kBlock (k < U) — every load instruction of a wave covers 1 KiB contiguous,
// all U*NIN loads are issued before the first combine.  NT selects nontemporal loads/stores
// (streamed once, keep them out of L2/MALL).
template <typename T, bool NT>
__device__ __forceinline__ T ld(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <typename T, bool NT>
__device__ __forceinline__ void st(T* p, T v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int DT, int OP, int NIN, int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_reduce_tile(void* __restrict__ out_, InPtrs<NIN> ins, int64_t nvec,
                                                        int64_t n) {
  using E = Elem<DT>;
  using S = typename E::S;
  using A = typename E::A;
  constexpr int W = 16 / sizeof(S);
  u32x4* out = reinterpret_cast<u32x4*>(out_);
  // grid-stride over tiles when the launch caps the grid (MP4X_K1_GRID).  Default: no cap, one
  // tile per block — a capped grid measured no better for NIN = 1-2 and 20% slower for NIN >= 4
  // (profiles/r1/k1_grid_cap.txt), although a bare copy kernel gains 4% from it
  // (tools/exp/copy_variants.hip, profiles/r1/copy_variants.txt)
  const int64_t step = (int64_t)gridDim.x * kBlock * U;
  for (int64_t base = (int64_t)blockIdx.x * kBlock * U + threadIdx.x; base < nvec; base += step) {
  if (base + (int64_t)(U - 1) * kBlock < nvec) {
    u32x4 r[U][NIN];
#pragma unroll
    for (int k = 0; k < NIN; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) r[u][k] = ld<u32x4, NT>(reinterpret_cast<const u32x4*>(ins.p[k]) + base + u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      S a_s[W];
      __builtin_memcpy(a_s, &r[u][0], 16);
      A acc[W];
#pragma unroll
      for (int j = 0; j < W; ++j) acc[j] = E::load(a_s[j]);
#pragma unroll
      for (int k = 1; k < NIN; ++k) {
        S x[W];
        __builtin_memcpy(x, &r[u][k], 16);
#pragma unroll
        for (int j = 0; j < W; ++j) acc[j] = combine<DT, OP>(acc[j], E::load(x[j]));
      }
#pragma unroll
      for (int j = 0; j < W; ++j) a_s[j] = E::store(acc[j]);
      u32x4 o;
      __builtin_memcpy(&o, a_s, 16);
      st<u32x4, NT>(out + base + u * kBlock, o);
    }
  } else {
    for (int u = 0; u < U; ++u) {
      const int64_t v = base + (int64_t)u * kBlock;
      if (v >= nvec) break;
      S a_s[W];
      u32x4 t0 = reinterpret_cast<const u32x4*>(ins.p[0])[v];
      __builtin_memcpy(a_s, &t0, 16);
      A acc[W];
      for (int j = 0; j < W; ++j) acc[j] = E::load(a_s[j]);
      for (int k = 1; k < NIN; ++k) {
        S x[W];
        u32x4 tk = reinterpret_cast<const u32x4*>(ins.p[k])[v];
        __builtin_memcpy(x, &tk, 16);
        for (int j = 0; j < W; ++j) acc[j] = combine<DT, OP>(acc[j], E::load(x[j]));
      }
      for (int j = 0; j < W; ++j) a_s[j] = E::store(acc[j]);
      u32x4 o;
      __builtin_memcpy(&o, a_s, 16);
      out[v] = o;
    }
  }
  }
  // scalar tail handled by block 0
  if (blockIdx.x == 0) {
    const int64_t tb = nvec * W;
    if ((int64_t)threadIdx.x < n - tb) {
      const int64_t i = tb + threadIdx.x;
      A acc = E::load(reinterpret_cast<const S*>(ins.p[0])[i]);
      for (int k = 1; k < NIN; ++k) acc = combine<DT, OP>(acc, E::load(reinterpret_cast<const S*>(ins.p[k])[i]));
      reinterpret_cast<S*>(out_)[i] = E::store(acc);
    }
  }
}

static int64_t g_k1_grid = -1;
static int64_t k1_grid_cap() {
  if (g_k1_grid < 0) {
    const char* e = getenv("MP4X_K1_GRID");
    g_k1_grid = e ? atoll(e) : -2;     // unset: per fan-in default (k1_grid_for)
  }
  return g_k1_grid;
}
// Grid cap of a launch with NIN inputs: MP4X_K1_GRID when set (0 = one tile per block), else
// 8192 grid-strided blocks for the single-input copy (in-situ N=1 bench A/B, interleaved rounds:
// 2992 vs 2957 GB/s mean, profiles/r3/k1/n1_grid_cap_ab.txt) and one tile per block from two
// inputs up (a capped grid measured 20% slower at NIN >= 4, profiles/r1/k1_grid_cap.txt).
static int64_t k1_grid_for(int nin) {
  const int64_t c = k1_grid_cap();
  return c >= 0 ? c : (nin == 1 ? 8192 : 0);
}

static int g_k1_variant = -1;
static int k1_variant() {
  if (g_k1_variant < 0) {
    const char* e = getenv("MP4X_K1_VARIANT");
    g_k1_variant = e ? atoi(e) : 2;   // default: tile + nontemporal (fastest, tools/bench_kernels.py --variants)
  }
  return g_k1_variant;
}

template <int DT, int OP, int NIN>
__global__ __launch_bounds__(kBlock) void k_reduce_scalar(void* __restrict__ out_, InPtrs<NIN> ins, int64_t n) {
  using E = Elem<DT>;
  using S = typename E::S;
  using A = typename E::A;
  const int64_t nthr = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += nthr) {
    A acc = E::load(reinterpret_cast<const S*>(ins.p[0])[i]);
#pragma unroll
    for (int k = 1; k < NIN; ++k) acc = combine<DT, OP>(acc, E::load(reinterpret_cast<const S*>(ins.p[k])[i]));
    reinterpret_cast<S*>(out_)[i] = E::store(acc);
  }
}

template <int DT, int OP, int NIN>
static int launch_nin(void* out, const void* const* ins, int64_t n, hipStream_t st) {
  using S = typename Elem<DT>::S;
  constexpr int W = 16 / sizeof(S);
  InPtrs<NIN> p;
  bool aligned = ((uintptr_t)out % 16) == 0;
  for (int k = 0; k < NIN; ++k) {
    p.p[k] = ins[k];
    aligned = aligned && ((uintptr_t)ins[k] % 16) == 0;
  }
  if (aligned) {
    int64_t nvec = n / W;
    // the A/B variants (MP4X_K1_VARIANT, tools/bench_kernels.py --variants) are built for f32
    // only: every other dtype runs the default tile + nontemporal kernel (a quarter of the
    // template instantiations, which dominated the library's build time)
    const int var = DT == MP4X_F32 ? k1_variant() : 2;
    if constexpr (DT != MP4X_F32) {
      constexpr int U = NIN >= 4 ? 1 : (NIN == 3 ? 2 : 4);
      int64_t per_block = (int64_t)kBlock * U;
      int64_t g = (nvec + per_block - 1) / per_block;
      if (g < 1) g = 1;
      const int64_t cap = k1_grid_for(NIN);
      if (cap > 0 && g > cap) g = cap;
      hipLaunchKernelGGL((k_reduce_tile<DT, OP, NIN, U, true>), dim3((unsigned)g), dim3(kBlock), 0, st, out, p, nvec, n);
      (void)var;
    } else if (var == 0) {
      int g = grid_for(nvec > 0 ? nvec : 1, 2);
      hipLaunchKernelGGL((k_reduce_vec<DT, OP, NIN>), dim3(g), dim3(kBlock), 0, st, out, p, nvec, n);
    } else {
      // U vectors per lane: keep ~4-8 16-B loads in flight per lane (variant 3: ~8-16)
      // measured (tools/bench_kernels.py --variants, profiles/r1/k1_variants2.txt): 4 vectors per
      // lane for 1-2 inputs (6.1 / 6.4 TB/s), 1 vector per lane from 4 inputs up
      constexpr int U = NIN >= 4 ? 1 : (NIN == 3 ? 2 : 4);
      constexpr int U2 = NIN >= 8 ? 1 : (NIN >= 4 ? 2 : 4);
      const int u = var == 3 ? U2 : U;
      int64_t per_block = (int64_t)kBlock * u;
      int64_t g = (nvec + per_block - 1) / per_block;
      if (g < 1) g = 1;
      const int64_t cap = k1_grid_for(NIN);
      if (cap > 0 && g > cap) g = cap;
      if (var == 1)
        hipLaunchKernelGGL((k_reduce_tile<DT, OP, NIN, U, false>), dim3((unsigned)g), dim3(kBlock), 0, st, out, p, nvec, n);
      else if (var == 3)
        hipLaunchKernelGGL((k_reduce_tile<DT, OP, NIN, U2, true>), dim3((unsigned)g), dim3(kBlock), 0, st, out, p, nvec, n);
      else
        hipLaunchKernelGGL((k_reduce_tile<DT, OP, NIN, U, true>), dim3((unsigned)g), dim3(kBlock), 0, st, out, p, nvec, n);
    }
  } else {
    int g = grid_for(n, 4);
    hipLaunchKernelGGL((k_reduce_scalar<DT, OP, NIN>), dim3(g), dim3(kBlock), 0, st, out, p, n);
  }
  return (int)hipGetLastError();
}

template <int DT, int OP>
static int launch_op(void* out, const void* const* ins, int nin, int64_t n, hipStream_t st) {
  if constexpr (!op_valid<DT, OP>()) {
    return MP4X_E_UNSUPPORTED;
  } else {
    switch (nin) {
      case 1: return launch_nin<DT, OP, 1>(out, ins, n, st);
      case 2: return launch_nin<DT, OP, 2>(out, ins, n, st);
      case 3: return launch_nin<DT, OP, 3>(out, ins, n, st);
      case 4: return launch_nin<DT, OP, 4>(out, ins, n, st);
      case 5: return launch_nin<DT, OP, 5>(out, ins, n, st);
      case 6: return launch_nin<DT, OP, 6>(out, ins, n, st);
      case 7: return launch_nin<DT, OP, 7>(out, ins, n, st);
      case 8: return launch_nin<DT, OP, 8>(out, ins, n, st);
      default: return MP4X_E_BADARG;
    }
  }
}

template <int DT>
static int launch_dt(int op, void* out, const void* const* ins, int nin, int64_t n, hipStream_t st) {
  switch (op) {
    case MP4X_SUM: return launch_op<DT, MP4X_SUM>(out, ins, nin, n, st);
    case MP4X_MAX: return launch_op<DT, MP4X_MAX>(out, ins, nin, n, st);
    case MP4X_MIN: return launch_op<DT, MP4X_MIN>(out, ins, nin, n, st);
    case MP4X_PROD: return launch_op<DT, MP4X_PROD>(out, ins, nin, n, st);
    case MP4X_BAND: return launch_op<DT, MP4X_BAND>(out, ins, nin, n, st);
    case MP4X_BOR: return launch_op<DT, MP4X_BOR>(out, ins, nin, n, st);
    case MP4X_BXOR: return launch_op<DT, MP4X_BXOR>(out, ins, nin, n, st);
    case MP4X_FMAXLOC: return launch_op<DT, MP4X_FMAXLOC>(out, ins, nin, n, st);
    case MP4X_FMINLOC: return launch_op<DT, MP4X_FMINLOC>(out, ins, nin, n, st);
    case MP4X_IMAXLOC: return launch_op<DT, MP4X_IMAXLOC>(out, ins, nin, n, st);
    case MP4X_IMINLOC: return launch_op<DT, MP4X_IMINLOC>(out, ins, nin, n, st);
    default: return MP4X_E_BADARG;
  }
}

static int dispatch(int dtype, int op, void* out, const void* const* ins, int nin, int64_t n, hipStream_t st) {
  switch (dtype) {
    case MP4X_F64: return launch_dt<MP4X_F64>(op, out, ins, nin, n, st);
    case MP4X_F32: return launch_dt<MP4X_F32>(op, out, ins, nin, n, st);
    case MP4X_I64: return launch_dt<MP4X_I64>(op, out, ins, nin, n, st);
    case MP4X_I32: return launch_dt<MP4X_I32>(op, out, ins, nin, n, st);
    case MP4X_I16: return launch_dt<MP4X_I16>(op, out, ins, nin, n, st);
    case MP4X_I8: return launch_dt<MP4X_I8>(op, out, ins, nin, n, st);
    case MP4X_U8: return launch_dt<MP4X_U8>(op, out, ins, nin, n, st);
    case MP4X_BF16: return launch_dt<MP4X_BF16>(op, out, ins, nin, n, st);
    case MP4X_F16: return launch_dt<MP4X_F16>(op, out, ins, nin, n, st);
    default: return MP4X_E_BADARG;
  }
}

static int elem_size(int dtype) {
  switch (dtype) {
    case MP4X_F64: case MP4X_I64: return 8;
    case MP4X_F32: case MP4X_I32: return 4;
    case MP4X_I16: case MP4X_BF16: case MP4X_F16: return 2;
    case MP4X_I8: case MP4X_U8: return 1;
    default: return 0;
  }
}

// ---------------------------------------------------------------- scale (averaging)
template <int DT>
__global__ __launch_bounds__(kBlock) void k_scale(void* out_, const void* in_, double scale, int64_t n) {
  using E = Elem<DT>;
  using S = typename E::S;
  using A = typename E::A;
  const int64_t nthr = (int64_t)gridDim.x * kBlock;
  const S* in = reinterpret_cast<const S*>(in_);
  S* out = reinterpret_cast<S*>(out_);
  const A s = (A)scale;
  const int64_t t0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  int64_t done = 0;
  if (((((uintptr_t)in | (uintptr_t)out) & 15) == 0)) {   // 16-byte vectors (the bf16 / f16 rows too)
    constexpr int W = 16 / (int)sizeof(S);
    const int64_t nv = n / W;
    const u32x4* vin = reinterpret_cast<const u32x4*>(in);
    u32x4* vout = reinterpret_cast<u32x4*>(out);
    for (int64_t v = t0; v < nv; v += nthr) {
      u32x4 t = __builtin_nontemporal_load(vin + v);
      S x[W];
      __builtin_memcpy(x, &t, 16);
#pragma unroll
      for (int j = 0; j < W; ++j) x[j] = E::store(E::load(x[j]) * s);
      __builtin_memcpy(&t, x, 16);
      __builtin_nontemporal_store(t, vout + v);
    }
    done = nv * W;
  }
  for (int64_t i = done + t0; i < n; i += nthr) out[i] = E::store(E::load(in[i]) * s);
}

}  // namespace mp4x

using namespace mp4x;

extern "C" int mp4x_reduce(int dtype, int op, void* out, const void* const* ins, int nin, int64_t n, void* stream) {
  if (n <= 0) return 0;
  if (nin < 1 || !out || !ins) return MP4X_E_BADARG;
  hipStream_t st = (hipStream_t)stream;
  if (nin == 1 && out == ins[0]) return 0;
  // chain fan-in > 8: out = op(in0..in7); out = op(out, in8..in14); ...
  const void* buf[MP4X_MAX_NIN];
  int done = 0;
  int rc = 0;
  bool first = true;
  while (done < nin) {
    int k = 0;
    if (!first) buf[k++] = out;
    while (k < MP4X_MAX_NIN && done < nin) buf[k++] = ins[done++];
    rc = dispatch(dtype, op, out, buf, k, n, st);
    if (rc) return rc;
    first = false;
  }
  return rc;
}

extern "C" int mp4x_reduce_strided(int dtype, int op, void* out, const void* base, int64_t stride_elems, int nin,
                                   int64_t n, void* stream) {
  int es = elem_size(dtype);
  if (!es || nin < 1 || nin > 64) return MP4X_E_BADARG;
  const void* ptrs[64];
  for (int k = 0; k < nin; ++k) ptrs[k] = (const char*)base + (int64_t)k * stride_elems * es;
  return mp4x_reduce(dtype, op, out, ptrs, nin, n, stream);
}

extern "C" int mp4x_scale(int dtype, void* out, const void* in, double scale, int64_t n, void* stream) {
  if (n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  int g = grid_for(n, 4);
  switch (dtype) {
    case MP4X_F64: hipLaunchKernelGGL(k_scale<MP4X_F64>, dim3(g), dim3(kBlock), 0, st, out, in, scale, n); break;
    case MP4X_F32: hipLaunchKernelGGL(k_scale<MP4X_F32>, dim3(g), dim3(kBlock), 0, st, out, in, scale, n); break;
    case MP4X_BF16: hipLaunchKernelGGL(k_scale<MP4X_BF16>, dim3(g), dim3(kBlock), 0, st, out, in, scale, n); break;
    case MP4X_F16: hipLaunchKernelGGL(k_scale<MP4X_F16>, dim3(g), dim3(kBlock), 0, st, out, in, scale, n); break;
    default: return MP4X_E_UNSUPPORTED;
  }
  return (int)hipGetLastError();
}

// A/B hook for the kernel-variant sweep (tools/bench_kernels.py --variants).
extern "C" void mp4x_set_k1_variant(int v) { g_k1_variant = v; }
extern "C" void mp4x_set_k1_grid(int64_t cap) { g_k1_grid = cap; }

extern "C" const char* mp4x_version(void) { return "mp4x-native 0.1 gfx950"; }

// Reads and clears this thread's last HIP error.  mp4x reports its own failures through return
// codes; a failed HIP call must not stay "last error" for PyTorch's next kernel-launch check to
// report as its own (native.check() and the best-effort release paths call this).
extern "C" int mp4x_clear_error(void) { return (int)hipGetLastError(); }

extern "C" int mp4x_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
