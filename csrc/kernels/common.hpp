// Shared device helpers for the mp4x CDNA4 kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mp4x/ops.h"

namespace mp4x {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Device-side bounds checks of the debug build (tools/build_native.py --debug): report and trap
// the wave, so a bad index fails at its source instead of as a later memory fault.
#ifdef MP4X_DEBUG
#define MP4X_DASSERT(cond)                                                                     \
  do {                                                                                         \
    if (!(cond)) {                                                                             \
      printf("mp4x device assert failed: %s (%s:%d) block %d thread %d\n", #cond, __FILE__,    \
             __LINE__, (int)blockIdx.x, (int)threadIdx.x);                                     \
      __builtin_trap();                                                                        \
    }                                                                                          \
  } while (0)
#else
#define MP4X_DASSERT(cond) ((void)0)
#endif

constexpr int kBlock = 256;          // 4 wave64 per workgroup

// Global wave index of a kBlock-thread workgroup, made provably wave-uniform
// (readfirstlane): everything derived from it (block indices, mask / offset loads) then
// lives in SGPRs and is fetched with scalar loads instead of 64 copies in VGPRs.
__device__ __forceinline__ int64_t wave_id() {
  return (int64_t)blockIdx.x * (kBlock / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}
constexpr int kMaxGrid = 256 * 8;    // 256 CUs x 8 resident blocks: grid-stride beyond this

inline int grid_for(int64_t work_items, int per_thread = 1) {
  int64_t per_block = (int64_t)kBlock * per_thread;
  int64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > kMaxGrid) g = kMaxGrid;
  return (int)g;
}

// ---------------------------------------------------------------- 16-bit float helpers
__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);                                          // round to nearest even
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float f16_to_f32(uint16_t h) {
  _Float16 x;
  __builtin_memcpy(&x, &h, 2);
  return (float)x;
}
__device__ __forceinline__ uint16_t f32_to_f16(float f) {
  _Float16 x = (_Float16)f;
  uint16_t h;
  __builtin_memcpy(&h, &x, 2);
  return h;
}

// ---------------------------------------------------------------- element traits
// Storage type S, accumulator type A, conversions.
template <int DT> struct Elem;
template <> struct Elem<MP4X_F64> { using S = double; using A = double;
  static __device__ A load(S s) { return s; } static __device__ S store(A a) { return a; } };
template <> struct Elem<MP4X_F32> { using S = float; using A = float;
  static __device__ A load(S s) { return s; } static __device__ S store(A a) { return a; } };
template <> struct Elem<MP4X_I64> { using S = int64_t; using A = int64_t;
  static __device__ A load(S s) { return s; } static __device__ S store(A a) { return a; } };
template <> struct Elem<MP4X_I32> { using S = int32_t; using A = int32_t;
  static __device__ A load(S s) { return s; } static __device__ S store(A a) { return a; } };
template <> struct Elem<MP4X_I16> { using S = int16_t; using A = int16_t;
  static __device__ A load(S s) { return s; } static __device__ S store(A a) { return a; } };
template <> struct Elem<MP4X_I8> { using S = int8_t; using A = int8_t;
  static __device__ A load(S s) { return s; } static __device__ S store(A a) { return a; } };
template <> struct Elem<MP4X_U8> { using S = uint8_t; using A = uint8_t;
  static __device__ A load(S s) { return s; } static __device__ S store(A a) { return a; } };
template <> struct Elem<MP4X_BF16> { using S = uint16_t; using A = float;
  static __device__ A load(S s) { return bf16_to_f32(s); } static __device__ S store(A a) { return f32_to_bf16(a); } };
template <> struct Elem<MP4X_F16> { using S = uint16_t; using A = float;
  static __device__ A load(S s) { return f16_to_f32(s); } static __device__ S store(A a) { return f32_to_f16(a); } };

template <int DT> constexpr bool is_float_dt() {
  return DT == MP4X_F64 || DT == MP4X_F32 || DT == MP4X_BF16 || DT == MP4X_F16;
}

// Which (dtype, op) pairs exist (mirrors the reference operator table + 16-bit floats).
template <int DT, int OP> constexpr bool op_valid() {
  if (OP == MP4X_SUM || OP == MP4X_MAX || OP == MP4X_MIN || OP == MP4X_PROD || OP == MP4X_FIRST) return true;
  if (OP == MP4X_BAND || OP == MP4X_BOR || OP == MP4X_BXOR) return !is_float_dt<DT>();
  if (OP == MP4X_FMAXLOC || OP == MP4X_FMINLOC) return DT == MP4X_F64;
  if (OP == MP4X_IMAXLOC || OP == MP4X_IMINLOC) return DT == MP4X_I64;
  return false;
}

template <typename T> struct Unsigned { using U = T; };
template <> struct Unsigned<int64_t> { using U = uint64_t; };
template <> struct Unsigned<int32_t> { using U = uint32_t; };
template <> struct Unsigned<int16_t> { using U = uint16_t; };
template <> struct Unsigned<int8_t> { using U = uint8_t; };

// combine(a, b): `a` is the accumulated (local / earlier) value, `b` the incoming one —
// the argument order of the reference's fused recv+reduce (DoubleOperand.java:196).
template <int DT, int OP>
__device__ __forceinline__ typename Elem<DT>::A combine(typename Elem<DT>::A a, typename Elem<DT>::A b) {
  using A = typename Elem<DT>::A;
  if constexpr (OP == MP4X_FIRST) {
    (void)b;
    return a;
  } else if constexpr (OP == MP4X_SUM) {
    if constexpr (is_float_dt<DT>()) return a + b;
    else { using U = typename Unsigned<A>::U; return (A)((U)a + (U)b); }
  } else if constexpr (OP == MP4X_PROD) {
    if constexpr (is_float_dt<DT>()) return a * b;
    else { using U = typename Unsigned<A>::U; return (A)((U)a * (U)b); }
  } else if constexpr (OP == MP4X_MAX) {
    if constexpr (is_float_dt<DT>()) return (a != a) ? a : ((b != b) ? b : (a >= b ? a : b));  // Java Math.max NaN rule
    else return a >= b ? a : b;
  } else if constexpr (OP == MP4X_MIN) {
    if constexpr (is_float_dt<DT>()) return (a != a) ? a : ((b != b) ? b : (a <= b ? a : b));
    else return a <= b ? a : b;
  } else if constexpr (OP == MP4X_BAND) {
    return a & b;
  } else if constexpr (OP == MP4X_BOR) {
    return a | b;
  } else if constexpr (OP == MP4X_BXOR) {
    return a ^ b;
  } else if constexpr (OP == MP4X_FMAXLOC || OP == MP4X_FMINLOC) {
    uint64_t ua, ub;
    __builtin_memcpy(&ua, &a, 8);
    __builtin_memcpy(&ub, &b, 8);
    float va = __uint_as_float((uint32_t)(ua >> 32)), vb = __uint_as_float((uint32_t)(ub >> 32));
    bool keep = (OP == MP4X_FMAXLOC) ? (va >= vb) : (va <= vb);   // ties keep the first argument
    return keep ? a : b;
  } else {  // IMAXLOC / IMINLOC on int64 words
    int32_t va = (int32_t)((uint64_t)a >> 32), vb = (int32_t)((uint64_t)b >> 32);
    bool keep = (OP == MP4X_IMAXLOC) ? (va >= vb) : (va <= vb);
    return keep ? a : b;
  }
}

}  // namespace mp4x
