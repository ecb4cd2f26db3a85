// Block-scaled e4m3 (OCP fp8, gfx950-native) device helpers shared by the K6 codec kernels
// (codec.hip) and the fused fp8 IPC two-shot allreduce (runtime/ipc.hip).
#pragma once

#include "common.hpp"

namespace mp4x {

constexpr int kQBlock = 256;        // elements per scale
constexpr float kFp8Max = 448.0f;   // e4m3fn max finite

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

template <int DT>
__device__ __forceinline__ void load4(const void* p, int64_t e, int64_t n, float (&x)[4]) {
  using E = Elem<DT>;
  using S = typename E::S;
  const S* s = reinterpret_cast<const S*>(p);
  if (e + 3 < n) {
    if constexpr (sizeof(S) == 4) {
      u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s + e));   // streamed once
      S t[4];
      __builtin_memcpy(t, &v, 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = (float)E::load(t[j]);
    } else if constexpr (sizeof(S) == 2) {
      uint2 v = *reinterpret_cast<const uint2*>(s + e);
      S t[4];
      __builtin_memcpy(t, &v, 8);
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = (float)E::load(t[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = (float)E::load(s[e + j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = (e + j < n) ? (float)E::load(s[e + j]) : 0.0f;
  }
}

template <int DT>
__device__ __forceinline__ void store4(void* p, int64_t e, int64_t n, const float (&x)[4]) {
  using E = Elem<DT>;
  using S = typename E::S;
  S* s = reinterpret_cast<S*>(p);
  if (e + 3 < n) {
    S t[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) t[j] = E::store((typename E::A)x[j]);
    if constexpr (sizeof(S) == 4) {
      u32x4 v;
      __builtin_memcpy(&v, t, 16);
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(s + e));
    } else if constexpr (sizeof(S) == 2) {
      uint2 v;
      __builtin_memcpy(&v, t, 8);
      *reinterpret_cast<uint2*>(s + e) = v;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) s[e + j] = t[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (e + j < n) s[e + j] = E::store((typename E::A)x[j]);
  }
}

__device__ __forceinline__ uint32_t pack_fp8(const float (&x)[4], float inv) {
  float a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = fminf(fmaxf(x[j] * inv, -kFp8Max), kFp8Max);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a[0], a[1], 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(a[2], a[3], w, true);
  return (uint32_t)w;
}

__device__ __forceinline__ void quant_block(const float (&x)[4], uint32_t* q, float* scales, int64_t blk, int lane) {
  float m = fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3])));
  m = wave_max(m);
  const float scale = m > 0.0f ? m / kFp8Max : 1.0f;
  __builtin_nontemporal_store(pack_fp8(x, 1.0f / scale), q + blk * 64 + lane);
  if (lane == 0) scales[blk] = scale;
}

// acc += dequant(w) * s as explicit FMAs: the codec's dequant-reduce and the fused IPC fp8
// two-shot share this, so both give bit-identical sums (no reliance on fp-contract choices)
__device__ __forceinline__ void fp8_fma_acc(uint32_t w, float s, float (&acc)[4]) {
  acc[0] = __builtin_fmaf(__builtin_amdgcn_cvt_f32_fp8((int)w, 0), s, acc[0]);
  acc[1] = __builtin_fmaf(__builtin_amdgcn_cvt_f32_fp8((int)w, 1), s, acc[1]);
  acc[2] = __builtin_fmaf(__builtin_amdgcn_cvt_f32_fp8((int)w, 2), s, acc[2]);
  acc[3] = __builtin_fmaf(__builtin_amdgcn_cvt_f32_fp8((int)w, 3), s, acc[3]);
}

// dequantise one dword of 4 packed e4m3 values with the block scale
__device__ __forceinline__ void unpack_fp8(uint32_t w, float s, float (&x)[4]) {
  x[0] = __builtin_amdgcn_cvt_f32_fp8((int)w, 0) * s;
  x[1] = __builtin_amdgcn_cvt_f32_fp8((int)w, 1) * s;
  x[2] = __builtin_amdgcn_cvt_f32_fp8((int)w, 2) * s;
  x[3] = __builtin_amdgcn_cvt_f32_fp8((int)w, 3) * s;
}

}  // namespace mp4x
