// Shared device helpers for libfaithdiff_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/faithdiff_hip.h"

typedef __bf16 bf16;
typedef _Float16 f16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

template <typename T> struct VecT;
template <> struct VecT<bf16> { typedef bf16x8 v8; };
template <> struct VecT<f16> { typedef f16x8 v8; };

__device__ __forceinline__ f32x4 mfma16x16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16x16x32(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

template <typename T> __device__ __forceinline__ float to_f32(T x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x) { return (T)x; }

// load/store helpers over the three storage types
template <typename T> __device__ __forceinline__ float ldf(const void* p, long long i) {
  return (float)((const T*)p)[i];
}
template <typename T> __device__ __forceinline__ void stf(void* p, long long i, float v) {
  ((T*)p)[i] = (T)v;
}

// Workgroups are dealt round-robin to the 8 XCDs (b and b+8 share one; each XCD has its own 4 MiB L2).
// Bijective remap giving XCD x the contiguous logical range [x*q + min(x, r), ...) of the nwg blocks, so
// neighbouring logical blocks (same weight panel, same attention head) share an L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + __expf(-x)); }
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float quickgelu_f(float x) { return x / (1.0f + __expf(-1.702f * x)); }

__device__ __forceinline__ float act_f(float v, int act) {
  switch (act) {
    case FD_ACT_SILU: return silu_f(v);
    case FD_ACT_GELU: return gelu_f(v);
    case FD_ACT_QUICKGELU: return quickgelu_f(v);
    default: return v;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

#define FD_LAUNCH_CHECK()                                  \
  do {                                                     \
    if (hipGetLastError() != hipSuccess) return FD_ERR_HIP; \
  } while (0)

#define FD_DISPATCH_T(dtype, ...)          \
  if ((dtype) == FD_BF16) {                \
    typedef bf16 T;                        \
    __VA_ARGS__;                           \
  } else if ((dtype) == FD_F16) {          \
    typedef f16 T;                         \
    __VA_ARGS__;                           \
  } else {                                 \
    return FD_ERR_DTYPE;                   \
  }

#define FD_DISPATCH_O(odtype, ...)         \
  if ((odtype) == FD_BF16) {               \
    typedef bf16 TO;                       \
    __VA_ARGS__;                           \
  } else if ((odtype) == FD_F16) {         \
    typedef f16 TO;                        \
    __VA_ARGS__;                           \
  } else if ((odtype) == FD_F32) {         \
    typedef float TO;                      \
    __VA_ARGS__;                           \
  } else {                                 \
    return FD_ERR_DTYPE;                   \
  }
