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

// Launch-planner knobs (knobs.hip): tested defaults, switched only by tests / probes through fd_set_knob.
enum fd_knob_id {
  FDK_GEMM8, FDK_GEMM8_S, FDK_GEMM8_GM, FDK_GEMM8_W160, FDK_GEMM8_LNP, FDK_GEMM8_MIDK, FDK_F8_TILE, FDK_GEMM_CFG,
  FDK_GEMM_SWZ, FDK_GEMM_MODE, FDK_GEMV, FDK_GEMM256, FDK_GEMM256_MIN_TILES,
  FDK_GN_MIN_CHUNKS, FDK_GN_APPLY_V, FDK_GN_APPLY_BLOCKS, FDK_GN_APPLY_U, FDK_FLASH_SWZ, FDK_FLASH_WAVES,
  FDK_FLASH_QPW, FDK_CONV_HALO, FDK_CONV_HALO_MIN_TILES, FDK_CONV_HALO_SPLIT, FDK_GEMM_GMP, FDK_CONV_HALO_PT,
  FDK_CONV_HALO_NS16, FDK_CONV_HALO_SPLIT16, FDK_CONV_HALO_PP, FDK_COUNT
};
int fd_knob(int id);
// gemm256.hip: whether fd_gemm256_try takes this launch
int gemm256_takes(const fd_gemm_params* p);
extern "C" int fd_conv_halo_try(fd_gemm_params* p, void* stream);
// split-K hand-off health per translation unit (gemm8.hip, conv_halo.hip); fd_splitk_health sums them
int g8_splitk_health(unsigned* timeouts, int reset, int drop);
int halo_splitk_health(unsigned* timeouts, int reset, int drop);

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

// Cache policy of the output stores of the GEMM / conv epilogues, GroupNorm apply, concat and flash attention
// (FD_EPI_WT, build time): 0 plain (write-back L2: the kernel-end release then writes every dirty line back, after
// the last wave), 1 sc1 (device scope: written through as stored, nothing left dirty at the end), 2 nt, 4 sc1 nt.
// The policy bits ride on a buffer store (raw_buffer_store_b128 / _b64 with the cache-policy operand), which the
// compiler sees -- its waitcnt pass and hazard recognizer account for it.  (Round 5 used inline-asm global stores
// with a hand-placed s_nop after the compiler put a VALU write into a store's data VGPRs right behind it.)  The
// buffer resource is wave-uniform: the first active lane's address - 2^31, so each lane's 32-bit offset is
// 2^31 + (its address - that lane's); every caller's per-instruction span across a wave is far below 2 GiB.
#ifndef FD_EPI_WT
#define FD_EPI_WT 1
#endif
constexpr int kWtAux = FD_EPI_WT == 1 ? 16 : FD_EPI_WT == 2 ? 2 : FD_EPI_WT == 4 ? 18 : 0;  // gfx950 cpol: sc1 16, nt 2
// Cache-policy bits of the GEMM / conv weight-operand LDS-DMA loads (build-time A/B): 0 default, 2 nt
#ifndef FD_WLD_AUX
#define FD_WLD_AUX 0
#endif
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* p, unsigned& voff) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const unsigned long long base = (((unsigned long long)hi << 32) | lo) - 0x80000000ull;
  voff = (unsigned)(a - base);
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)0xffffffff, 0x00020000);
}
// 16-B store (other widths: plain)
template <typename V>
__device__ __forceinline__ void st_out16(V* p, const V& v) {
  if constexpr (FD_EPI_WT == 0 || sizeof(V) != 16) {
    *p = v;
  } else {
    unsigned off;
    const __amdgpu_buffer_rsrc_t rs = wt_rsrc(p, off);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, off, 0, kWtAux);
  }
}
// 8-B store (other widths: plain)
template <typename V>
__device__ __forceinline__ void st_out8(V* p, const V& v) {
  if constexpr (FD_EPI_WT == 0 || sizeof(V) != 8) {
    *p = v;
  } else {
    unsigned off;
    const __amdgpu_buffer_rsrc_t rs = wt_rsrc(p, off);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rs, off, 0, kWtAux);
  }
}

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
// Round an fp32 result to T in two steps (fp32 first, then T), as torch's half kernels do.  Without the empty asm
// the backend may fuse fma + convert into v_fma_mixlo_f16, which rounds the exact product-sum to f16 once: a
// different f16 value at double-rounding ties, so two kernels that should agree bitwise would not.
template <typename T> __device__ __forceinline__ T round_f32(float x) {
  asm("" : "+v"(x));
  return (T)x;
}

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

// Epilogue activations, branch-free: the quotient by v_rcp_f32 (1 ulp) instead of the ~10-instruction IEEE
// division, and erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, one v_rcp + one v_exp) instead of ocml's
// erff, whose two polynomial branches both run in a mixed-sign wave (~40 VALU per element: the GEGLU epilogue
// of the 2048 x 10240 projection spent ~10 us in it).  Both far below the bf16 / fp16 rounding of the stored value.
__device__ __forceinline__ float silu_f(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
// GELU(x) = x * Phi(x) (diffusers GELU / GEGLU, approximate="none") as x * sigmoid(z(x)) with z = logit(Phi(x)) fitted as
// an odd polynomial x * (c0 + c1 x^2 + c2 x^4) on |x| <= 5.5, x clamped there (beyond it Phi is 0 or 1 to within 2e-8);
// -log2(e) folded into the coefficients (scripts/gelu_fit.py).  Max |error| 2.6e-5 over the real line in fp32, far
// inside the bf16 rounding of the output; 7 plain + 2 transcendental VALU ops where the Abramowitz-Stegun 7.1.26 erf
// form (max |error| 1.5e-7) took 14 + 2 -- the GEGLU epilogue runs with no MFMA beside it.
#ifndef FD_GELU_AS
#define FD_GELU_AS 0  // A/B builds only: 1 = the round-5 Abramowitz-Stegun 7.1.26 erf form
#endif
__device__ __forceinline__ float gelu_f(float x) {
  if constexpr (FD_GELU_AS) {
    const float z = x * 0.70710678118654752f, a = fabsf(z);
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.0f));
    const float y =
        t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f), 0.254829592f);
    return 0.5f * x * (1.0f + copysignf(fmaf(-y, __expf(-a * a), 1.0f), z));
  }
  const float xc = __builtin_amdgcn_fmed3f(x, -5.5f, 5.5f);
  const float x2 = xc * xc;
  const float p = fmaf(fmaf(1.014481299e-03f, x2, -1.067767218e-01f), x2, -2.301120520e+00f) * xc;
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(p));
}
__device__ __forceinline__ float quickgelu_f(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * x)); }
// LeakyReLU(negative_slope = 0.2) of the BSRNet pre-pass (bsrnet_arch.py:52, nn.LeakyReLU(0.2))
__device__ __forceinline__ float lrelu_f(float x) { return x >= 0.f ? x : 0.2f * x; }

__device__ __forceinline__ float act_f(float v, int act) {
  switch (act) {
    case FD_ACT_SILU: return silu_f(v);
    case FD_ACT_GELU: return gelu_f(v);
    case FD_ACT_QUICKGELU: return quickgelu_f(v);
    case FD_ACT_LRELU: return lrelu_f(v);
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

// GroupNorm statistics of a 256-row (or 128-row) GEMM / conv output tile (fd_gemm_params.gn_part): in the vector epilogue
// each thread owns one 8-column chunk (NTHR % VPR == 0), whose columns fall in at most two groups (cpg >= 4 and
// the tile's first column a multiple of cpg); sums of the STORED values, then one fixed-order reduction per group.
struct GnTile {
  float s0 = 0.f, q0 = 0.f, s1 = 0.f, q1 = 0.f;
  template <typename TO8>
  __device__ __forceinline__ void add(const TO8& o, int split) {  // chunk columns < split: the first group
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float f = (float)o[i];
      if (i < split) {
        s0 += f;
        q0 += f * f;
      } else {
        s1 += f;
        q1 += f * f;
      }
    }
  }
};
// red: 2 * nthr float2 of LDS no other thread still reads; every thread of the workgroup calls this
__device__ __forceinline__ void gn_tile_write(const GnTile& a, float2* red, int tid, int nthr, int vpr, int cpg,
                                              int ncols, int n0, int m0, const fd_gemm_params& p, int rows = 256) {
  red[2 * tid] = make_float2(a.s0, a.q0);
  red[2 * tid + 1] = make_float2(a.s1, a.q1);
  __syncthreads();
  if (tid < ncols / cpg) {
    float s = 0.f, q = 0.f;
    for (int c = tid * cpg / 8; c <= ((tid + 1) * cpg - 1) / 8; ++c) {
      const int slot = (c * 8) / cpg == tid ? 0 : 1;
      for (int k = c; k < nthr; k += vpr) {
        const float2 v = red[2 * k + slot];
        s += v.x;
        q += v.y;
      }
    }
    const long long blk = (long long)(m0 / p.gn_hw) * (p.gn_hw / rows) + (m0 % p.gn_hw) / rows;
    ((float2*)p.gn_part)[blk * p.gn_groups + n0 / cpg + tid] = make_float2(s, q);
  }
}

// OCP MX e4m3 (32-element blocks, one E8M0 scale byte each): the block's scale exponent E is the least one with
// amax <= 448 * 2^E (448 = 1.75 * 2^8, so no element saturates), q = RNE_e4m3(v * 2^-E) (the scaling is exact),
// byte = E + 127.  All-zero (or NaN) blocks: E = 0.  Shared by every MX producer so they write the same bytes.
__device__ __forceinline__ int mx_exp(float amax) {
  if (!(amax > 0.f)) return 0;
  const unsigned b = __float_as_uint(amax);
  const int e = (int)((b >> 23) & 255u) - 127;
  const int E = (b & 0x7fffffu) <= 0x600000u ? e - 8 : e - 7;
  return E < -127 ? -127 : (E > 127 ? 127 : E);
}
// 4 floats * 2^-E -> 4 e4m3 bytes (RNE) in one dword, element 0 in the low byte
__device__ __forceinline__ unsigned mx_pack4(float a, float b, float c, float d, int E) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_ldexpf(a, -E), __builtin_amdgcn_ldexpf(b, -E), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_ldexpf(c, -E), __builtin_amdgcn_ldexpf(d, -E), w, true);
  return (unsigned)w;
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
