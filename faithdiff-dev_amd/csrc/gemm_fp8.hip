// OCP e4m3 GEMM on the gfx950 block-scaled MFMA (v_mfma_scale_f32_16x16x128_f8f6f4) -- the fp8 leg of
// the reference's quantize_8bit (utils/system.py:13-32) stores every UNet weight
// as unscaled float8_e4m3fn; here those bytes ARE the B operand (no widening), and the activations are
// quantized per row to e4m3 with an fp32 scale (fd_quant_rows_e4m3), so both operands run on the fp8
// matrix pipe at 2x the bf16 rate with half the operand bytes.
//
//   C[m][n] = out( act(a_scale[m] * w_scale * sum_k A8[m][k] * W8[n][k] + bias[n]) + residual[m][n] )
//   (act = SiLU / GELU / QuickGELU, or GEGLU over packed [hidden | gate] row groups -> N/2 columns)
//
// Tiles: 128x128 (or 64x128 when 128-row tiles cannot fill 256 CUs) per 256-thread workgroup, 2x2 waves,
// K-step 128 bytes.  These 4-wave kernels take ragged K only (K % 128 != 0); K % 128 == 0 runs on the eight-wave
// family (gemm8.hip).  Operands go global -> registers (next K-step prefetched while the MFMAs run) ->
// double-buffered LDS (144-B pitch: the 16 rows one ds_read_b128 phase touches land on 16 disjoint 4-bank groups)
// -> fragments.
// MFMA operand map (16x16x128, 8-bit): lane l holds row (l & 15), k = 32*(l >> 4) + j, j = 0..31,
// i.e. 32 contiguous bytes of one row; C/D: col = l & 15, row = 4*(l >> 4) + r.
#include <stdlib.h>

#include "fd_common.h"

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(2))) int i32x2;

namespace {
constexpr int F8_BN = 128, F8_BK = 128;
constexpr int F8_PITCH = F8_BK + 16;
constexpr int F8_NT = 256;

__device__ __forceinline__ f32x4 mfma_e4m3(const i32x8& a, const i32x8& b, f32x4 c) {
  // cbsz = blgp = 0 -> both operands e4m3; E8M0 block scales 127 = 2^0 (per-row scaling happens in the epilogue)
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}

// ROWS x 128 bytes of a row-major [rows][ld] e4m3 matrix -> ROWS/32 x 16 B per thread, zero outside.
template <int ROWS>
__device__ __forceinline__ void f8_load_tile(const uint8_t* __restrict__ base, long long ld, int r0, int rows,
                                             int k0, int K, u32x4 (&r)[ROWS / 32]) {
#pragma unroll
  for (int i = 0; i < ROWS / 32; ++i) {
    const int c = threadIdx.x + i * F8_NT;
    const int row = c >> 3, kc = k0 + (c & 7) * 16;
    if (r0 + row < rows && kc < K)
      r[i] = *(const u32x4*)(base + (long long)(r0 + row) * ld + kc);
    else
      r[i] = u32x4{0u, 0u, 0u, 0u};
  }
}

template <int ROWS>
__device__ __forceinline__ void f8_store_tile(uint8_t* lds, const u32x4 (&r)[ROWS / 32]) {
#pragma unroll
  for (int i = 0; i < ROWS / 32; ++i) {
    const int c = threadIdx.x + i * F8_NT;
    *(u32x4*)(lds + (c >> 3) * F8_PITCH + (c & 7) * 16) = r[i];
  }
}

__device__ __forceinline__ i32x8 f8_frag(const uint8_t* lds, int row, int lane) {
  const uint8_t* p = lds + row * F8_PITCH + (lane >> 4) * 32;
  const u32x4 lo = *(const u32x4*)p, hi = *(const u32x4*)(p + 16);
  return i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
}

// Epilogue shared by both e4m3 kernels: acc[i][j] = C[m0 + wm + 16 i + 4 (lane >> 4) + r][n0 + wn + 16 j + (lane & 15)].
template <typename TO, int MI>
__device__ __forceinline__ void f8_epilogue(const f32x4 (&acc)[MI][4], int m0, int n0, int wm, int wn, int lane,
                                            const float* __restrict__ a_scale, float w_scale, TO* __restrict__ C,
                                            long long ldc, int M, int N, const float* __restrict__ bias,
                                            const TO* __restrict__ R, long long ldr, int act) {
  // epilogue: per-row activation scale x weight scale, bias, residual; 16 lanes store 16 adjacent columns.
  // GEGLU: W rows are packed [16 hidden | 16 gate] per 32 (ops.pack_geglu), so a wave's column tiles j = 0,1
  // and 2,3 are the hidden / gate halves of output columns ((n0 + wn) / 32 + j / 2) * 16 + (lane & 15).
#pragma unroll
  for (int i = 0; i < MI; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
      if (m >= M) continue;
      const float s = a_scale[m] * w_scale;
      if (act == FD_ACT_GEGLU) {
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          const int nh = n0 + wn + g * 32 + (lane & 15);
          if (nh >= N) continue;
          // explicit fma / product roundings (no compiler contraction): the eight-wave kernel's form, same bits
          const float hv = __builtin_fmaf(acc[i][2 * g][r], s, bias ? bias[nh] : 0.f);
          const float gv = __builtin_fmaf(acc[i][2 * g + 1][r], s, bias ? bias[nh + 16] : 0.f);
          const int o = ((n0 + wn) / 32 + g) * 16 + (lane & 15);
          float v = __fmul_rn(hv, gelu_f(gv));
          if (R) v += (float)R[(long long)m * ldr + o];
          C[(long long)m * ldc + o] = (TO)v;
        }
        continue;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn + j * 16 + (lane & 15);
        if (n >= N) continue;
        float v = __fmul_rn(acc[i][j][r], s);
        if (bias) v += bias[n];
        if (act != FD_ACT_NONE) v = act_f(v, act);
        if (R) v += (float)R[(long long)m * ldr + n];
        C[(long long)m * ldc + n] = (TO)v;
      }
    }
  }
}

// BM x 128 tile per workgroup: 2x2 waves of (BM/2) x 64.  LDS is double-buffered: K-step kt+1's operands
// are loaded to registers before kt's MFMAs and written to the other buffer after them, so one barrier per
// K-step orders both the reads of buffer kt and the writes of buffer kt+1.
template <typename TO, int BM>
__global__ __launch_bounds__(F8_NT) void gemm_e4m3_kernel(const uint8_t* __restrict__ A, long long lda,
                                                           const float* __restrict__ a_scale,
                                                           const uint8_t* __restrict__ W, long long ldw,
                                                           float w_scale, TO* __restrict__ C, long long ldc, int M,
                                                           int N, int K, const float* __restrict__ bias,
                                                           const TO* __restrict__ R, long long ldr, int act) {
  constexpr int MI = BM / 32;  // 16-row MFMA tiles per wave
  __shared__ __attribute__((aligned(16))) uint8_t lds_a[2][BM * F8_PITCH];
  __shared__ __attribute__((aligned(16))) uint8_t lds_b[2][F8_BN * F8_PITCH];
  const int tn = (N + F8_BN - 1) / F8_BN, tm = (M + BM - 1) / BM;
  const int b = xcd_remap(blockIdx.x, tn * tm);  // neighbouring tiles (same A row panel) share one XCD's L2
  const int m0 = (b / tn) * BM, n0 = (b % tn) * F8_BN;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = (wid >> 1) * (BM / 2), wn = (wid & 1) * 64;

  f32x4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[BM / 32], rb[F8_BN / 32];
  const int nk = (K + F8_BK - 1) / F8_BK;
  f8_load_tile<BM>(A, lda, m0, M, 0, K, ra);
  f8_load_tile<F8_BN>(W, ldw, n0, N, 0, K, rb);
  f8_store_tile<BM>(lds_a[0], ra);
  f8_store_tile<F8_BN>(lds_b[0], rb);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {  // next K-step's operands in flight under this step's MFMAs
      f8_load_tile<BM>(A, lda, m0, M, (kt + 1) * F8_BK, K, ra);
      f8_load_tile<F8_BN>(W, ldw, n0, N, (kt + 1) * F8_BK, K, rb);
    }
    i32x8 fa[MI], fb[4];
#pragma unroll
    for (int i = 0; i < MI; ++i) fa[i] = f8_frag(lds_a[cur], wm + i * 16 + (lane & 15), lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = f8_frag(lds_b[cur], wn + j * 16 + (lane & 15), lane);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma_e4m3(fa[i], fb[j], acc[i][j]);
    if (more) {
      f8_store_tile<BM>(lds_a[cur ^ 1], ra);
      f8_store_tile<F8_BN>(lds_b[cur ^ 1], rb);
    }
    __syncthreads();
  }

  f8_epilogue<TO, MI>(acc, m0, n0, wm, wn, lane, a_scale, w_scale, C, ldc, M, N, bias, R, ldr, act);
}

template <typename TO> struct F8Vec;
template <> struct F8Vec<bf16> {
  static __device__ __forceinline__ void ld(const bf16* p, float (&v)[8]) {
    const bf16x8 x = *(const bf16x8*)p;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)x[i];
  }
  static __device__ __forceinline__ void st(bf16* p, const float (&v)[8]) {
    bf16x8 x;
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = (bf16)v[i];
    *(bf16x8*)p = x;
  }
};
template <> struct F8Vec<f16> {
  static __device__ __forceinline__ void ld(const f16* p, float (&v)[8]) {
    const f16x8 x = *(const f16x8*)p;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)x[i];
  }
  static __device__ __forceinline__ void st(f16* p, const float (&v)[8]) {
    f16x8 x;
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = (f16)v[i];
    *(f16x8*)p = x;
  }
};
template <> struct F8Vec<float> {
  static __device__ __forceinline__ void ld(const float* p, float (&v)[8]) {
    const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
    v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w, v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
  }
  static __device__ __forceinline__ void st(float* p, const float (&v)[8]) {
    *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
    *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
};

// One workgroup per row: amax over the row, q = RNE_e4m3(x * 448 / amax), scale = amax / 448.
template <typename T>
__global__ __launch_bounds__(256) void quant_rows_e4m3_kernel(const T* __restrict__ x, long long ldx,
                                                              uint8_t* __restrict__ q, long long ldq,
                                                              float* __restrict__ scale, int K) {
  typedef typename VecT<T>::v8 V8;
  __shared__ float red[4];
  const long long row = blockIdx.x;
  const T* xr = x + row * ldx;
  float amax = 0.f;
  for (int k = threadIdx.x * 8; k < K; k += 256 * 8) {
    const V8 v = *(const V8*)(xr + k);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf((float)v[j]));
  }
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  // correctly rounded divisions (hipcc's default f32 '/' is not), so the scale is exactly amax / 448 in fp32
  const float inv = amax > 0.f ? __fdiv_rn(448.0f, amax) : 0.f;
  if (threadIdx.x == 0) scale[row] = __fdiv_rn(amax, 448.0f);
  uint8_t* qr = q + row * ldq;
  for (int k = threadIdx.x * 8; k < K; k += 256 * 8) {
    const V8 v = *(const V8*)(xr + k);
    int lo = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[0] * inv, (float)v[1] * inv, 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[2] * inv, (float)v[3] * inv, lo, true);
    int hi = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[4] * inv, (float)v[5] * inv, 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[6] * inv, (float)v[7] * inv, hi, true);
    *(i32x2*)(qr + k) = i32x2{lo, hi};
  }
}
// K <= 64 * 8 * MAXV: one wave per row, 4 rows per workgroup, the row held in registers between the amax
// and the conversion (one HBM read instead of two, and no idle lanes on short rows).  Same arithmetic as
// quant_rows_e4m3_kernel, so both give identical bytes.
template <typename T, int MAXV>
__global__ __launch_bounds__(256) void quant_rows_e4m3_wave_kernel(const T* __restrict__ x, long long ldx,
                                                                   uint8_t* __restrict__ q, long long ldq,
                                                                   float* __restrict__ scale, int M, int K) {
  typedef typename VecT<T>::v8 V8;
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int VPR = K / 8;
  const T* xr = x + row * ldx;
  V8 v[MAXV];
  float amax = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j)
    if (lane + j * 64 < VPR) v[j] = *(const V8*)(xr + (lane + j * 64) * 8);
#pragma unroll
  for (int j = 0; j < MAXV; ++j)
    if (lane + j * 64 < VPR)
#pragma unroll
      for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf((float)v[j][i]));
  amax = wave_max(amax);
  const float inv = amax > 0.f ? __fdiv_rn(448.0f, amax) : 0.f;
  if (lane == 0) scale[row] = __fdiv_rn(amax, 448.0f);
  uint8_t* qr = q + row * ldq;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int c = lane + j * 64;
    if (c < VPR) {
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[j][0] * inv, (float)v[j][1] * inv, 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[j][2] * inv, (float)v[j][3] * inv, lo, true);
      int hi = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[j][4] * inv, (float)v[j][5] * inv, 0, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[j][6] * inv, (float)v[j][7] * inv, hi, true);
      *(i32x2*)(qr + c * 8) = i32x2{lo, hi};
    }
  }
}
// MX e4m3 quantization (fd_quant_rows_mx): one thread per 8 consecutive elements of a row, a 32-element block = 4
// consecutive threads (K % 32 == 0), block amax by two xor shuffles, then mx_exp / mx_pack4 (fd_common.h).
template <typename T>
__global__ __launch_bounds__(256) void quant_rows_mx_kernel(const T* __restrict__ x, long long ldx,
                                                            uint8_t* __restrict__ q, long long ldq,
                                                            uint8_t* __restrict__ sb, long long lds, int M, int K) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  const int vpr = K / 8;
  const long long row = t / vpr;
  const int v = (int)(t - row * vpr);
  const bool ok = row < M;  // groups of 4 threads share a row: all in or all out
  float f[8];
  if (ok) {
    F8Vec<T>::ld(x + row * ldx + v * 8, f);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = 0.f;
  }
  float am = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) am = fmaxf(am, fabsf(f[i]));
  am = fmaxf(am, __shfl_xor(am, 1, 64));
  am = fmaxf(am, __shfl_xor(am, 2, 64));
  if (!ok) return;
  const int E = mx_exp(am);
  *(u32x2*)(q + row * ldq + v * 8) = u32x2{mx_pack4(f[0], f[1], f[2], f[3], E), mx_pack4(f[4], f[5], f[6], f[7], E)};
  if ((v & 3) == 0) sb[row * lds + v / 4] = (uint8_t)(E + 127);
}
}  // namespace

extern "C" int fd_quant_rows_mx(const void* x, long long ldx, void* q, long long ldq, void* s, long long lds, int M,
                                int K, int dtype, void* stream) {
  if (!x || !q || !s) return FD_ERR_ARG;
  if (M <= 0 || K <= 0 || (K % 32) || ldx < K || ldq < K || lds < K / 32 || (ldq % 8)) return FD_ERR_SHAPE;
  const int esz = dtype == FD_F32 ? 4 : 2;
  if ((((unsigned long long)x) & 15) || ((ldx * esz) % 16) || (((unsigned long long)q) & 7)) return FD_ERR_ARG;
  const long long threads = (long long)M * (K / 8);
  const dim3 grid((unsigned)((threads + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == FD_BF16)
    hipLaunchKernelGGL(quant_rows_mx_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)x, ldx, (uint8_t*)q, ldq,
                       (uint8_t*)s, lds, M, K);
  else if (dtype == FD_F16)
    hipLaunchKernelGGL(quant_rows_mx_kernel<f16>, grid, dim3(256), 0, st, (const f16*)x, ldx, (uint8_t*)q, ldq,
                       (uint8_t*)s, lds, M, K);
  else if (dtype == FD_F32)
    hipLaunchKernelGGL(quant_rows_mx_kernel<float>, grid, dim3(256), 0, st, (const float*)x, ldx, (uint8_t*)q, ldq,
                       (uint8_t*)s, lds, M, K);
  else
    return FD_ERR_DTYPE;
  FD_LAUNCH_CHECK();
  return FD_OK;
}

extern "C" int fd_quant_rows_e4m3(const void* x, long long ldx, void* q, long long ldq, float* scale, int M, int K,
                                  int dtype, void* stream) {
  if (!x || !q || !scale) return FD_ERR_ARG;
  if (M <= 0 || K <= 0 || (K % 16) || (ldx % 8) || (ldq % 16) || ldx < K || ldq < K) return FD_ERR_SHAPE;
  // 16-B vector loads of x rows and 8-B stores of q rows: an offset view (x[:, 8:]) must be rejected, not faulted
  if ((((unsigned long long)x) | ((unsigned long long)q)) & 15) return FD_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (K <= 2048) {
    FD_DISPATCH_T(dtype, hipLaunchKernelGGL((quant_rows_e4m3_wave_kernel<T, 4>), dim3((M + 3) / 4), dim3(256), 0, s,
                                            (const T*)x, ldx, (uint8_t*)q, ldq, scale, M, K));
  } else {  // long rows (the 5120-wide GEGLU output): a workgroup per row measured faster (6.3 vs 7.0 us at M = 2048)
    FD_DISPATCH_T(dtype, hipLaunchKernelGGL(quant_rows_e4m3_kernel<T>, dim3(M), dim3(256), 0, s, (const T*)x, ldx,
                                            (uint8_t*)q, ldq, scale, K));
  }
  FD_LAUNCH_CHECK();
  return FD_OK;
}

extern "C" int fd_gemm8_e4m3_try(fd_gemm_params* p, const float* a_scale, void* stream);  // gemm8.hip

extern "C" int fd_gemm_e4m3(const void* A, long long lda, const float* a_scale, const void* W, long long ldw,
                            float w_scale, void* C, long long ldc, int M, int N, int K, const float* bias,
                            const void* residual, long long ldr, int act, int out_dtype, void* stream) {
  if (!A || !a_scale || !W || !C) return FD_ERR_ARG;
  if (act < FD_ACT_NONE || act > FD_ACT_GEGLU) return FD_ERR_ARG;
  const int nout = act == FD_ACT_GEGLU ? N / 2 : N;
  if (M <= 0 || N <= 0 || K <= 0 || (K % 16) || (lda % 16) || (ldw % 16) || lda < K || ldw < K || ldc < nout)
    return FD_ERR_SHAPE;
  if (act == FD_ACT_GEGLU && (N % 32)) return FD_ERR_SHAPE;
  // both kernels stage A / W rows with 16-B loads (register or LDS-DMA): base pointers must be 16-B aligned
  if ((((unsigned long long)A) | ((unsigned long long)W)) & 15) return FD_ERR_ARG;
  if (residual && ldr < nout) return FD_ERR_SHAPE;
  if (residual && out_dtype == FD_F32) return FD_ERR_DTYPE;
  // 64-row tiles when 128-row tiles leave CUs idle (fewer than 256 workgroups, e.g. the M = 2048 projections)
  const int tn = (N + F8_BN - 1) / F8_BN, t128 = ((M + 127) / 128) * tn;
  const bool small = t128 < 256;
  const int tiles = small ? ((M + 63) / 64) * tn : t128;
  // K % 128 == 0: the eight-wave kernel family (gemm8.hip, every tile shape); ragged K (K % 128 != 0, e.g. the 128^2
  // level's K = 320 projections) or a shape it declines: the register-staged 4-wave kernel below.  (Round 6: the
  // 4-wave LDS-DMA ring kernel, selectable only by a knob since round 3, was removed.)
  {
    fd_gemm_params p{};
    p.A = A;
    p.B = W;
    p.C = C;
    p.lda = lda;
    p.ldb = ldw;
    p.ldc = ldc;
    p.M = M;
    p.N = N;
    p.K = K;
    p.batch = 1;
    p.bias = bias;
    p.residual = residual;
    p.ldr = ldr;
    p.alpha = w_scale;
    p.act = act;
    p.out_dtype = out_dtype;
    p.m_ref = M;
    const int r8 = fd_gemm8_e4m3_try(&p, a_scale, stream);
    if (r8 < 0) return r8;
    if (r8 == 1) return FD_OK;
  }
  FD_DISPATCH_O(out_dtype, {
    auto kern = small ? gemm_e4m3_kernel<TO, 64> : gemm_e4m3_kernel<TO, 128>;
    hipLaunchKernelGGL(kern, dim3(tiles), dim3(F8_NT), 0, (hipStream_t)stream, (const uint8_t*)A, lda, a_scale,
                       (const uint8_t*)W, ldw, w_scale, (TO*)C, ldc, M, N, K, bias, (const TO*)residual, ldr, act);
  });
  FD_LAUNCH_CHECK();
  return FD_OK;
}
