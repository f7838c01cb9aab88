// Elementwise, layout, direct-conv and denoise-loop kernels (all HBM- or latency-bound).
#include <math.h>

#include <type_traits>

#include "fd_common.h"

static inline dim3 grid1d(long long n, int per_thread = 1) {
  long long blocks = (n + 256LL * per_thread - 1) / (256LL * per_thread);
  if (blocks > 65535LL * 32) blocks = 65535LL * 32;
  return dim3((unsigned)blocks);
}

// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void concat_channels_kernel(const T* __restrict__ a, int C1, const T* __restrict__ b, int C2,
                                       T* __restrict__ y, long long M) {
  typedef typename VecT<T>::v8 V8;
  const int C = C1 + C2, VPR = C / 8;
  const long long total = M * VPR;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const long long m = e / VPR;
    const int v = e - m * VPR;
    const int c = v * 8;
    const V8 val = c < C1 ? *(const V8*)(a + m * C1 + c) : *(const V8*)(b + m * C2 + (c - C1));
    st_out16((V8*)(y + m * C + c), val);
  }
}

extern "C" int fd_concat_channels(const void* a, int C1, const void* b, int C2, void* y, long long M, int dtype,
                                  void* stream) {
  if (!a || !b || !y) return FD_ERR_ARG;
  if (C1 % 8 || C2 % 8 || M <= 0) return FD_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_T(dtype, hipLaunchKernelGGL(concat_channels_kernel<T>, grid1d(M * (C1 + C2) / 8), dim3(256), 0, s,
                                          (const T*)a, C1, (const T*)b, C2, (T*)y, M));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// ------------------------------------------------------------------------------------------------
template <typename TI, typename TO>
__global__ void unary_kernel(const TI* __restrict__ x, TO* __restrict__ y, long long n, int act) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    y[i] = (TO)act_f((float)x[i], act);
}

#define FD_DISPATCH_I(dtype, ...)          \
  if ((dtype) == FD_BF16) {                \
    typedef bf16 TI;                       \
    __VA_ARGS__;                           \
  } else if ((dtype) == FD_F16) {          \
    typedef f16 TI;                        \
    __VA_ARGS__;                           \
  } else if ((dtype) == FD_F32) {          \
    typedef float TI;                      \
    __VA_ARGS__;                           \
  } else {                                 \
    return FD_ERR_DTYPE;                   \
  }

extern "C" int fd_unary(const void* x, void* y, long long n, int act, int dtype, int out_dtype, void* stream) {
  if (!x || !y) return FD_ERR_ARG;
  if (n <= 0) return FD_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_I(dtype, FD_DISPATCH_O(out_dtype, hipLaunchKernelGGL((unary_kernel<TI, TO>), grid1d(n), dim3(256), 0, s,
                                                                   (const TI*)x, (TO*)y, n, act)));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

template <typename TI, typename TO>
__global__ void add_strided_kernel(const TI* __restrict__ x, long long ldx, const TI* __restrict__ a, long long lda,
                                   TO* __restrict__ y, long long ldy, int M, int N) {
  const long long total = (long long)M * N;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const long long m = e / N;
    const int n = e - m * N;
    float v = (float)x[m * ldx + n];
    if (a) v += (float)a[m * lda + n];
    y[m * ldy + n] = (TO)v;
  }
}

extern "C" int fd_add_strided(const void* x, long long ldx, const void* a, long long lda, void* y, long long ldy, int M,
                              int N, int dtype, int out_dtype, void* stream) {
  if (!x || !y) return FD_ERR_ARG;
  if (M <= 0 || N <= 0) return FD_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_I(dtype, FD_DISPATCH_O(out_dtype, hipLaunchKernelGGL((add_strided_kernel<TI, TO>),
                                                                   grid1d((long long)M * N), dim3(256), 0, s,
                                                                   (const TI*)x, ldx, (const TI*)a, lda, (TO*)y, ldy, M,
                                                                   N)));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// y[m][n] = alpha * x[m][n] + beta * z[m][n], general row strides (y may alias z: the RRDB residual
// out * 0.2 + x of the BSRNet pre-pass, bsrnet_arch.py:72-76).  Vectorised when every row is 16-B aligned.
template <typename T>
__global__ void axpby_kernel(const T* __restrict__ x, long long ldx, const T* z, long long ldz, T* y,
                             long long ldy, int M, int N, float alpha, float beta) {
  typedef typename VecT<T>::v8 V8;
  const int nv = N / 8;
  const long long total = (long long)M * nv;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const long long m = e / nv;
    const int c = (int)(e - m * nv) * 8;
    const V8 a = *(const V8*)(x + m * ldx + c);
    const V8 b = *(const V8*)(z + m * ldz + c);
    V8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (T)(alpha * (float)a[i] + beta * (float)b[i]);
    *(V8*)(y + m * ldy + c) = o;
  }
}

extern "C" int fd_axpby(const void* x, long long ldx, const void* z, long long ldz, void* y, long long ldy, int M,
                        int N, float alpha, float beta, int dtype, void* stream) {
  if (!x || !z || !y) return FD_ERR_ARG;
  if (M <= 0 || N <= 0 || N % 8 || (ldx | ldz | ldy) & 7) return FD_ERR_SHAPE;
  if (((unsigned long long)x | (unsigned long long)z | (unsigned long long)y) & 15) return FD_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_T(dtype, hipLaunchKernelGGL((axpby_kernel<T>), grid1d((long long)M * (N / 8)), dim3(256), 0, s,
                                          (const T*)x, ldx, (const T*)z, ldz, (T*)y, ldy, M, N, alpha, beta));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// ------------------------------------------------------------------------------------------------
// layout transposes.  NCHW [n][C][HW] <-> NHWC [n][HW][C]; 32x32 LDS tiles.
template <typename TI, typename TO, bool TO_NHWC>
__global__ void layout_kernel(const TI* __restrict__ x, TO* __restrict__ y, int C, int HW, float scale) {
  __shared__ float tile[32][33];
  const int n = blockIdx.z;
  // tile over (C, HW)
  const int c0 = blockIdx.y * 32, p0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: ty 0..7
  const long long base = (long long)n * C * HW;
  for (int k = ty; k < 32; k += 8) {
    if (TO_NHWC) {  // read NCHW: rows c, cols p
      const int c = c0 + k, p = p0 + tx;
      tile[k][tx] = (c < C && p < HW) ? (float)x[base + (long long)c * HW + p] : 0.f;
    } else {  // read NHWC: rows p, cols c
      const int p = p0 + k, c = c0 + tx;
      tile[k][tx] = (c < C && p < HW) ? (float)x[base + (long long)p * C + c] : 0.f;
    }
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    if (TO_NHWC) {  // write NHWC: rows p, cols c
      const int p = p0 + k, c = c0 + tx;
      if (c < C && p < HW) y[base + (long long)p * C + c] = (TO)(tile[tx][k] * scale);
    } else {
      const int c = c0 + k, p = p0 + tx;
      if (c < C && p < HW) y[base + (long long)c * HW + p] = (TO)(tile[tx][k] * scale);
    }
  }
}

extern "C" int fd_nchw_to_nhwc(const void* x, void* y, int nimg, int C, int HW, float scale, int dtype, int out_dtype,
                               void* stream) {
  if (!x || !y) return FD_ERR_ARG;
  if (nimg <= 0 || C <= 0 || HW <= 0) return FD_ERR_SHAPE;
  dim3 grid((HW + 31) / 32, (C + 31) / 32, nimg);
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_I(dtype, FD_DISPATCH_O(out_dtype, hipLaunchKernelGGL((layout_kernel<TI, TO, true>), grid, dim3(256), 0,
                                                                   s, (const TI*)x, (TO*)y, C, HW, scale)));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

extern "C" int fd_nhwc_to_nchw(const void* x, void* y, int nimg, int C, int HW, float scale, int dtype, int out_dtype,
                               void* stream) {
  if (!x || !y) return FD_ERR_ARG;
  if (nimg <= 0 || C <= 0 || HW <= 0) return FD_ERR_SHAPE;
  dim3 grid((HW + 31) / 32, (C + 31) / 32, nimg);
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_I(dtype, FD_DISPATCH_O(out_dtype, hipLaunchKernelGGL((layout_kernel<TI, TO, false>), grid, dim3(256), 0,
                                                                   s, (const TI*)x, (TO*)y, C, HW, scale)));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

template <typename T>
__global__ void transpose_kernel(const T* __restrict__ x, long long ldx, T* __restrict__ y, long long ldy, int R, int C,
                                 long long sx, long long sy) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const T* xb = x + (long long)b * sx;
  T* yb = y + (long long)b * sy;
  for (int k = ty; k < 32; k += 8) {
    const int r = r0 + k, c = c0 + tx;
    tile[k][tx] = (r < R && c < C) ? (float)xb[(long long)r * ldx + c] : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int c = c0 + k, r = r0 + tx;
    if (r < R && c < C) yb[(long long)c * ldy + r] = (T)tile[tx][k];
  }
}

extern "C" int fd_transpose(const void* x, long long ldx, void* y, long long ldy, int R, int C, int batch, long long sx,
                            long long sy, int dtype, void* stream) {
  if (!x || !y) return FD_ERR_ARG;
  if (R <= 0 || C <= 0 || batch <= 0) return FD_ERR_SHAPE;
  dim3 grid((C + 31) / 32, (R + 31) / 32, batch);
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_T(dtype, hipLaunchKernelGGL(transpose_kernel<T>, grid, dim3(256), 0, s, (const T*)x, ldx, (T*)y, ldy, R,
                                          C, sx, sy));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// ------------------------------------------------------------------------------------------------
// Direct conv for Cin < 64 (K = k*k*Cin <= 72).  Block = 32 consecutive output pixels x all Cout
// (threads stride over Cout); each thread keeps its output channel's K weights in registers and
// reuses them for the 32 pixels (8 pixels per block re-read the whole weight matrix 4x as often: conv_in at
// 128^2 took 84 us); input taps are wave-uniform (broadcast) LDS reads; stores are coalesced.
template <typename TI, typename TO, int KK>
__global__ void __launch_bounds__(256) conv_direct_kernel(const TI* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ bias, TO* __restrict__ y, int nimg,
                                                          int Hin, int Win, int Cin, int Cout, int Hout, int Wout,
                                                          int ks, int stride, int pad, float in_scale) {
  constexpr int P = 32;
  const long long npix = (long long)nimg * Hout * Wout;
  const long long p0 = (long long)blockIdx.x * P;
  // im2col of the block's 8 output pixels (8 x K values) staged once in LDS, read as broadcasts
  __shared__ float patch[P][KK];
  for (int e = threadIdx.x; e < P * KK; e += blockDim.x) {
    const int pi = e / KK, k = e % KK;
    const long long pix = p0 + pi;
    float v = 0.f;
    if (pix < npix) {
      const int ox = pix % Wout;
      const long long t = pix / Wout;
      const int oy = t % Hout;
      const int img = t / Hout;
      const int c = k % Cin, tap = k / Cin;
      const int iy = oy * stride - pad + tap / ks, ix = ox * stride - pad + tap % ks;
      if (iy >= 0 && iy < Hin && ix >= 0 && ix < Win) v = (float)x[(((long long)img * Hin + iy) * Win + ix) * Cin + c];
    }
    patch[pi][k] = v * in_scale;
  }
  __syncthreads();
  constexpr int K = KK;  // exact k*k*Cin (compile-time: the weights live in registers)
  for (int co = threadIdx.x; co < Cout; co += blockDim.x) {
    float wr[K];
#pragma unroll
    for (int k = 0; k < K; ++k) wr[k] = w[(long long)co * K + k];
    const float b = bias ? bias[co] : 0.f;
    for (int pi = 0; pi < P; ++pi) {
      const long long pix = p0 + pi;
      if (pix >= npix) break;
      float acc = b;
#pragma unroll
      for (int k = 0; k < K; ++k) acc += patch[pi][k] * wr[k];
      y[pix * Cout + co] = (TO)acc;
    }
  }
}

extern "C" int fd_conv2d_direct(const void* x, const float* w, const float* bias, void* y, int nimg, int Hin, int Win,
                                int Cin, int Cout, int ksize, int stride, int pad, float in_scale, int dtype,
                                int out_dtype, void* stream) {
  if (!x || !w || !y) return FD_ERR_ARG;
  if (nimg <= 0 || Hin <= 0 || Win <= 0 || Cin <= 0 || Cout <= 0 || ksize <= 0 || stride <= 0) return FD_ERR_SHAPE;
  const int K = ksize * ksize * Cin;
  const int Hout = (Hin + 2 * pad - ksize) / stride + 1, Wout = (Win + 2 * pad - ksize) / stride + 1;
  const long long npix = (long long)nimg * Hout * Wout;
  dim3 grid((unsigned)((npix + 31) / 32)), block(Cout >= 256 ? 256 : ((Cout + 63) / 64) * 64);
  hipStream_t s = (hipStream_t)stream;
#define FD_CONV_DIRECT(KK)                                                                                    \
  FD_DISPATCH_I(dtype, FD_DISPATCH_O(out_dtype, hipLaunchKernelGGL((conv_direct_kernel<TI, TO, KK>), grid, block, 0, \
                                                                   s, (const TI*)x, w, bias, (TO*)y, nimg, Hin, Win,  \
                                                                   Cin, Cout, Hout, Wout, ksize, stride, pad,         \
                                                                   in_scale)))
  switch (K) {  // the FaithDiff convs with Cin < 64: 3x3x4, 3x3x3, 1x1x8, 1x1x4
    case 36: FD_CONV_DIRECT(36); break;
    case 27: FD_CONV_DIRECT(27); break;
    case 8: FD_CONV_DIRECT(8); break;
    case 4: FD_CONV_DIRECT(4); break;
    default: return FD_ERR_SHAPE;
  }
#undef FD_CONV_DIRECT
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// ------------------------------------------------------------------------------------------------
// Narrow 3x3 conv (Cout <= 4, stride 1, pad 1, Cin 32 / 64 / 128): the VAE decoder's conv_out (128 -> 3 at 1024^2),
// which the implicit-GEMM tiles run at 3 of 64 columns while gathering every input element 9 times (285 us,
// profiles/r03_vae_pmc_kernel_stats.csv), with the decoder's conv_norm_out GroupNorm + SiLU optionally folded in
// (gi_affine: the (scale, shift) per (image, channel) of fd_group_norm_affine, applied to every staged element
// exactly as fd_group_norm stores it, zero padding after the transform).
// One workgroup = a strip of TH output rows x 64 pixels.  Input rows pass through a 4-slot LDS ring (66 pixels x Cin,
// pixel pitch Cin + 8 elements: lane-consecutive pixels on consecutive 16-B bank groups, conflict-free
// ds_read_b128): each input row is loaded, transformed and staged once per strip (TH + 2 rows for TH outputs), and
// row r + 2's global loads are in flight while row r is computed.  Wave w sums channels [w Cin/4, (w+1) Cin/4) of the
// 9 taps for the 64 pixels (lane = pixel) against wave-uniform fp32 weights (scalar loads); the 4 partial sums are
// added in wave order.  fp32 accumulation; a different summation order than the GEMM path.  (The round-3 form staged
// 3 rows per output row in 64-pixel workgroups: every input row loaded 3 times, no overlap, ~0.3 ms at 1024^2.)
template <typename T>
__device__ __forceinline__ float dot2_acc(unsigned a, unsigned b, float c) {
  if constexpr (std::is_same<T, f16>::value) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(h2, a), __builtin_bit_cast(h2, b), c, false);
  } else {
    typedef __bf16 b2 __attribute__((ext_vector_type(2)));
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(b2, a), __builtin_bit_cast(b2, b), c, false);
  }
}

template <typename T, typename TO, int CIN, int NOUT, int TH>
__global__ void __launch_bounds__(256, 2) conv3x3_narrow_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                                const float* __restrict__ bias,
                                                                const float* __restrict__ aff, int silu,
                                                                TO* __restrict__ y, int nimg, int H, int W) {
  typedef typename VecT<T>::v8 V8;
  typedef __attribute__((ext_vector_type(4))) unsigned U4;
  constexpr int PP = CIN + 8, VPP = CIN / 8, CPW = CIN / 4;  // pixel pitch (elements), vectors per pixel, ch per wave
  constexpr int RW = 66, ROW = RW * PP, NV = RW * VPP, VPT = (NV + 255) / 256;
  // weights as 16-bit pairs, [tap][8-channel vector][out][4 pairs]: one broadcast ds_read_b128 per (vector, out)
  constexpr int WV = 9 * VPP * NOUT;  // 16-B weight vectors
  __shared__ __attribute__((aligned(16))) T ring[3 * ROW];
  __shared__ __attribute__((aligned(16))) U4 wsh[WV];
  __shared__ float red[256 * 4];
  __shared__ __attribute__((aligned(16))) float aff_s[CIN * 2];
  const int tid = threadIdx.x;
  const int tpr = (W + 63) / 64, tpc = (H + TH - 1) / TH;
  int bid = blockIdx.x;
  const int tx = bid % tpr;
  bid /= tpr;
  const int ty = bid % tpc;
  const long long img = bid / tpc;
  const int x0 = tx * 64, y0 = ty * TH, y1 = min(y0 + TH, H);
  if (aff && tid < CIN * 2 / 4) *(f32x4*)(aff_s + tid * 4) = *(const f32x4*)(aff + img * CIN * 2 + tid * 4);
  for (int e = tid; e < WV; e += 256) {  // e = (tap * VPP + v) * NOUT + n
    const int n = e % NOUT, tv = e / NOUT, v = tv % VPP, tap = tv / VPP;
    const float* src = w + (long long)n * 9 * CIN + tap * CIN + v * 8;
    V8 h;
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = (T)src[i];
    wsh[e] = __builtin_bit_cast(U4, h);
  }
  // two register sets of staged-row loads: row oy + 3's global loads go out while row oy + 2's (issued one row
  // earlier, so they had a row of compute to land) are transformed into the ring
  V8 ldA[VPT], ldB[VPT];
  unsigned okA = 0, okB = 0;  // bit k: vector k of this thread lies inside the image
  auto load_row = [&] __attribute__((always_inline)) (int iy, V8 (&ld)[VPT], unsigned& okm) {
    okm = 0;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int e = tid + k * 256;
      const int v = e % VPP, col = e / VPP, ix = x0 - 1 + col;
      if (e < NV && iy >= 0 && iy < H && ix >= 0 && ix < W) {
        ld[k] = *(const V8*)(x + ((img * H + iy) * W + ix) * CIN + v * 8);
        okm |= 1u << k;
      }
    }
  };
  auto store_row = [&] __attribute__((always_inline)) (int slot, const V8 (&ld)[VPT], unsigned okm) {
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int e = tid + k * 256;
      if (e < NV) {
        const int v = e % VPP, col = e / VPP;
        const bool ok = (okm >> k) & 1;
        typedef __attribute__((ext_vector_type(4))) unsigned U4;
        U4 bits = ok ? __builtin_bit_cast(U4, ld[k]) : (U4){0u, 0u, 0u, 0u};  // zero padding: raw bits, no fp round trip
        if (aff) {
          V8 val;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            float f = __builtin_fmaf((float)ld[k][i], aff_s[(v * 8 + i) * 2], aff_s[(v * 8 + i) * 2 + 1]);
            if (silu) f = silu_f(f);
            val[i] = (T)f;
          }
          bits = ok ? __builtin_bit_cast(U4, val) : (U4){0u, 0u, 0u, 0u};
        }
        *(U4*)(ring + slot * ROW + col * PP + v * 8) = bits;
      }
    }
  };
  __syncthreads();  // aff_s, wsh
  for (int r = 0; r < 3; ++r) {
    load_row(y0 - 1 + r, ldA, okA);
    store_row(r, ldA, okA);
  }
  if (y0 + 1 < y1) load_row(y0 + 2, ldA, okA);  // input row of output row y0 + 1
  __syncthreads();
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const U4* wq = wsh + wv * (CPW / 8) * NOUT;  // this wave's channel vectors start at v = wv * CPW / 8
  auto row = [&] __attribute__((always_inline)) (int oy, V8 (&cur)[VPT], unsigned& okc, V8 (&nxt)[VPT],
                                                   unsigned& okn) {
    const int r = oy - y0;
    const bool more = oy + 1 < y1;  // output row oy + 1 needs input row oy + 2 (in cur since one row ago)
    if (oy + 2 < y1) load_row(oy + 3, nxt, okn);
    float acc[NOUT];
#pragma unroll
    for (int n = 0; n < NOUT; ++n) acc[n] = 0.f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int sl = r + ky >= 3 ? (r + ky) % 3 : r + ky;
      const T* rp = ring + sl * ROW + lane * PP + wv * CPW;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
#pragma unroll
        for (int cv = 0; cv < CPW / 8; ++cv) {
          const U4 xv = __builtin_bit_cast(U4, *(const V8*)(rp + kx * PP + cv * 8));
#pragma unroll
          for (int n = 0; n < NOUT; ++n) {
            const U4 wn = wq[((ky * 3 + kx) * VPP + cv) * NOUT + n];
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[n] = dot2_acc<T>(xv[j], wn[j], acc[n]);
          }
        }
      }
    }
#pragma unroll
    for (int n = 0; n < NOUT; ++n) red[(wv * 64 + lane) * 4 + n] = acc[n];
    __syncthreads();  // red[] written; every wave done reading the slot of input row oy - 1
    if (more) store_row(r % 3, cur, okc);  // input row oy + 2 = (y0 - 1) + r + 3: the slot of row oy - 1
    if (wv == 0 && x0 + lane < W) {
      TO* yp = y + ((img * H + oy) * W + x0 + lane) * NOUT;
#pragma unroll
      for (int n = 0; n < NOUT; ++n) {
        const float sum = ((red[lane * 4 + n] + red[(64 + lane) * 4 + n]) + red[(128 + lane) * 4 + n]) +
                          red[(192 + lane) * 4 + n];
        yp[n] = (TO)(sum + (bias ? bias[n] : 0.f));
      }
    }
    __syncthreads();  // red[] read; the new slot visible
  };
  for (int oy = y0; oy < y1; oy += 2) {
    row(oy, ldA, okA, ldB, okB);
    if (oy + 1 < y1) row(oy + 1, ldB, okB, ldA, okA);
  }
}

static int conv3x3_narrow(const void* x, const float* w, const float* bias, const float* aff, int silu, void* y,
                          int nimg, int H, int W, int Cin, int Cout, int dtype, int out_dtype, void* stream) {
  if (!x || !w || !y) return FD_ERR_ARG;
  if (nimg <= 0 || H <= 0 || W <= 0) return FD_ERR_SHAPE;
  if (((unsigned long long)x) & 15) return FD_ERR_ARG;  // 16-B vector loads of the input rows
  if (aff && (((unsigned long long)aff) & 15)) return FD_ERR_ARG;
  constexpr int TH = 16;
  const long long nblk = (long long)nimg * ((H + TH - 1) / TH) * ((W + 63) / 64);
  if (nblk > 0x7fffffff) return FD_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  dim3 g((unsigned)nblk), b(256);
  // instances: Cin 32 / 64 / 128 (the decoder's conv_out is 128 -> 3), Cout 1..4
#define FD_NARROW(CI, NO)                                                                                         \
  FD_DISPATCH_T(dtype, FD_DISPATCH_O(out_dtype, hipLaunchKernelGGL((conv3x3_narrow_kernel<T, TO, CI, NO, TH>), g, b, \
                                                                   0, s, (const T*)x, w, bias, aff, silu, (TO*)y,    \
                                                                   nimg, H, W)))
#define FD_NARROW_N(CI)                  \
  switch (Cout) {                        \
    case 1: FD_NARROW(CI, 1); break;     \
    case 2: FD_NARROW(CI, 2); break;     \
    case 3: FD_NARROW(CI, 3); break;     \
    case 4: FD_NARROW(CI, 4); break;     \
    default: return FD_ERR_SHAPE;        \
  }
  if (Cin == 128) {
    FD_NARROW_N(128)
  } else if (Cin == 64) {
    FD_NARROW_N(64)
  } else if (Cin == 32) {
    FD_NARROW_N(32)
  } else {
    return FD_ERR_SHAPE;
  }
#undef FD_NARROW_N
#undef FD_NARROW
  FD_LAUNCH_CHECK();
  return FD_OK;
}

extern "C" int fd_conv3x3_narrow(const void* x, const float* w, const float* bias, void* y, int nimg, int H, int W,
                                 int Cin, int Cout, int dtype, int out_dtype, void* stream) {
  return conv3x3_narrow(x, w, bias, nullptr, 0, y, nimg, H, W, Cin, Cout, dtype, out_dtype, stream);
}

extern "C" int fd_conv3x3_narrow_gn(const void* x, const float* w, const float* bias, const float* gi_affine,
                                    int gi_silu, void* y, int nimg, int H, int W, int Cin, int Cout, int dtype,
                                    int out_dtype, void* stream) {
  if (!gi_affine) return FD_ERR_ARG;
  return conv3x3_narrow(x, w, bias, gi_affine, gi_silu, y, nimg, H, W, Cin, Cout, dtype, out_dtype, stream);
}

// ------------------------------------------------------------------------------------------------
// SDXL time features (diffusers get_timestep_embedding: half = dim/2, exponent = -ln(1e4) * i / half,
// emb = [cos, sin] after flip_sin_to_cos).
__device__ __forceinline__ float sinus_feat(float t, int i, int dim) {
  const int half = dim / 2;
  const int k = i < half ? i : i - half;  // flipped: first half cos, second half sin
  const float freq = expf(-9.210340371976184f * (float)k / (float)half);
  const float a = t * freq;
  return i < half ? cosf(a) : sinf(a);
}

template <typename TO>
__global__ void time_features_kernel(const float* __restrict__ t, const float* __restrict__ tids,
                                     const float* __restrict__ text, TO* __restrict__ tfeat, TO* __restrict__ afeat,
                                     int batch) {
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < 320; i += blockDim.x) tfeat[b * 320 + i] = (TO)sinus_feat(t[b], i, 320);
  for (int i = threadIdx.x; i < 2816; i += blockDim.x) {
    float v;
    if (i < 1280) {
      v = text[b * 1280 + i];
    } else {
      const int j = i - 1280, which = j / 256, k = j % 256;
      v = sinus_feat(tids[b * 6 + which], k, 256);
    }
    afeat[b * 2816 + i] = (TO)v;
  }
}

extern "C" int fd_time_features(const float* t, const float* time_ids, const float* text_embeds, void* tfeat,
                                void* afeat, int batch, int dtype, void* stream) {
  if (!t || !time_ids || !text_embeds || !tfeat || !afeat) return FD_ERR_ARG;
  if (batch <= 0) return FD_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_O(dtype, hipLaunchKernelGGL(time_features_kernel<TO>, dim3(batch), dim3(256), 0, s, t, time_ids,
                                          text_embeds, (TO*)tfeat, (TO*)afeat, batch));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// ------------------------------------------------------------------------------------------------
// TLC denoise-loop fusions.  Tile t (global index tid = tile_begin + t) has origin
// (row_org[tid / nc], col_org[tid % nc]) on the latent canvas (LocalAttention.grids order).
template <typename TO>
__global__ void tlc_scale_input_kernel(const float* __restrict__ canvas, const int* __restrict__ row_org,
                                       const int* __restrict__ col_org, int nc, int H, int W, int kh, int kw,
                                       int tile_begin, int ntiles, int cfg, float s, TO* __restrict__ out,
                                       float* __restrict__ t_out, int t_n, float t_val) {
  if (t_out) {  // the step's UNet timesteps (grid-stride: any number of UNet rows)
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < t_n; i += gridDim.x * blockDim.x) t_out[i] = t_val;
  }
  const long long per = (long long)kh * kw;
  const long long total = (long long)ntiles * per;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int t = e / per;
    const int p = e - (long long)t * per;
    const int y = p / kw, x = p - y * kw;
    const int tid = tile_begin + t;
    const int oy = row_org[tid / nc] + y, ox = col_org[tid % nc] + x;
    float v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = __fdiv_rn(canvas[((long long)c * H + oy) * W + ox], s);
    for (int d = 0; d < cfg; ++d) {
      TO* o = out + (((long long)(t * cfg + d)) * per + p) * 4;
#pragma unroll
      for (int c = 0; c < 4; ++c) o[c] = (TO)v[c];
    }
  }
}

extern "C" int fd_tlc_scale_input_t(const float* canvas, const int* row_org, int nr, const int* col_org, int nc,
                                    int H, int W, int kh, int kw, int tile_begin, int ntiles, int cfg, float sigma,
                                    void* out, int dtype, float* t_out, int t_n, float timestep, void* stream) {
  if (!canvas || !row_org || !col_org || !out) return FD_ERR_ARG;
  if (t_n < 0 || (t_n > 0 && !t_out)) return FD_ERR_SHAPE;
  if (ntiles <= 0 || tile_begin < 0 || tile_begin + ntiles > nr * nc || kh > H || kw > W || cfg <= 0)
    return FD_ERR_SHAPE;
  // scale_model_input divides by (sigma^2 + 1)^0.5 (diffusers EulerDiscreteScheduler; pipeline:1336): `sigma`
  // here is that divisor, computed by the caller the way torch does in fp32; correctly rounded division per element
  if (!(sigma > 0.f)) return FD_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  FD_DISPATCH_O(dtype, hipLaunchKernelGGL(tlc_scale_input_kernel<TO>, grid1d((long long)ntiles * kh * kw), dim3(256), 0,
                                          st, canvas, row_org, col_org, nc, H, W, kh, kw, tile_begin, ntiles, cfg, sigma,
                                          (TO*)out, t_n > 0 ? t_out : nullptr, t_n, timestep));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

extern "C" int fd_tlc_scale_input(const float* canvas, const int* row_org, int nr, const int* col_org, int nc, int H,
                                  int W, int kh, int kw, int tile_begin, int ntiles, int cfg, float sigma, void* out,
                                  int dtype, void* stream) {
  return fd_tlc_scale_input_t(canvas, row_org, nr, col_org, nc, H, W, kh, kw, tile_begin, ntiles, cfg, sigma, out,
                              dtype, nullptr, 0, 0.f, stream);
}

// CFG combine + Euler step for each tile; x taken from the canvas at the tile origin.
template <typename TI>
__global__ void tlc_cfg_euler_kernel(const TI* __restrict__ eps, const float* __restrict__ canvas,
                                     const int* __restrict__ row_org, const int* __restrict__ col_org, int nc, int H,
                                     int W, int kh, int kw, int tile_begin, int ntiles, int cfg, float g, float sigma,
                                     float sigma_next, float* __restrict__ out) {
  const long long per = (long long)kh * kw;
  const long long total = (long long)ntiles * per;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int t = e / per;
    const int p = e - (long long)t * per;
    const int y = p / kw, x = p - y * kw;
    const int tid = tile_begin + t;
    const int oy = row_org[tid / nc] + y, ox = col_org[tid % nc] + x;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float ev;
      if (cfg == 2) {
        const float u = (float)eps[(((long long)(t * 2)) * per + p) * 4 + c];
        const float cc = (float)eps[(((long long)(t * 2 + 1)) * per + p) * 4 + c];
        ev = u + g * (cc - u);
      } else {
        ev = (float)eps[((long long)t * per + p) * 4 + c];
      }
      const float xv = canvas[((long long)c * H + oy) * W + ox];
      // EulerDiscreteScheduler.step, gamma = 0: pred = x - sigma*eps; d = (x - pred)/sigma; x + d*dt
      const float pred = xv - sigma * ev;
      const float d = (xv - pred) / sigma;
      out[((long long)t * 4 + c) * per + p] = xv + d * (sigma_next - sigma);
    }
  }
}

// guidance_rescale > 0: one block per tile (needs the tile-wide std of the CFG and text predictions)
template <typename TI>
__global__ void __launch_bounds__(256) tlc_cfg_rescale_euler_kernel(
    const TI* __restrict__ eps, const float* __restrict__ canvas, const int* __restrict__ row_org,
    const int* __restrict__ col_org, int nc, int H, int W, int kh, int kw, int tile_begin, float g, float rescale,
    float sigma, float sigma_next, float* __restrict__ out) {
  __shared__ double red[4][4];
  const int t = blockIdx.x;
  const long long per = (long long)kh * kw;
  const long long n = per * 4;
  double s_cfg = 0, q_cfg = 0, s_txt = 0, q_txt = 0;
  for (long long e = threadIdx.x; e < n; e += 256) {
    const float u = (float)eps[(long long)(t * 2) * n + e];
    const float c = (float)eps[(long long)(t * 2 + 1) * n + e];
    const float v = u + g * (c - u);
    s_cfg += v; q_cfg += (double)v * v; s_txt += c; q_txt += (double)c * c;
  }
  // block reduce (doubles)
  for (int o = 32; o > 0; o >>= 1) {
    s_cfg += __shfl_xor(s_cfg, o, 64); q_cfg += __shfl_xor(q_cfg, o, 64);
    s_txt += __shfl_xor(s_txt, o, 64); q_txt += __shfl_xor(q_txt, o, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[w][0] = s_cfg; red[w][1] = q_cfg; red[w][2] = s_txt; red[w][3] = q_txt; }
  __syncthreads();
  double S[4];
  for (int k = 0; k < 4; ++k) S[k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
  // torch.std: unbiased
  const double var_cfg = (S[1] - S[0] * S[0] / n) / (n - 1), var_txt = (S[3] - S[2] * S[2] / n) / (n - 1);
  const float ratio = (float)(sqrt(var_txt) / sqrt(var_cfg));
  const int tid = tile_begin + t;
  const int r0 = row_org[tid / nc], c0 = col_org[tid % nc];
  for (long long e = threadIdx.x; e < n; e += 256) {
    // eps layout NHWC [p][c]; out layout NCHW [c][p]
    const int c = e & 3;
    const long long p = e >> 2;
    const float u = (float)eps[(long long)(t * 2) * n + e];
    const float cc = (float)eps[(long long)(t * 2 + 1) * n + e];
    const float v = u + g * (cc - u);
    const float ev = rescale * (v * ratio) + (1.f - rescale) * v;
    const int y = p / kw, x = p - (long long)y * kw;
    const float xv = canvas[((long long)c * H + r0 + y) * W + c0 + x];
    const float pred = xv - sigma * ev;
    const float d = (xv - pred) / sigma;
    out[((long long)t * 4 + c) * per + p] = xv + d * (sigma_next - sigma);
  }
}

extern "C" int fd_tlc_cfg_euler_step(const void* eps, const float* canvas, const int* row_org, int nr,
                                     const int* col_org, int nc, int H, int W, int kh, int kw, int tile_begin,
                                     int ntiles, int cfg, float guidance, float guidance_rescale, float sigma,
                                     float sigma_next, float* out_tiles, int dtype, void* stream) {
  if (!eps || !canvas || !row_org || !col_org || !out_tiles) return FD_ERR_ARG;
  if (ntiles <= 0 || tile_begin < 0 || tile_begin + ntiles > nr * nc || (cfg != 1 && cfg != 2)) return FD_ERR_SHAPE;
  if (sigma == 0.f) return FD_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (guidance_rescale > 0.f && cfg == 2) {
    FD_DISPATCH_T(dtype, hipLaunchKernelGGL(tlc_cfg_rescale_euler_kernel<T>, dim3(ntiles), dim3(256), 0, s,
                                            (const T*)eps, canvas, row_org, col_org, nc, H, W, kh, kw, tile_begin,
                                            guidance, guidance_rescale, sigma, sigma_next, out_tiles));
  } else {
    FD_DISPATCH_T(dtype, hipLaunchKernelGGL(tlc_cfg_euler_kernel<T>, grid1d((long long)ntiles * kh * kw), dim3(256), 0,
                                            s, (const T*)eps, canvas, row_org, col_org, nc, H, W, kh, kw, tile_begin,
                                            ntiles, cfg, guidance, sigma, sigma_next, out_tiles));
  }
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// grids_inverse: per canvas element, accumulate the covering tiles in tile order (row-major over the
// origin grid), fp64 product rounded to fp32 per add -- the reference's  preds(fp32) += tile * w(fp64).
__global__ void tlc_blend_kernel(const float* __restrict__ tiles, const double* __restrict__ wts,
                                 const int* __restrict__ row_org, int nr, const int* __restrict__ col_org, int nc, int C,
                                 int H, int W, int kh, int kw, float* __restrict__ canvas) {
  const long long total = (long long)C * H * W;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int x = e % W;
    const int y = (e / W) % H;
    const int c = e / ((long long)W * H);
    float pred = 0.f, cnt = 0.f;
    for (int r = 0; r < nr; ++r) {
      const int dy = y - row_org[r];
      if (dy < 0 || dy >= kh) continue;
      for (int q = 0; q < nc; ++q) {
        const int dx = x - col_org[q];
        if (dx < 0 || dx >= kw) continue;
        const int t = r * nc + q;
        const double w = wts[dy * kw + dx];
        const float v = tiles[(((long long)t * C + c) * kh + dy) * kw + dx];
        pred = (float)((double)pred + (double)v * w);
        cnt = (float)((double)cnt + w);
      }
    }
    canvas[e] = pred / cnt;
  }
}

extern "C" int fd_tlc_blend(const float* tiles, const double* weights, const int* row_org, int nr, const int* col_org,
                            int nc, int C, int H, int W, int kh, int kw, float* canvas, void* stream) {
  if (!tiles || !weights || !row_org || !col_org || !canvas) return FD_ERR_ARG;
  if (nr <= 0 || nc <= 0 || C <= 0 || kh > H || kw > W) return FD_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(tlc_blend_kernel, grid1d((long long)C * H * W), dim3(256), 0, s, tiles, weights, row_org, nr,
                     col_org, nc, C, H, W, kh, kw, canvas);
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// grids on an NHWC canvas (image latents, 512 ch): tiles [n*cfg][kh][kw][C]
template <typename T>
__global__ void tlc_grids_nhwc_kernel(const T* __restrict__ canvas, const int* __restrict__ row_org,
                                      const int* __restrict__ col_org, int nc, int H, int W, int C, int kh, int kw,
                                      int tile_begin, int ntiles, int cfg, T* __restrict__ out) {
  typedef typename VecT<T>::v8 V8;
  const int VPR = C / 8;
  const long long per = (long long)kh * kw * VPR;
  const long long total = (long long)ntiles * per;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int t = e / per;
    const long long r = e - (long long)t * per;
    const int v = r % VPR;
    const long long p = r / VPR;
    const int y = p / kw, x = p - (long long)y * kw;
    const int tid = tile_begin + t;
    const int oy = row_org[tid / nc] + y, ox = col_org[tid % nc] + x;
    const V8 val = *(const V8*)(canvas + ((long long)oy * W + ox) * C + v * 8);
    for (int d = 0; d < cfg; ++d) *(V8*)(out + (((long long)(t * cfg + d)) * kh * kw + p) * C + v * 8) = val;
  }
}

extern "C" int fd_tlc_grids_nhwc(const void* canvas, const int* row_org, int nr, const int* col_org, int nc, int H,
                                 int W, int C, int kh, int kw, int tile_begin, int ntiles, int cfg, void* out, int dtype,
                                 void* stream) {
  if (!canvas || !row_org || !col_org || !out) return FD_ERR_ARG;
  if (C % 8 || ntiles <= 0 || tile_begin + ntiles > nr * nc || kh > H || kw > W || cfg <= 0) return FD_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_T(dtype, hipLaunchKernelGGL(tlc_grids_nhwc_kernel<T>, grid1d((long long)ntiles * kh * kw * C / 8),
                                          dim3(256), 0, s, (const T*)canvas, row_org, col_org, nc, H, W, C, kh, kw,
                                          tile_begin, ntiles, cfg, (T*)out));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// DiagonalGaussianDistribution.sample + scaling + DDPM add_noise at t=999 (pipeline:1271-1276), fused:
// moments NHWC [HW][8] (mean 0..3, logvar 4..7) -> canvas fp32 NCHW [4][HW]
//   z = (mean + exp(0.5*clamp(logvar,-30,20)) * post_eps) * scaling;  lat = a*z + b*(noise*init_sigma)
template <typename TI>
__global__ void vae_sample_add_noise_kernel(const TI* __restrict__ moments, const float* __restrict__ post_eps,
                                            const float* __restrict__ noise, float* __restrict__ out, int HW,
                                            float scaling, float init_sigma, float a, float b, int start_lr) {
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < 4LL * HW; e += (long long)gridDim.x * blockDim.x) {
    const int c = e / HW;
    const long long p = e - (long long)c * HW;
    const float nz = noise[e] * init_sigma;
    if (!start_lr) {
      out[e] = nz;
      continue;
    }
    const float mean = (float)moments[p * 8 + c];
    float lv = (float)moments[p * 8 + 4 + c];
    lv = fminf(fmaxf(lv, -30.f), 20.f);
    const float z = (mean + expf(0.5f * lv) * post_eps[e]) * scaling;
    out[e] = a * z + b * nz;
  }
}

extern "C" int fd_vae_sample_add_noise(const void* moments, const float* post_eps, const float* noise, float* out,
                                       int HW, float scaling, float init_sigma, float a, float b, int start_lr,
                                       int dtype, void* stream) {
  if (!noise || !out || (start_lr && (!moments || !post_eps))) return FD_ERR_ARG;
  if (HW <= 0) return FD_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_I(dtype, hipLaunchKernelGGL(vae_sample_add_noise_kernel<TI>, grid1d(4LL * HW), dim3(256), 0, s,
                                          (const TI*)moments, post_eps, noise, out, HW, scaling, init_sigma, a, b,
                                          start_lr));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// VaeImageProcessor.postprocess in float: NHWC [HW][3] -> uint8 HWC  ((x/2+0.5).clamp(0,1)*255).round()
template <typename TI>
__global__ void postprocess_kernel(const TI* __restrict__ x, unsigned char* __restrict__ y, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float v = (float)x[i] / 2.f + 0.5f;
    v = fminf(fmaxf(v, 0.f), 1.f);
    y[i] = (unsigned char)rintf(v * 255.f);
  }
}

extern "C" int fd_postprocess_u8(const void* x, void* y, long long n, int dtype, void* stream) {
  if (!x || !y) return FD_ERR_ARG;
  if (n <= 0) return FD_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_I(dtype, hipLaunchKernelGGL(postprocess_kernel<TI>, grid1d(n), dim3(256), 0, s, (const TI*)x,
                                          (unsigned char*)y, n));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// ------------------------------------------------------------------------------------------------
// Tiled VAE / encoder seam blending (diffusers AutoencoderKL.blend_v / blend_h, FaithDiff
// Encoder.blend_v / blend_h ext:150-162), in place on tile b (NHWC [Hb][Wb][C]):
//   vertical:   b[y][x] = a[Ha - e + y][x] * (1 - y/e) + b[y][x] * (y/e)   for y < e
//   horizontal: b[y][x] = a[y][Wa - e + x] * (1 - x/e) + b[y][x] * (x/e)   for x < e
// e = min(extent, Ha|Wa, Hb|Wb) as in the reference.  Tiles are blended in the reference's order
// (row by row, vertical then horizontal), each call reading the already-blended neighbour.
template <typename T>
__global__ void blend_edge_kernel(const T* __restrict__ a, T* __restrict__ b, int Ha, int Wa, int Hb, int Wb, int C,
                                  int e, int vertical) {
  const long long total = vertical ? (long long)e * Wb * C : (long long)Hb * e * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = i % C;
    const long long r = i / C;
    int y, x;
    float w;
    long long ai;
    if (vertical) {
      x = r % Wb;
      y = r / Wb;
      w = (float)y / (float)e;
      ai = ((long long)(Ha - e + y) * Wa + x) * C + c;
    } else {
      x = r % e;
      y = r / e;
      w = (float)x / (float)e;
      ai = ((long long)y * Wa + (Wa - e + x)) * C + c;
    }
    const long long bi = ((long long)y * Wb + x) * C + c;
    b[bi] = (T)((float)a[ai] * (1.f - w) + (float)b[bi] * w);
  }
}

extern "C" int fd_blend_edge(const void* a, void* b, int Ha, int Wa, int Hb, int Wb, int C, int extent, int vertical,
                             int dtype, void* stream) {
  if (!a || !b) return FD_ERR_ARG;
  if (C <= 0 || Ha <= 0 || Wa <= 0 || Hb <= 0 || Wb <= 0) return FD_ERR_SHAPE;
  int e = extent;
  if (vertical) {
    e = min(e, min(Ha, Hb));
    if (Wa != Wb) return FD_ERR_SHAPE;
  } else {
    e = min(e, min(Wa, Wb));
    if (Ha != Hb) return FD_ERR_SHAPE;
  }
  if (e <= 0) return FD_OK;
  const long long total = vertical ? (long long)e * Wb * C : (long long)Hb * e * C;
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_I(dtype, hipLaunchKernelGGL(blend_edge_kernel<TI>, grid1d(total), dim3(256), 0, s, (const TI*)a, (TI*)b,
                                          Ha, Wa, Hb, Wb, C, e, vertical));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// ------------------------------------------------------------------------------------------------
extern "C" int fd_device_check(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return FD_ERR_HIP;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return FD_ERR_HIP;
  const char* a = prop.gcnArchName;
  if (!(a[0] == 'g' && a[1] == 'f' && a[2] == 'x' && a[3] == '9' && a[4] == '5' && a[5] == '0')) return FD_ERR_ARCH;
  return FD_OK;
}

extern "C" const char* fd_version(void) { return "libfaithdiff_hip 0.1 gfx950"; }

// ------------------------------------------------------------------------------------------------
// CLIP text embeddings (transformers CLIPTextEmbeddings, called from encode_prompt, pipeline:587-598):
// out[b*L + l][:] = tok[ids[b*L + l]][:] + pos[l][:]   (tables in the compute dtype, sum in fp32).
// One thread per 8 channels (16-B loads / store).
template <typename T>
__global__ void embed_tokens_kernel(const int* __restrict__ ids, const T* __restrict__ tok, const T* __restrict__ pos,
                                    T* __restrict__ out, int rows, int L, int D, int vocab) {
  typedef typename VecT<T>::v8 V8;
  const int per = D / 8;
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)rows * per) return;
  const int r = e / per, c = (e - (long long)r * per) * 8;
  int id = ids[r];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  const V8 a = *(const V8*)(tok + (long long)id * D + c);
  const V8 p = *(const V8*)(pos + (long long)(r % L) * D + c);
  V8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (T)((float)a[i] + (float)p[i]);
  *(V8*)(out + (long long)r * D + c) = o;
}

extern "C" int fd_embed_tokens(const int* ids, const void* tok, const void* pos, void* out, int batch, int L, int D,
                               int vocab, int dtype, void* stream) {
  if (!ids || !tok || !pos || !out) return FD_ERR_ARG;
  if (batch <= 0 || L <= 0 || D <= 0 || (D % 8) || vocab <= 0) return FD_ERR_SHAPE;
  const long long total = (long long)batch * L * (D / 8);
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_T(dtype, hipLaunchKernelGGL(embed_tokens_kernel<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                                          s, ids, (const T*)tok, (const T*)pos, (T*)out, batch * L, L, D, vocab));
  FD_LAUNCH_CHECK();
  return FD_OK;
}
