// GroupNorm (+ fused SiLU) and LayerNorm for NHWC activations, fp32 statistics.  HBM-bound.
//
// GroupNorm runs as three launches so that a (batch, group) reduction of up to 16384 x 80 elements is
// spread over the whole chip: (1) gn_partial: one block per (image, row-chunk) reads its rows once,
// coalesced (16-B vectors along C), and writes per-group (sum, sumsq) partials; (2) gn_finalize: one
// wave per (image, group) folds them in fp64 (E[x^2]-E[x]^2 in double) into (mean, rstd); (3) gn_apply: every
// block builds per-channel scale/shift in LDS and streams its rows: y = x*scale[c] + shift[c] (+ SiLU).
#include <stdlib.h>

#include "fd_common.h"

#define GN_MAXC 2560

static inline int gn_rows_per_chunk(int nimg, int HW) {
  // chunk count chosen from HW alone: the per-(image, group) reduction order -- and so
  // every bit of the result -- does not depend on how many images share the launch (tile batching, CFG
  // rows, tile-parallel sharding all give identical outputs).  512+ blocks at the UNet's B >= 2.
  // Large images (the VAE at 512^2 / 1024^2: HW up to 1M rows) get up to 1024 chunks of >= 64 rows: 256 chunks
  // of 4096 rows left one 4-wave block per CU, latency-bound at ~4 TB/s.
  (void)nimg;
  const int lo = fd_knob(FDK_GN_MIN_CHUNKS);  // chunk floor for small images
  const int target = HW / 64 > 1024 ? 1024 : (HW / 64 < lo ? lo : HW / 64);
  int r = 1;
  while ((HW + r - 1) / r > target) r *= 2;
  return r;
}

// CAT (fd_concat_channels_gn, round 6): x is the channel concat of a [.., C1] and b [.., C - C1], gathered per 8-channel
// vector (C1 % 8 == 0) and also stored to y -- the up-block concat and its GroupNorm statistics pass in one launch,
// the same values in the same order as the concat then this pass (bit-identical partials).
template <typename T, int NV, bool CAT = false>
__global__ void __launch_bounds__(256) gn_partial_kernel(const T* __restrict__ x, float2* __restrict__ part, int HW,
                                                         int C, int groups, int rows_per_chunk,
                                                         const T* __restrict__ b = nullptr, int C1 = 0,
                                                         T* __restrict__ y = nullptr) {
  typedef typename VecT<T>::v8 V8;
  // per-(row-slot, channel) partials, reduced in a fixed order (bitwise reproducible; no atomics)
  __shared__ float lds_s[256 * 8 * NV], lds_q[256 * 8 * NV];
  __shared__ float ch_s[GN_MAXC], ch_q[GN_MAXC];
  const int img = blockIdx.y, chunk = blockIdx.x;
  const int VPR = C / (8 * NV);  // thread slots per row (each slot = NV vectors of 8)
  const int RP = 256 / VPR;      // rows per pass
  const int t = threadIdx.x;
  const int v = t % VPR, ro = t / VPR;
  float s[8 * NV], q[8 * NV];
#pragma unroll
  for (int i = 0; i < 8 * NV; ++i) s[i] = q[i] = 0.f;
  const int r0 = chunk * rows_per_chunk;
  const int r1 = min(r0 + rows_per_chunk, HW);
  if (ro < RP) {
    // U rows' loads in flight per thread, accumulated in row order (same sums as a one-row loop)
    constexpr int U = 4;
    for (int r = r0 + ro; r < r1; r += RP * U) {
      V8 val[U][NV];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rr = r + u * RP;
        const long long m = (long long)img * HW + (rr < r1 ? rr : r);
        if constexpr (CAT) {
#pragma unroll
          for (int n = 0; n < NV; ++n) {
            const int c = (v + n * VPR) * 8;
            val[u][n] = c < C1 ? *(const V8*)(x + m * C1 + c) : *(const V8*)(b + m * (C - C1) + (c - C1));
          }
        } else {
          const T* row = x + m * C;
#pragma unroll
          for (int n = 0; n < NV; ++n) val[u][n] = *(const V8*)(row + (v + n * VPR) * 8);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (r + u * RP >= r1) break;
        if constexpr (CAT) {
#pragma unroll
          for (int n = 0; n < NV; ++n)
            st_out16((V8*)(y + ((long long)img * HW + r + u * RP) * C + (v + n * VPR) * 8), val[u][n]);
        }
#pragma unroll
        for (int n = 0; n < NV; ++n)
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float f = (float)val[u][n][i];
            s[n * 8 + i] += f;
            q[n * 8 + i] += f * f;
          }
      }
    }
#pragma unroll
    for (int n = 0; n < NV; ++n)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        lds_s[ro * C + (v + n * VPR) * 8 + i] = s[n * 8 + i];
        lds_q[ro * C + (v + n * VPR) * 8 + i] = q[n * 8 + i];
      }
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < RP; ++r) {
      a += lds_s[r * C + c];
      b += lds_q[r * C + c];
    }
    ch_s[c] = a;
    ch_q[c] = b;
  }
  __syncthreads();
  const int cpg = C / groups;
  if (t < groups) {
    float a = 0.f, b = 0.f;
    for (int c = t * cpg; c < (t + 1) * cpg; ++c) {
      a += ch_s[c];
      b += ch_q[c];
    }
    part[((long long)img * gridDim.x + chunk) * groups + t] = make_float2(a, b);
  }
}

// fold the per-chunk partials into per-group (mean, rstd): one wave per (group, image), lane j takes chunks
// j, j + 64, ... with all of its loads in flight at once (one L2 round trip instead of a chain of them: the
// one-block-per-image version took 12 us at 1024 chunks), then a shuffle tree in fp64.  Fixed order ->
// bitwise reproducible.  Once per (image, group) -- the apply blocks only read the result.
__global__ void __launch_bounds__(64) gn_finalize_kernel(const float2* __restrict__ part, float2* __restrict__ stats,
                                                         int HW, int C, int groups, int nchunks, float eps) {
  const int g = blockIdx.x, img = blockIdx.y, j = threadIdx.x;
  const int cpg = C / groups;
  const float2* p = part + (long long)img * nchunks * groups + g;
  constexpr int U = 16;  // nchunks <= 1024 = 64 lanes x U
  float2 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = j + 64 * u;
    v[u] = c < nchunks ? p[(long long)c * groups] : make_float2(0.f, 0.f);
  }
  double s = 0.0, q = 0.0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    s += v[u].x;
    q += v[u].y;
  }
  // nchunks > 1024 goes to gn_finalize_wide_kernel (up to 8192); beyond that this loop takes U more loads in flight
  // per round, each lane still summing its chunks j, j + 64, ... in ascending order
  for (int c0 = j + 64 * U; c0 < nchunks; c0 += 64 * U) {
    float2 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + 64 * u;
      w[u] = c < nchunks ? p[(long long)c * groups] : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      s += w[u].x;
      q += w[u].y;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    q += __shfl_xor(q, o, 64);
  }
  if (j == 0) {
    const double n = (double)HW * cpg;
    const double mean = s / n;
    double var = q / n - mean * mean;
    if (var < 0) var = 0;
    stats[img * groups + g] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)eps)));
  }
}

// The same fold for the long partial lists of large images (nchunks > 1024: the producer-epilogue partials of the
// VAE's 512^2 / 1024^2 levels, HW / 128 up to 8192): 1024 threads per (group, image), thread j summing chunks j,
// j + 1024, ... (all in flight) in fp64, a butterfly per wave, then the 16 wave sums in wave order.  Fixed order
// (bitwise reproducible); replaces gn_finalize_kernel's serial 1024-chunk rounds (~12 us per VAE GroupNorm).
__global__ void __launch_bounds__(1024) gn_finalize_wide_kernel(const float2* __restrict__ part,
                                                                float2* __restrict__ stats, int HW, int C, int groups,
                                                                int nchunks, float eps) {
  __shared__ double red[2][16];
  const int g = blockIdx.x, img = blockIdx.y, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const float2* p = part + (long long)img * nchunks * groups + g;
  constexpr int U = 8;  // nchunks <= 8192
  float2 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = t + 1024 * u;
    v[u] = c < nchunks ? p[(long long)c * groups] : make_float2(0.f, 0.f);
  }
  double s = 0.0, q = 0.0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    s += v[u].x;
    q += v[u].y;
  }
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    q += __shfl_xor(q, o, 64);
  }
  if (lane == 0) {
    red[0][w] = s;
    red[1][w] = q;
  }
  __syncthreads();
  if (t == 0) {
    double S = 0.0, Q = 0.0;
    for (int i = 0; i < 16; ++i) {
      S += red[0][i];
      Q += red[1][i];
    }
    const double n = (double)HW * (C / groups);
    const double mean = S / n;
    double var = Q / n - mean * mean;
    if (var < 0) var = 0;
    stats[img * groups + g] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)eps)));
  }
}

static void gn_finalize_launch(const float2* part, float2* stats, int nimg, int HW, int C, int groups, int nchunks,
                               float eps, hipStream_t s) {
  if (nchunks > 1024 && nchunks <= 8192)
    hipLaunchKernelGGL(gn_finalize_wide_kernel, dim3(groups, nimg), dim3(1024), 0, s, part, stats, HW, C, groups,
                       nchunks, eps);
  else
    hipLaunchKernelGGL(gn_finalize_kernel, dim3(groups, nimg), dim3(64), 0, s, part, stats, HW, C, groups, nchunks,
                       eps);
}

template <typename T, int NV, int U = 4>
__global__ void __launch_bounds__(256) gn_apply_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                       const float2* __restrict__ stats, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, int HW, int C, int groups,
                                                       int rows_per_block, int silu) {
  typedef typename VecT<T>::v8 V8;
  __shared__ float sc[GN_MAXC], sh[GN_MAXC];
  __shared__ float mean_s[64], rstd_s[64];
  const int img = blockIdx.y;
  const int t = threadIdx.x;
  const int cpg = C / groups;
  const int VPR = C / 8;
  const long long base = (long long)img * HW * C;
  const long long e1 = (long long)min(blockIdx.x * rows_per_block + rows_per_block, HW) * VPR;
  const long long eb = (long long)blockIdx.x * rows_per_block * VPR;  // a whole-row boundary
  long long e = eb + t;
  // the block's first U vectors are requested before the stats / gamma / beta round trips, and each
  // batch of U is in flight together (a load-compute-store loop exposes one HBM latency per vector)
  V8 val[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (e + u * 256 < e1) val[u] = *(const V8*)(x + base + (e + u * 256) * 8);
  if (t < groups) {
    const float2 st = stats[img * groups + t];
    mean_s[t] = st.x;
    rstd_s[t] = st.y;
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    const int g = c / cpg;
    const float a = rstd_s[g] * (gamma ? gamma[c] : 1.f);
    sc[c] = a;
    sh[c] = __builtin_fmaf(-mean_s[g], a, beta ? beta[c] : 0.f);
  }
  __syncthreads();
  for (; e < e1; e += 256 * U) {
    V8 nxt[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (e + (U + u) * 256 < e1) nxt[u] = *(const V8*)(x + base + (e + (U + u) * 256) * 8);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long ee = e + u * 256;
      if (ee >= e1) break;
      const int v = (int)(ee - eb) % VPR;
      V8 out;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float f = __builtin_fmaf((float)val[u][i], sc[v * 8 + i], sh[v * 8 + i]);
        if (silu) f = silu_f(f);
        out[i] = (T)f;
      }
      st_out16((V8*)(y + base + ee * 8), out);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) val[u] = nxt[u];
  }
  (void)NV;
}

// gn_apply2: the same y = x * scale[c] + shift[c] (+ SiLU), with each thread pinned to one 8-channel chunk
// (t % VPR, the block's first (256 / VPR) * VPR threads): its 8 scales and shifts live in registers, built straight
// from the group statistics -- no LDS tables, no barrier, no per-vector 64-bit modulo -- and U rows' vectors are
// in flight per thread.  Same arithmetic per element as gn_apply_kernel (bitwise equal output).
template <typename T, int U>
__global__ void __launch_bounds__(256) gn_apply2_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                        const float2* __restrict__ stats, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, int HW, int C, int groups,
                                                        int rows_per_block, int silu) {
  typedef typename VecT<T>::v8 V8;
  const int img = blockIdx.y, t = threadIdx.x;
  const int VPR = C / 8, RPP = 256 / VPR;  // chunks per row, rows per pass
  if (t >= RPP * VPR) return;
  const int v = t % VPR, r0 = t / VPR;
  const int cpg = C / groups;
  const int rb = blockIdx.x * rows_per_block, re = min(rb + rows_per_block, HW);
  const T* xb = x + (long long)img * HW * C + v * 8;
  T* yb = y + (long long)img * HW * C + v * 8;
  // the first U rows' vectors are requested before the statistics round trip
  V8 val[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int r = rb + r0 + u * RPP;
    if (r < re) val[u] = *(const V8*)(xb + (long long)r * C);
  }
  float sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = v * 8 + i, g = c / cpg;
    const float2 st = stats[img * groups + g];
    const float a = st.y * (gamma ? gamma[c] : 1.f);
    sc[i] = a;
    sh[i] = __builtin_fmaf(-st.x, a, beta ? beta[c] : 0.f);
  }
  for (int r = rb + r0; r < re; r += RPP * U) {
    V8 nxt[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rn = r + (U + u) * RPP;
      if (rn < re) nxt[u] = *(const V8*)(xb + (long long)rn * C);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rr = r + u * RPP;
      if (rr >= re) break;
      V8 out;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float f = __builtin_fmaf((float)val[u][i], sc[i], sh[i]);
        if (silu) f = silu_f(f);
        out[i] = (T)f;
      }
      st_out16((V8*)(yb + (long long)rr * C), out);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) val[u] = nxt[u];
  }
}

static int gn_apply_version() {
  const int v = fd_knob(FDK_GN_APPLY_V);  // 1 = the LDS-table kernel (A/B)
  return v;
}

// the apply launch shared by fd_group_norm and fd_group_norm_partials (grid: ~1024 blocks of whole rows)
static int gn_apply_launch(const void* x, void* y, const float2* stats, const float* gamma, const float* beta, int nimg,
                           int HW, int C, int groups, int silu, int dtype, hipStream_t s) {
  const int apply_blocks = fd_knob(FDK_GN_APPLY_BLOCKS);
  const int apply_u = fd_knob(FDK_GN_APPLY_U);  // vectors in flight per thread (4 or 8)
  int rpb = 1;
  while ((long long)nimg * ((HW + rpb - 1) / rpb) > apply_blocks) rpb *= 2;
  const int nblk = (HW + rpb - 1) / rpb;
  if (gn_apply_version() == 2 && C / 8 <= 256) {
    if (apply_u == 8) {
      FD_DISPATCH_T(dtype, hipLaunchKernelGGL((gn_apply2_kernel<T, 8>), dim3(nblk, nimg), dim3(256), 0, s,
                                              (const T*)x, (T*)y, stats, gamma, beta, HW, C, groups, rpb, silu));
    } else {
      FD_DISPATCH_T(dtype, hipLaunchKernelGGL((gn_apply2_kernel<T, 4>), dim3(nblk, nimg), dim3(256), 0, s,
                                              (const T*)x, (T*)y, stats, gamma, beta, HW, C, groups, rpb, silu));
    }
  } else if (apply_u == 8) {
    FD_DISPATCH_T(dtype, hipLaunchKernelGGL((gn_apply_kernel<T, 1, 8>), dim3(nblk, nimg), dim3(256), 0, s,
                                            (const T*)x, (T*)y, stats, gamma, beta, HW, C, groups, rpb, silu));
  } else {
    FD_DISPATCH_T(dtype, hipLaunchKernelGGL((gn_apply_kernel<T, 1>), dim3(nblk, nimg), dim3(256), 0, s, (const T*)x,
                                            (T*)y, stats, gamma, beta, HW, C, groups, rpb, silu));
  }
  FD_LAUNCH_CHECK();
  return FD_OK;
}

extern "C" long long fd_group_norm_ws_bytes(int nimg, int HW, int C, int groups) {
  const int rpc = gn_rows_per_chunk(nimg, HW);
  const int nch = (HW + rpc - 1) / rpc;
  return (long long)nimg * (nch + 1) * groups * sizeof(float2);  // partials, then per-group stats
}

extern "C" int fd_group_norm(const void* x, void* y, const float* gamma, const float* beta, int nimg, int HW, int C,
                             int groups, float eps, int silu, int dtype, void* ws, void* stream) {
  if (!x || !y || !ws) return FD_ERR_ARG;
  if (nimg <= 0 || HW <= 0 || C <= 0 || groups <= 0 || groups > 64 || (groups & (groups - 1)) || C % groups ||
      C % 8 || C > GN_MAXC)
    return FD_ERR_SHAPE;
  const int rpc = gn_rows_per_chunk(nimg, HW);
  const int nch = (HW + rpc - 1) / rpc;
  hipStream_t s = (hipStream_t)stream;
  const int NV = (C / 8 > 256) ? 2 : 1;
  if (NV == 2 && (C % 16)) return FD_ERR_SHAPE;
  if (NV == 1) {
    FD_DISPATCH_T(dtype, hipLaunchKernelGGL((gn_partial_kernel<T, 1>), dim3(nch, nimg), dim3(256), 0, s, (const T*)x,
                                            (float2*)ws, HW, C, groups, rpc));
  } else {
    FD_DISPATCH_T(dtype, hipLaunchKernelGGL((gn_partial_kernel<T, 2>), dim3(nch, nimg), dim3(256), 0, s, (const T*)x,
                                            (float2*)ws, HW, C, groups, rpc));
  }
  FD_LAUNCH_CHECK();
  float2* stats = (float2*)ws + (long long)nimg * nch * groups;
  gn_finalize_launch((const float2*)ws, stats, nimg, HW, C, groups, nch, eps, s);
  FD_LAUNCH_CHECK();
  return gn_apply_launch(x, y, stats, gamma, beta, nimg, HW, C, groups, silu, dtype, s);
}

// Rows per statistics chunk of fd_group_norm's own pass (and of fd_concat_channels_gn's partials) for this image size.
extern "C" int fd_group_norm_chunk_rows(int nimg, int HW) { return HW > 0 ? gn_rows_per_chunk(nimg, HW) : 0; }

// y = concat(a [M, C1], b [M, C2]) along channels (M = nimg * HW) AND the GroupNorm statistics of y, per image,
// fd_group_norm_chunk_rows(nimg, HW)-row chunk and group, into part[(img * HW / rows + chunk) * groups + g] (float2):
// the input for fd_group_norm_partials / fd_group_norm_affine with part_rows = those rows.  One launch instead of the
// concat and the statistics pass; the partials are bit for bit fd_group_norm's own.
extern "C" int fd_concat_channels_gn(const void* a, int C1, const void* b, int C2, void* y, int nimg, int HW,
                                     int groups, void* part, int dtype, void* stream) {
  if (!a || !b || !y || !part) return FD_ERR_ARG;
  const int C = C1 + C2;
  if (C1 % 8 || C2 % 8 || C1 <= 0 || C2 <= 0 || nimg <= 0 || HW <= 0 || groups <= 0 || groups > 64 || C % groups ||
      C > GN_MAXC)
    return FD_ERR_SHAPE;
  const int rpc = gn_rows_per_chunk(nimg, HW);
  const int nch = (HW + rpc - 1) / rpc;
  const int NV = (C / 8 > 256) ? 2 : 1;
  if (NV == 2 && (C % 16)) return FD_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  if (NV == 1) {
    FD_DISPATCH_T(dtype, hipLaunchKernelGGL((gn_partial_kernel<T, 1, true>), dim3(nch, nimg), dim3(256), 0, s,
                                            (const T*)a, (float2*)part, HW, C, groups, rpc, (const T*)b, C1, (T*)y));
  } else {
    FD_DISPATCH_T(dtype, hipLaunchKernelGGL((gn_partial_kernel<T, 2, true>), dim3(nch, nimg), dim3(256), 0, s,
                                            (const T*)a, (float2*)part, HW, C, groups, rpc, (const T*)b, C1, (T*)y));
  }
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// GroupNorm whose statistics the producing GEMM / conv epilogue already wrote (fd_gemm_params.gn_part, gn_done):
// part[(img * HW/256 + b) * groups + g] = (sum, sumsq) of the 256-row block b.  Finalize (fp64 fold, fixed order)
// into stats (nimg * groups float2, caller's) + apply: the gn_partial pass (one full read of x) is gone.
extern "C" int fd_group_norm_partials(const void* x, void* y, const float* gamma, const float* beta, int nimg, int HW,
                                      int C, int groups, float eps, int silu, const void* part, int part_rows,
                                      void* stats, int dtype, void* stream) {
  if (!x || !y || !part || !stats) return FD_ERR_ARG;
  // 256 / 128: the GEMM / conv epilogue partials; other powers of two: the statistics-pass chunks of
  // fd_concat_channels_gn (fd_group_norm_chunk_rows)
  if (part_rows <= 0 || (part_rows & (part_rows - 1)) || HW % part_rows) return FD_ERR_ARG;
  if (nimg <= 0 || HW <= 0 || HW % part_rows || C <= 0 || groups <= 0 || groups > 64 || C % groups || C % 8 ||
      C > GN_MAXC)
    return FD_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  gn_finalize_launch((const float2*)part, (float2*)stats, nimg, HW, C, groups, HW / part_rows, eps, s);
  FD_LAUNCH_CHECK();
  return gn_apply_launch(x, y, (const float2*)stats, gamma, beta, nimg, HW, C, groups, silu, dtype, s);
}

// GroupNorm as a per-(image, channel) affine (a, b) = (rstd * gamma, beta - mean * a): gn_apply2's scale / shift, for
// a consumer that applies it in its own staging pass (the halo conv, fd_gemm_params.gi_affine).  The 64 channels
// after the last image are zeroed (the conv DMAs the table 1 KB at a time).
__global__ void __launch_bounds__(256) gn_affine_kernel(const float2* __restrict__ stats, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float2* __restrict__ aff,
                                                        int nimg, int C, int groups) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long tot = (long long)nimg * C;
  if (e >= tot) {
    if (e < tot + 64) aff[e] = make_float2(0.f, 0.f);
    return;
  }
  const int img = (int)(e / C), c = (int)(e - (long long)img * C);
  const float2 st = stats[img * groups + c / (C / groups)];
  const float a = st.y * (gamma ? gamma[c] : 1.f);
  aff[e] = make_float2(a, __builtin_fmaf(-st.x, a, beta ? beta[c] : 0.f));
}

// gn_finalize_kernel + gn_affine_kernel in one launch (the per-resnet GroupNorm of the halo conv: two ~5 us
// latency-bound launches -> one): one wave per (group, image) folds the partials exactly as gn_finalize_kernel, then
// writes the group's channels' (a, b) exactly as gn_affine_kernel; block (0, 0) also zeroes the 64-channel pad.
__global__ void __launch_bounds__(64) gn_finalize_affine_kernel(const float2* __restrict__ part,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta, float2* __restrict__ aff,
                                                                int HW, int C, int groups, int nchunks, float eps) {
  const int g = blockIdx.x, img = blockIdx.y, j = threadIdx.x, nimg = gridDim.y;
  const int cpg = C / groups;
  const float2* p = part + (long long)img * nchunks * groups + g;
  constexpr int U = 16;
  double s = 0.0, q = 0.0;
  for (int c0 = j; c0 < nchunks; c0 += 64 * U) {
    float2 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + 64 * u;
      w[u] = c < nchunks ? p[(long long)c * groups] : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      s += w[u].x;
      q += w[u].y;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    q += __shfl_xor(q, o, 64);
  }
  const double n = (double)HW * cpg;
  const double mean = s / n;
  double var = q / n - mean * mean;
  if (var < 0) var = 0;
  const float2 st = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)eps)));
  for (int k = j; k < cpg; k += 64) {
    const int c = g * cpg + k;
    const float a = st.y * (gamma ? gamma[c] : 1.f);
    aff[(long long)img * C + c] = make_float2(a, __builtin_fmaf(-st.x, a, beta ? beta[c] : 0.f));
  }
  if (g == 0 && img == 0) aff[(long long)nimg * C + j] = make_float2(0.f, 0.f);
}

extern "C" int fd_group_norm_affine(const void* x, const void* part, int part_rows, const float* gamma,
                                    const float* beta, int nimg, int HW, int C, int groups, float eps, void* ws,
                                    void* affine, int dtype, void* stream) {
  if (!ws || !affine || (!x && !part)) return FD_ERR_ARG;
  if (nimg <= 0 || HW <= 0 || C <= 0 || groups <= 0 || groups > 64 || C % groups || C % 8 || C > GN_MAXC)
    return FD_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  float2* stats;
  if (part) {
    if (part_rows <= 0 || (part_rows & (part_rows - 1)) || HW % part_rows) return FD_ERR_ARG;
    stats = (float2*)ws;
    const int nch = HW / part_rows;
    if (nch <= 1024) {  // one launch (the wide fold's long lists keep the two-launch form)
      hipLaunchKernelGGL(gn_finalize_affine_kernel, dim3(groups, nimg), dim3(64), 0, s, (const float2*)part, gamma,
                         beta, (float2*)affine, HW, C, groups, nch, eps);
      FD_LAUNCH_CHECK();
      return FD_OK;
    }
    gn_finalize_launch((const float2*)part, stats, nimg, HW, C, groups, nch, eps, s);
  } else {
    if ((groups & (groups - 1))) return FD_ERR_SHAPE;
    const int rpc = gn_rows_per_chunk(nimg, HW);
    const int nch = (HW + rpc - 1) / rpc;
    const int NV = (C / 8 > 256) ? 2 : 1;
    if (NV == 2 && (C % 16)) return FD_ERR_SHAPE;
    if (NV == 1) {
      FD_DISPATCH_T(dtype, hipLaunchKernelGGL((gn_partial_kernel<T, 1>), dim3(nch, nimg), dim3(256), 0, s,
                                              (const T*)x, (float2*)ws, HW, C, groups, rpc));
    } else {
      FD_DISPATCH_T(dtype, hipLaunchKernelGGL((gn_partial_kernel<T, 2>), dim3(nch, nimg), dim3(256), 0, s,
                                              (const T*)x, (float2*)ws, HW, C, groups, rpc));
    }
    FD_LAUNCH_CHECK();
    if (nch <= 1024) {
      // the fused fold + affine, the same fp64 order as gn_finalize_kernel: one ~5 us latency-bound launch fewer per
      // halo conv whose input statistics no producer wrote (round 6)
      hipLaunchKernelGGL(gn_finalize_affine_kernel, dim3(groups, nimg), dim3(64), 0, s, (const float2*)ws, gamma,
                         beta, (float2*)affine, HW, C, groups, nch, eps);
      FD_LAUNCH_CHECK();
      return FD_OK;
    }
    stats = (float2*)ws + (long long)nimg * nch * groups;
    gn_finalize_launch((const float2*)ws, stats, nimg, HW, C, groups, nch, eps, s);
  }
  FD_LAUNCH_CHECK();
  const long long n = (long long)nimg * C + 64;
  hipLaunchKernelGGL(gn_affine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const float2*)stats, gamma,
                     beta, (float2*)affine, nimg, C, groups);
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// ------------------------------------------------------------------------------------------------
// LayerNorm: one wave per row, 4 rows per 256-thread block; row kept in registers (C <= 2048).  Every output path
// computes fma((x - mean) * rstd, gamma, beta) explicitly and rounds it fp32 -> T (round_f32), so the y / e4m3 / MX
// forms round identically.
// Q8 = 1: instead of y, write the row quantized to e4m3 for fd_gemm_e4m3 (the use_fp8 model): the LayerNorm output is
// rounded to T first and then quantized exactly as fd_quant_rows_e4m3 does, so LN + quant fused == LN; quant.
// Q8 = 2: the same rounded output as MX e4m3 (fd_quant_rows_mx's bytes): a 32-element block = 4 consecutive lanes.
template <typename T, int Q8>
__global__ void __launch_bounds__(256) layer_norm_kernel(const T* __restrict__ x, long long ldx, T* __restrict__ y,
                                                         long long ldy, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, int M, int C, float eps,
                                                         uint8_t* __restrict__ q8, long long ldq,
                                                         float* __restrict__ qscale, uint8_t* __restrict__ qbs = nullptr,
                                                         long long ldbs = 0) {
  typedef typename VecT<T>::v8 V8;
  constexpr int MAXV = 4;  // up to 4 vectors of 8 per lane => C <= 2048
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int VPR = C / 8;
  const T* xr = x + row * ldx;
  // row, gamma and beta are all requested up front: one memory round trip per row, not two
  V8 raw[MAXV];
  f32x4 g4[MAXV][2], b4[MAXV][2];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int v = lane + k * 64;
    if (v < VPR) {
      raw[k] = *(const V8*)(xr + v * 8);
      g4[k][0] = *(const f32x4*)(gamma + v * 8);
      g4[k][1] = *(const f32x4*)(gamma + v * 8 + 4);
      b4[k][0] = *(const f32x4*)(beta + v * 8);
      b4[k][1] = *(const f32x4*)(beta + v * 8 + 4);
    }
  }
  float vals[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int v = lane + k * 64;
    if (v < VPR) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        vals[k][i] = (float)raw[k][i];
        s += vals[k][i];
      }
    }
  }
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int v = lane + k * 64;
    if (v < VPR) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = vals[k][i] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / C + eps);
  if (Q8 == 2) {  // C % 32 == 0: a lane's vectors are whole quarters of blocks, groups of 4 lanes all in or out
    V8 outs[MAXV];  // the rounded output first (as the y path stores it), then quantized from those values
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int v = lane + k * 64;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        outs[k][i] = v < VPR ? round_f32<T>(__builtin_fmaf((vals[k][i] - mean) * rstd, g4[k][i >> 2][i & 3],
                                                           b4[k][i >> 2][i & 3]))
                             : (T)0.f;
    }
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int v = lane + k * 64;
      float am = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) am = fmaxf(am, fabsf((float)outs[k][i]));
      am = fmaxf(am, __shfl_xor(am, 1, 64));
      am = fmaxf(am, __shfl_xor(am, 2, 64));
      if (v < VPR) {
        const int E = mx_exp(am);
        const V8 o = outs[k];
        *(u32x2*)(q8 + row * ldq + v * 8) =
            u32x2{mx_pack4((float)o[0], (float)o[1], (float)o[2], (float)o[3], E),
                  mx_pack4((float)o[4], (float)o[5], (float)o[6], (float)o[7], E)};
        if ((v & 3) == 0) qbs[row * ldbs + v / 4] = (uint8_t)(E + 127);
      }
    }
    return;
  }
  if (Q8 == 1) {
    V8 outs[MAXV];
    float amax = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int v = lane + k * 64;
      if (v < VPR) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          outs[k][i] =
              round_f32<T>(__builtin_fmaf((vals[k][i] - mean) * rstd, g4[k][i >> 2][i & 3], b4[k][i >> 2][i & 3]));
          amax = fmaxf(amax, fabsf((float)outs[k][i]));
        }
      }
    }
    amax = wave_max(amax);
    const float inv = amax > 0.f ? __fdiv_rn(448.0f, amax) : 0.f;
    if (lane == 0) qscale[row] = __fdiv_rn(amax, 448.0f);
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int v = lane + k * 64;
      if (v < VPR) {
        const V8 o = outs[k];
        int lo = __builtin_amdgcn_cvt_pk_fp8_f32((float)o[0] * inv, (float)o[1] * inv, 0, false);
        lo = __builtin_amdgcn_cvt_pk_fp8_f32((float)o[2] * inv, (float)o[3] * inv, lo, true);
        int hi = __builtin_amdgcn_cvt_pk_fp8_f32((float)o[4] * inv, (float)o[5] * inv, 0, false);
        hi = __builtin_amdgcn_cvt_pk_fp8_f32((float)o[6] * inv, (float)o[7] * inv, hi, true);
        *(u32x2*)(q8 + row * ldq + v * 8) = u32x2{(unsigned)lo, (unsigned)hi};
      }
    }
    return;
  }
  T* yr = y + row * ldy;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int v = lane + k * 64;
    if (v < VPR) {
      V8 out;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        out[i] = round_f32<T>(__builtin_fmaf((vals[k][i] - mean) * rstd, g4[k][i >> 2][i & 3], b4[k][i >> 2][i & 3]));
      st_out16((V8*)(yr + v * 8), out);
    }
  }
}

extern "C" int fd_layer_norm(const void* x, long long ldx, void* y, long long ldy, const float* gamma,
                             const float* beta, int M, int C, float eps, int dtype, void* stream) {
  if (!x || !y || !gamma || !beta) return FD_ERR_ARG;
  if ((((unsigned long long)gamma) | ((unsigned long long)beta)) & 15) return FD_ERR_ARG;  // 16-B vector loads
  if (M <= 0 || C <= 0 || C % 8 || C > 2048 || (ldx & 7) || (ldy & 7)) return FD_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_T(dtype, hipLaunchKernelGGL((layer_norm_kernel<T, 0>), dim3((M + 3) / 4), dim3(256), 0, s,
                                          (const T*)x, ldx, (T*)y, ldy, gamma, beta, M, C, eps, nullptr, 0, nullptr));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

extern "C" int fd_layer_norm_e4m3(const void* x, long long ldx, void* q, long long ldq, float* scale,
                                  const float* gamma, const float* beta, int M, int C, float eps, int dtype,
                                  void* stream) {
  if (!x || !q || !scale || !gamma || !beta) return FD_ERR_ARG;
  if ((((unsigned long long)gamma) | ((unsigned long long)beta)) & 15) return FD_ERR_ARG;
  if (M <= 0 || C <= 0 || C % 8 || C > 2048 || (ldx & 7) || (ldq & 7) || ldq < C) return FD_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_T(dtype, hipLaunchKernelGGL((layer_norm_kernel<T, 1>), dim3((M + 3) / 4), dim3(256), 0, s,
                                          (const T*)x, ldx, (T*)nullptr, 0, gamma, beta, M, C, eps, (uint8_t*)q, ldq,
                                          scale, nullptr, 0));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

extern "C" int fd_layer_norm_mx(const void* x, long long ldx, void* q, long long ldq, void* sb, long long lds,
                                const float* gamma, const float* beta, int M, int C, float eps, int dtype, void* stream) {
  if (!x || !q || !sb || !gamma || !beta) return FD_ERR_ARG;
  if ((((unsigned long long)gamma) | ((unsigned long long)beta)) & 15) return FD_ERR_ARG;
  if (((unsigned long long)q) & 7) return FD_ERR_ARG;
  if (M <= 0 || C <= 0 || C % 32 || C > 2048 || (ldx & 7) || (ldq & 7) || ldq < C || lds < C / 32)
    return FD_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_T(dtype, hipLaunchKernelGGL((layer_norm_kernel<T, 2>), dim3((M + 3) / 4), dim3(256), 0, s,
                                          (const T*)x, ldx, (T*)nullptr, 0, gamma, beta, M, C, eps, (uint8_t*)q, ldq,
                                          nullptr, (uint8_t*)sb, lds));
  FD_LAUNCH_CHECK();
  return FD_OK;
}
