// MFMA GEMM and implicit-GEMM 3x3 convolution for gfx950.
//
// One kernel template serves every nn.Linear and every 3x3 / 1x1 nn.Conv2d (Cin % 64 == 0) of the
// SDXL UNet, the FaithDiff extras and the fp16 VAE.  Design (cdna_hip_programming.md
// section 5): 256-thread workgroups (4 waves of 64), tile BM x BN x 64, each wave a WM x WN sub-tile
// of v_mfma_f32_16x16x32_{bf16,f16}; both operands K-contiguous ([rows][K]) and staged
// global -> LDS with global_load_lds_dwordx4 (no VGPR round trip) into a double buffer; the
// bank-conflict XOR swizzle (chunk ^= (row>>1)&7 on 128-B rows) is applied on the per-lane global
// SOURCE address, because the LDS-DMA destination is lane-linear (guide rule 21), and on the
// ds_read_b128 fragment address.  The conv variant gathers its A rows straight from the NHWC
// image (im2col never materialised): out-of-image taps point at a zero page, the nearest x2
// Upsample2D and the up-block skip concat are folded into that gather.
#include "fd_common.h"

__device__ __attribute__((aligned(256))) unsigned char g_zero_page[256];

template <typename T, int BM, int BN, int WM, int WN, bool CONV, bool GEGLU, typename TO>
__global__ void __launch_bounds__(256) gemm_kernel(const fd_gemm_params p) {
  typedef typename VecT<T>::v8 V8;
  constexpr int WAVES_N = BN / WN;
  constexpr int MT = WM / 16, NT = WN / 16;
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_INSTR = BM / 32, B_INSTR = BN / 32;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const long long bz = blockIdx.z;
  const T* __restrict__ A = (const T*)p.A + bz * p.strideA;
  const T* __restrict__ Bw = (const T*)p.B + bz * p.strideB;
  const int M = p.M, N = p.N, K = p.K;
  const int lrow = lane >> 3, slot = lane & 7;

  // ---- per-lane A-row state (rows fixed over the K loop)
  const T* a_row[A_INSTR];
  int a_iy0[A_INSTR], a_ix0[A_INSTR], a_chunk[A_INSTR];
  long long a_pix[A_INSTR];
  bool a_ok[A_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int row = (i * 4 + wave) * 8 + lrow;
    const int m = m0 + row;
    a_ok[i] = m < M;
    const int mm = m < M ? m : M - 1;
    a_chunk[i] = slot ^ ((row >> 1) & 7);
    if (CONV) {
      const int hw = p.Hout * p.Wout;
      const int img = mm / hw;
      const int rem = mm - img * hw;
      const int oy = rem / p.Wout, ox = rem - (rem / p.Wout) * p.Wout;
      a_iy0[i] = oy * p.stride - p.pad;
      a_ix0[i] = ox * p.stride - p.pad;
      a_pix[i] = (long long)img * p.Hin * p.Win;
      a_row[i] = nullptr;
    } else {
      a_row[i] = A + (long long)mm * p.lda + a_chunk[i] * 8;
      a_iy0[i] = a_ix0[i] = 0;
      a_pix[i] = 0;
    }
  }
  const T* b_row[B_INSTR];
#pragma unroll
  for (int i = 0; i < B_INSTR; ++i) {
    const int row = (i * 4 + wave) * 8 + lrow;
    const int n = n0 + row;
    b_row[i] = Bw + (long long)(n < N ? n : N - 1) * p.ldb + (slot ^ ((row >> 1) & 7)) * 8;
  }
  // upsample: the conv runs on a nearest-resized (Hout x Wout) image; exact x2 or diffusers' upsample_size
  const int Hl = p.upsample ? p.Hout : p.Hin, Wl = p.upsample ? p.Wout : p.Win;
  const int C1 = p.C1 > 0 ? p.C1 : p.Cin;
  const T* __restrict__ A2 = (const T*)p.A2;

  auto stage = [&](int kt, int buf) {
    const int k0 = kt * 64;
    unsigned char* sa = smem + buf * STAGE;
    if (CONV) {
      const int tap = k0 / p.Cin;
      const int c0 = k0 - tap * p.Cin;
      const int ky = tap / 3, kx = tap - (tap / 3) * 3;
      const bool second = (A2 != nullptr) && (c0 >= C1);
#pragma unroll
      for (int i = 0; i < A_INSTR; ++i) {
        const int iy = a_iy0[i] + ky, ix = a_ix0[i] + kx;
        const bool ok = a_ok[i] && iy >= 0 && iy < Hl && ix >= 0 && ix < Wl;
        const int py = p.upsample ? (iy * p.Hin) / Hl : iy, px = p.upsample ? (ix * p.Win) / Wl : ix;
        const long long pix = a_pix[i] + (long long)py * p.Win + px;
        const T* src = second ? (A2 + pix * (p.Cin - C1) + (c0 - C1) + a_chunk[i] * 8)
                              : (A + pix * p.lda + c0 + a_chunk[i] * 8);
        const void* s = ok ? (const void*)src : (const void*)g_zero_page;
        __builtin_amdgcn_global_load_lds(s, LDS_PTR(sa + (i * 4 + wave) * 1024), 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_INSTR; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(a_row[i] + k0), LDS_PTR(sa + (i * 4 + wave) * 1024), 16, 0, 0);
    }
    unsigned char* sb = sa + A_BYTES;
#pragma unroll
    for (int i = 0; i < B_INSTR; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(b_row[i] + k0), LDS_PTR(sb + (i * 4 + wave) * 1024), 16, 0, 0);
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = K / 64;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int fr = lane & 15, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, buf ^ 1);
    const unsigned char* sa = smem + buf * STAGE;
    const unsigned char* sb = sa + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      V8 af[MT], bfr[NT];
      const int ch = kk * 4 + fg;
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int r = wm * WM + mi * 16 + fr;
        af[mi] = *(const V8*)(sa + r * 128 + ((ch ^ ((r >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) {
        const int r = wn * WN + ni * 16 + fr;
        bfr[ni] = *(const V8*)(sb + r * 128 + ((ch ^ ((r >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NT; ++ni) acc[mi][ni] = mfma16x16x32(af[mi], bfr[ni], acc[mi][ni]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: acc[mi][ni][j] = C[m0 + wm*WM + mi*16 + 4*fg + j][n0 + wn*WN + ni*16 + fr]
  TO* __restrict__ C = (TO*)p.C + bz * p.strideC;
  const TO* __restrict__ R = p.residual ? (const TO*)p.residual + bz * p.strideR : nullptr;
  const float alpha = p.alpha;
  if (GEGLU) {
    const int Nout = N / 2;
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NT; ni += 2) {
        const int np = n0 + wn * WN + ni * 16 + fr;      // packed "hidden" column
        const int no = (n0 + wn * WN) / 2 + (ni / 2) * 16 + fr;
        if (np >= N) continue;
        const float bh = p.bias ? p.bias[np] : 0.f, bg = p.bias ? p.bias[np + 16] : 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = m0 + wm * WM + mi * 16 + fg * 4 + j;
          if (m >= M) continue;
          const float h = acc[mi][ni][j] * alpha + bh;
          const float g = acc[mi][ni + 1][j] * alpha + bg;
          float v = h * gelu_f(g);
          if (R) v += (float)R[(long long)m * p.ldr + no];
          C[(long long)m * p.ldc + no] = (TO)v;
          (void)Nout;
        }
      }
  } else {
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) {
        const int n = n0 + wn * WN + ni * 16 + fr;
        if (n >= N) continue;
        const float b = p.bias ? p.bias[n] : 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = m0 + wm * WM + mi * 16 + fg * 4 + j;
          if (m >= M) continue;
          float v = acc[mi][ni][j] * alpha + b;
          if (p.rowbias) v += p.rowbias[(long long)(m / p.rows_per_group) * p.rowbias_ld + n];
          v = act_f(v, p.act);
          if (R) v += (float)R[(long long)m * p.ldr + n];
          C[(long long)m * p.ldc + n] = (TO)v;
        }
      }
  }
}

template <typename T, int BM, int BN, int WM, int WN, typename TO>
static int launch_cfg(const fd_gemm_params* p, hipStream_t s) {
  const int tiles = ((p->M + BM - 1) / BM) * ((p->N + BN - 1) / BN);
  dim3 grid(tiles, 1, p->batch > 0 ? p->batch : 1), block(256);
  if (p->conv) {
    if (p->act == FD_ACT_GEGLU) return FD_ERR_ARG;
    hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WM, WN, true, false, TO>), grid, block, 0, s, *p);
  } else if (p->act == FD_ACT_GEGLU) {
    hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WM, WN, false, true, TO>), grid, block, 0, s, *p);
  } else {
    hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WM, WN, false, false, TO>), grid, block, 0, s, *p);
  }
  FD_LAUNCH_CHECK();
  return FD_OK;
}

template <typename T, typename TO>
static int dispatch_tiles(const fd_gemm_params* p, hipStream_t s) {
  const long long t128 = (long long)((p->M + 127) / 128) * ((p->N + 127) / 128) * (p->batch > 0 ? p->batch : 1);
  const long long t12864 = (long long)((p->M + 127) / 128) * ((p->N + 63) / 64) * (p->batch > 0 ? p->batch : 1);
  if (p->N > 64 && t128 >= 256) return launch_cfg<T, 128, 128, 64, 64, TO>(p, s);
  if (t12864 >= 256 || p->N <= 64) return launch_cfg<T, 128, 64, 64, 32, TO>(p, s);
  return launch_cfg<T, 64, 64, 32, 32, TO>(p, s);
}

extern "C" int fd_gemm(const fd_gemm_params* p, void* stream) {
  if (!p || !p->A || !p->B || !p->C) return FD_ERR_ARG;
  if (p->M <= 0 || p->N <= 0 || p->K <= 0 || (p->K % 64) != 0) return FD_ERR_SHAPE;
  if (p->act == FD_ACT_GEGLU && (p->N % 32) != 0) return FD_ERR_SHAPE;
  if (p->rowbias && p->rows_per_group <= 0) return FD_ERR_ARG;
  if (p->conv) {
    if (p->Cin % 64 || (p->C1 > 0 && (p->C1 % 64 || !p->A2)) || p->K != 9 * p->Cin) return FD_ERR_SHAPE;
    if (p->M != p->nimg * p->Hout * p->Wout) return FD_ERR_SHAPE;
    if (p->stride != 1 && p->stride != 2) return FD_ERR_SHAPE;
    if (p->upsample && (p->stride != 1 || p->pad != 1 || p->Hout < p->Hin || p->Wout < p->Win)) return FD_ERR_SHAPE;
  }
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_T(p->dtype, FD_DISPATCH_O(p->out_dtype, return dispatch_tiles<T, TO>(p, s)));
}
