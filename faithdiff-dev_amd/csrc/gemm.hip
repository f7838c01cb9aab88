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
#include <stdlib.h>

#include <type_traits>

#include "fd_common.h"

__device__ __attribute__((aligned(256))) unsigned char g_zero_page[256];

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Tile order.  Workgroups are dealt round-robin to the 8 XCDs (blocks b and b+8 share one; each XCD has
// its own 4 MiB L2).  swz = 1: give each XCD a contiguous chunk of the tile space (bijective remap,
// cdna_hip_programming.md section 5 "XCD swizzle must be bijective"), and walk that chunk in groups of
// GROUP_M tile rows so the ~32 tiles an XCD runs at once share A row-panels and B column-panels in L2.
__device__ __forceinline__ void tile_coords(int bid, int nwg, int tiles_m, int tiles_n, int swz, int GROUP_M, int& tm,
                                            int& tn) {
  if (!swz) {
    tm = bid / tiles_n;
    tn = bid % tiles_n;
    return;
  }
  const int pid = xcd_remap(bid, nwg);
  const int group = pid / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int in_group = pid - group * (GROUP_M * tiles_n);
  tm = first_m + in_group % gsz;
  tn = in_group / gsz;
}

// KS = 2: intra-workgroup split of every 64-deep K step.  Eight waves: waves 0-3 (the loaders) take the
// first 32 of each K step, waves 4-7 the second 32, each over the same wave tile; the halves are summed
// through LDS before the epilogue.  Same LDS traffic and tile shape, but two waves per SIMD, so one
// wave's LDS fragment reads overlap the other's MFMAs (with one 4-wave workgroup per CU -- 256-tile
// launches -- the single wave per SIMD otherwise serialises them).
template <typename T, int BM, int BN, int WM, int WN, int NS, bool CONV, bool GEGLU, typename TO, int KS,
          bool LNF = false>
__global__ void __launch_bounds__(256 * KS) gemm_kernel(const fd_gemm_params p, int swz) {
  typedef typename VecT<T>::v8 V8;
  constexpr int WAVES_N = BN / WN;
  constexpr int MT = WM / 16, NT = WN / 16;
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  // loader waves: all eight under KS = 2 when both panels split into 64-row groups, else waves 0-3
  constexpr int NL = (KS == 2 && BM % 64 == 0 && BN % 64 == 0) ? 8 : 4;
  constexpr int A_INSTR = BM / (8 * NL), B_INSTR = BN / (8 * NL);
  constexpr int PER = A_INSTR + B_INSTR;  // global_load_lds per loader lane per pipeline stage
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves");
  static_assert(NS >= 2 && NS <= 4 && (NS - 2) * PER < 64, "pipeline depth");
  constexpr int BNO = GEGLU ? BN / 2 : BN;   // output columns of the tile
  constexpr int LDE = BNO + 4;               // fp32 epilogue staging row stride (16-B aligned rows)
  constexpr int EPB = (KS == 2 && BN + 4 > LDE) ? BM * (BN + 4) * 4 : BM * LDE * 4;
  // LN-fold producer (64 x 160 tiles only, the configuration fd_gemm forces for it): per-(row, 8-column
  // slot) (sum, sumsq) after the fp32 staging tile
  constexpr bool LNP = (BM == 64 && BN == 160 && !GEGLU && !CONV);
  constexpr int LNS_OFF = (EPB + 15) / 16 * 16, LNS = LNP ? BM * (BNO / 8) * 8 : 0;
  // LN-fold consumer (LNF): (mean, rstd) of the tile's rows and ln_c of its columns, in the same LDS object
  // as the ring (a second __shared__ array makes hipcc assume ds_reads may alias the LDS-DMA targets and
  // drain vmcnt(0) in front of them)
  // (after the ring AND the staging areas: ln_cs is written while other waves may still read the ring)
  constexpr int LNC_OFF = (NS * STAGE > LNS_OFF + LNS) ? NS * STAGE : LNS_OFF + LNS;
  constexpr int LNC = LNF ? BM * 8 + BN * 4 : 0;
  // GroupNorm output statistics (fd_gemm_params.gn_part, 128-row blocks) from the 128 x 128 tiles: every thread
  // keeps one 8-column chunk in every row pass (NTHR % 16 == 0); reduction scratch after everything else
  constexpr bool GN4 = !GEGLU && !LNF && BM == 128 && BN == 128;
  constexpr int SMEM = LNC_OFF + LNC + (GN4 ? 16 * 256 * KS : 0);
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];
  float2* const ln_tab = (float2*)(smem + LNC_OFF);
  float* const ln_cs = (float*)(smem + LNC_OFF + BM * 8);

  constexpr int NTHR = 256 * KS;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kh = wave_all >> 2;     // K half (KS = 2), 0 otherwise
  const int wave = wave_all & 3;    // position in the 4-wave tile grid / loader index
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int lw = NL == 8 ? wave_all : wave;  // loader index
  const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
  // swz bits 4-5: diagnostic mode (FD_GEMM_MODE, benchmarks only): 1 = operand loads only (no LDS reads,
  // no MFMA), 2 = LDS reads + MFMA only (no global loads).  0 in every product launch.
  const int mode = (swz >> 4) & 3;
  const int group_m = (swz >> 8) > 0 ? (swz >> 8) : 4;  // bits 8+: tile-row group height (host-planned)
  swz &= 1;
  int tm, tn;
  tile_coords(blockIdx.x, gridDim.x, tiles_m, tiles_n, swz, group_m, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  // batch offsets (two-level: z -> (z / batch_inner, z % batch_inner)) and the per-row-group B slot (bsel)
  const int zb = blockIdx.z;
  const int zi = p.batch_inner > 1 ? zb % p.batch_inner : zb, zo = p.batch_inner > 1 ? zb / p.batch_inner : 0;
  const int bslot = p.bsel_rows > 0 ? (p.bsel_mod > 0 ? (m0 / p.bsel_rows) % p.bsel_mod : m0 / p.bsel_rows) : 0;
  const long long bsn = (long long)bslot * p.bsel_strideN;
  // residual prefetch (64 x 160 tiles, one workgroup per CU for the M = 2048 projections): the epilogue's
  // residual rows are requested before the first operand stage, so no memory round trip is left between
  // the last MFMA and the stores
  constexpr bool PREF = (BM == 64 && BN == 160 && !GEGLU);
  constexpr int PF_VPR = BN / 8, PF_TOT = BM * PF_VPR, PF_ITER = (PF_TOT + 256 * KS - 1) / (256 * KS);
  typedef __attribute__((ext_vector_type(8))) TO TO8P;
  TO8P res_pf[PREF ? PF_ITER : 1];
  const bool pf = PREF && p.residual && (p.ldr % 8 == 0) && ((((unsigned long long)p.residual) & 15) == 0) &&
                  m0 + BM <= p.M && n0 + BN <= p.N;
  if (PREF && pf) {
    const TO* Rp = (const TO*)p.residual + (long long)zb * p.strideR;
#pragma unroll
    for (int it = 0; it < (PREF ? PF_ITER : 1); ++it) {
      const int e = threadIdx.x + it * 256 * KS;
      if (PF_TOT % (256 * KS) == 0 || e < PF_TOT)
        res_pf[it] = *(const TO8P*)(Rp + (long long)(m0 + e / PF_VPR) * p.ldr + n0 + (e % PF_VPR) * 8);
    }
  }
  // LN-fold consumer: the producer's (sum, sumsq) partials of this tile's rows and ln_c of its columns,
  // requested before the first operand stage so their latency is hidden by the K loop (unconditional
  // 16-B loads, index clamped, lnP even: a conditional load per partial gets sunk into the fold's
  // branches, one dependent round trip each)
  const int lnP = p.K / 160;
  f32x4 lnv4[LNF ? 4 : 1];
  float lncv = 0.f;
  if (LNF) {
    if (tid < BM) {
      const f32x4* src = (const f32x4*)((const float2*)p.ln_in + (long long)min(m0 + tid, p.M - 1) * lnP);
#pragma unroll
      for (int i = 0; i < (LNF ? 4 : 1); ++i) lnv4[i] = src[min(i, lnP / 2 - 1)];
    }
    if (tid < BN) lncv = p.ln_c[bsn + min(n0 + tid, p.N - 1)];
  }
  const long long bz = zb;
  const T* __restrict__ A = (const T*)p.A + zi * p.strideA + zo * p.strideA_o;
  const T* __restrict__ Bw = (const T*)p.B + zi * p.strideB + zo * p.strideB_o + bslot * p.bsel_strideB;
  const int M = p.M, N = p.N, K = p.K;
  const int lrow = lane >> 3, slot = lane & 7;

  // ---- per-lane A-row state (rows fixed over the K loop)
  const T* a_row[A_INSTR];
  int a_iy0[A_INSTR], a_ix0[A_INSTR], a_chunk[A_INSTR];
  long long a_pix[A_INSTR];
  bool a_ok[A_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int row = (i * NL + lw) * 8 + lrow;
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
    const int row = (i * NL + lw) * 8 + lrow;
    const int n = n0 + row;
    b_row[i] = Bw + (long long)(n < N ? n : N - 1) * p.ldb + (slot ^ ((row >> 1) & 7)) * 8;
  }
  // upsample: the conv runs on a nearest-resized (Hout x Wout) image; exact x2 or diffusers' upsample_size
  const int Hl = p.upsample ? p.Hout : p.Hin, Wl = p.upsample ? p.Wout : p.Win;
  const bool up2 = p.upsample && Hl == 2 * p.Hin && Wl == 2 * p.Win;
  const int C1 = p.C1 > 0 ? p.C1 : p.Cin;
  const T* __restrict__ A2 = (const T*)p.A2;

  auto stage = [&](int kt, int buf) {
    if (mode == 2 || (NL == 4 && kh)) return;  // waves 4-7 only compute unless all eight load
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
        // exact x2 (every Upsample2D except diffusers' odd-size upsample_size path): a shift, not a VALU
        // integer division per lane and load (the two divisions cost ~60 VALU instructions per A load)
        int py = iy, px = ix;
        if (p.upsample) {
          if (up2) {
            py = iy >> 1;
            px = ix >> 1;
          } else {
            py = (iy * p.Hin) / Hl;
            px = (ix * p.Win) / Wl;
          }
        }
        const long long pix = a_pix[i] + (long long)py * p.Win + px;
        const T* src = second ? (A2 + pix * (p.Cin - C1) + (c0 - C1) + a_chunk[i] * 8)
                              : (A + pix * p.lda + c0 + a_chunk[i] * 8);
        const void* s = ok ? (const void*)src : (const void*)g_zero_page;
        __builtin_amdgcn_global_load_lds(s, LDS_PTR(sa + (i * NL + lw) * 1024), 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_INSTR; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(a_row[i] + k0), LDS_PTR(sa + (i * NL + lw) * 1024), 16, 0, 0);
    }
    unsigned char* sb = sa + A_BYTES;
#pragma unroll
    for (int i = 0; i < B_INSTR; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(b_row[i] + k0), LDS_PTR(sb + (i * NL + lw) * 1024), 16, 0, FD_WLD_AUX);
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // NS-deep LDS ring: stages kt+1 .. kt+NS-2 stay in flight (counted vmcnt) while stage kt is
  // consumed; one raw s_barrier per K-step (guide section 5, "Pipelining across barriers").
  const int nk = K / 64;
#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0)
    if (s0 < nk) stage(s0, s0);

  const int fr = lane & 15, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(NS - 2, nk - 1 - kt);  // stages issued after kt that may still be in flight
    if (NS >= 4 && ahead >= 2) wait_vmcnt<(NS >= 4 ? 2 * PER : 0)>();
    else if (NS >= 3 && ahead >= 1) wait_vmcnt<(NS >= 3 ? PER : 0)>();
    else wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + NS - 1 < nk) stage(kt + NS - 1, (kt + NS - 1) % NS);
    const unsigned char* sa = smem + (kt % NS) * STAGE;
    const unsigned char* sb = sa + A_BYTES;
    if (mode == 1) continue;
#pragma unroll
    for (int kq = 0; kq < 2 / KS; ++kq) {
      const int kk = KS == 2 ? kh : kq;
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
  }

  constexpr bool lnf = LNF;
  if (LNF && tid < BN) ln_cs[tid] = lncv;

  // ---- epilogue, phase 1: acc[mi][ni][j] = C[wm*WM + mi*16 + 4*fg + j][wn*WN + ni*16 + fr] (tile-local)
  // -> alpha, bias, per-row-group bias, activation / GEGLU in fp32 -> LDS tile [BM][LDE] (fp32)
  __syncthreads();  // every wave is done reading the operand ring
  float* ep = (float*)smem;
  const float alpha = p.alpha;
  if (KS == 2) {  // fold the second K half into the first (fixed order: bitwise reproducible)
    constexpr int LDP = BN + 4;
    if (kh) {
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NT; ++ni)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            ep[(wm * WM + mi * 16 + fg * 4 + j) * LDP + wn * WN + ni * 16 + fr] = acc[mi][ni][j];
    }
    __syncthreads();
    if (!kh) {
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NT; ++ni)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[mi][ni][j] += ep[(wm * WM + mi * 16 + fg * 4 + j) * LDP + wn * WN + ni * 16 + fr];
    }
    __syncthreads();
  }
  // phase 1 writes alpha * acc (GEGLU: the combined h * gelu(g), bias hoisted); phase 2 (whole-row, 8 columns
  // per thread) adds bias / row-group bias, applies the activation and the residual with 16-B vector loads
  // issued together -- no per-element branches or dependent loads (they serialise a 1-WG/CU launch).
  const float* __restrict__ bias = p.bias ? p.bias + bsn : nullptr;
  const float* __restrict__ rbias = p.rowbias;
  const int act = p.act;
  if (lnf) {  // (mean, rstd) per row from the partials, fp64 fold in a fixed order
    if (tid < BM) {
      double s = 0.0, q = 0.0;
#pragma unroll
      for (int i = 0; i < (LNF ? 4 : 1); ++i)
        if (2 * i < lnP) {
          s += lnv4[i][0];
          q += lnv4[i][1];
          s += lnv4[i][2];
          q += lnv4[i][3];
        }
      const double ik = 1.0 / 1024.0 * (1024.0f / (float)K);  // 1/K without an fp64 divide
      const double mu = s * ik;
      double var = q * ik - mu * mu;
      if (var < 0.0) var = 0.0;
      ln_tab[tid] = make_float2((float)mu, rsqrtf((float)var + p.ln_eps));
    }
    __syncthreads();
  }
  if (!kh) {
    if (GEGLU) {
      float gbh[NT / 2 > 0 ? NT / 2 : 1], gbg[NT / 2 > 0 ? NT / 2 : 1];
      float lch[NT / 2 > 0 ? NT / 2 : 1], lcg[NT / 2 > 0 ? NT / 2 : 1];
#pragma unroll
      for (int q = 0; q < NT / 2; ++q) {
        const int np = min(n0 + wn * WN + 2 * q * 16 + fr, N - 17);
        gbh[q] = bias ? bias[np] : 0.f;
        gbg[q] = bias ? bias[np + 16] : 0.f;
        lch[q] = lnf ? ln_cs[min(wn * WN + 2 * q * 16 + fr, BN - 17)] : 0.f;
        lcg[q] = lnf ? ln_cs[min(wn * WN + 2 * q * 16 + fr, BN - 17) + 16] : 0.f;
      }
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        float2 st[LNF ? 4 : 1];  // read ahead of the staging stores (same LDS object)
        if (LNF) {
#pragma unroll
          for (int j = 0; j < (LNF ? 4 : 1); ++j) st[j] = ln_tab[wm * WM + mi * 16 + fg * 4 + j];
        }
#pragma unroll
        for (int ni = 0; ni + 1 < NT; ni += 2) {
          const int col = (wn * WN) / 2 + (ni / 2) * 16 + fr;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = wm * WM + mi * 16 + fg * 4 + j;
            float h = acc[mi][ni][j] * alpha, g = acc[mi][ni + 1][j] * alpha;
            if (LNF) {
              const float2 t = st[j & (LNF ? 3 : 0)];
              h = t.y * (h - t.x * lch[ni / 2]);
              g = t.y * (g - t.x * lcg[ni / 2]);
            }
            h += gbh[ni / 2];
            g += gbg[ni / 2];
            ep[row * LDE + col] = h * gelu_f(g);
          }
        }
      }
    } else {
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NT; ++ni) {
          const int col = wn * WN + ni * 16 + fr;
#pragma unroll
          for (int j = 0; j < 4; ++j) ep[(wm * WM + mi * 16 + fg * 4 + j) * LDE + col] = acc[mi][ni][j] * alpha;
        }
    }
  }  // !kh
  __syncthreads();

  // ---- phase 2
  TO* __restrict__ C = (TO*)p.C + zi * p.strideC + zo * p.strideC_o;
  const TO* __restrict__ R = p.residual ? (const TO*)p.residual + bz * p.strideR : nullptr;
  const int Nout = GEGLU ? N / 2 : N;
  const int n0o = GEGLU ? n0 / 2 : n0;
  const bool vec = (Nout % 8 == 0) && (p.ldc % 8 == 0) && ((((unsigned long long)C) & 15) == 0) &&
                   (!R || ((p.ldr % 8 == 0) && ((((unsigned long long)R) & 15) == 0))) &&
                   (GEGLU || !bias || ((((unsigned long long)bias) & 15) == 0)) &&
                   (GEGLU || !rbias || ((p.rowbias_ld % 4 == 0) && ((((unsigned long long)rbias) & 15) == 0)));
  constexpr int VPR = BNO / 8;
  constexpr int TOT = BM * VPR;
  constexpr int ITER = (TOT + NTHR - 1) / NTHR;
  typedef __attribute__((ext_vector_type(8))) TO TO8;
  const bool lno = LNP && p.ln_out != nullptr;
  float2* lnslot = (float2*)(smem + LNS_OFF);
  const bool gn = GN4 && p.gn_part != nullptr;  // the host asks only for interior, group-aligned tiles
  const int gcpg = gn ? N / p.gn_groups : 8;
  const int gsplit = (((tid % VPR) * 8) / gcpg + 1) * gcpg - (tid % VPR) * 8;
  GnTile gna;
  // vector epilogue for every tile with whole rows; a tile that runs past N (Nout % 8 == 0 under vec) skips its
  // 8-column chunks beyond N (the BSRNet dense convs: N = 32 on 64-column tiles)
  const bool full_n = n0o + BNO <= Nout;
  if (vec && m0 + BM <= M) {
    float v[ITER][8], bv[ITER][8], rv[ITER][8];
    TO8 res[ITER];
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int e = tid + it * NTHR;
      if ((TOT % NTHR == 0 || e < TOT) && (full_n || n0o + (e - (e / VPR) * VPR) * 8 < Nout)) {
        const int r = e / VPR, cv = e - (e / VPR) * VPR;
        const int m = m0 + r, n = n0o + cv * 8;
        *(f32x4*)&v[it][0] = *(const f32x4*)(ep + r * LDE + cv * 8);
        *(f32x4*)&v[it][4] = *(const f32x4*)(ep + r * LDE + cv * 8 + 4);
        if (!GEGLU && bias) {
          *(f32x4*)&bv[it][0] = *(const f32x4*)(bias + n);
          *(f32x4*)&bv[it][4] = *(const f32x4*)(bias + n + 4);
        }
        if (!GEGLU && rbias) {
          const float* rb = rbias + (long long)(m / p.rows_per_group) * p.rowbias_ld + n;
          *(f32x4*)&rv[it][0] = *(const f32x4*)rb;
          *(f32x4*)&rv[it][4] = *(const f32x4*)(rb + 4);
        }
        if (R) {
          if (PREF && pf) res[it] = __builtin_bit_cast(TO8, res_pf[PREF ? it : 0]);
          else res[it] = *(const TO8*)(R + (long long)m * p.ldr + n);
        }
      }
    }
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int e = tid + it * NTHR;
      if ((TOT % NTHR == 0 || e < TOT) && (full_n || n0o + (e - (e / VPR) * VPR) * 8 < Nout)) {
        const int r = e / VPR, cv = e - (e / VPR) * VPR;
        const int m = m0 + r, n = n0o + cv * 8;
        if (!GEGLU) {
          if (lnf) {
            const float2 st = ln_tab[r];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[it][i] = st.y * (v[it][i] - st.x * ln_cs[cv * 8 + i]);
          }
          if (bias) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[it][i] += bv[it][i];
          }
          if (rbias) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[it][i] += rv[it][i];
          }
          if (act == FD_ACT_SILU) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[it][i] = silu_f(v[it][i]);
          } else if (act == FD_ACT_GELU) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[it][i] = gelu_f(v[it][i]);
          } else if (act == FD_ACT_QUICKGELU) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[it][i] = quickgelu_f(v[it][i]);
          } else if (act == FD_ACT_LRELU) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[it][i] = lrelu_f(v[it][i]);
          }
        }
        if (R) {
#pragma unroll
          for (int i = 0; i < 8; ++i) v[it][i] += (float)res[it][i];
        }
        TO8 o;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (TO)v[it][i];
        st_out16((TO8*)(C + (long long)m * p.ldc + n), o);
        if (GN4 && gn) gna.add(o, gsplit);
        if (lno) {  // statistics of the values as stored (what the consumer GEMM multiplies)
          float s = 0.f, q = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float f = (float)o[i];
            s += f;
            q += f * f;
          }
          lnslot[r * VPR + cv] = make_float2(s, q);
        }
      }
    }
  } else {  // edge tiles / unaligned operands: scalar, bounds-checked
    for (int e = tid; e < TOT; e += NTHR) {
      const int r = e / VPR, cv = e - (e / VPR) * VPR;
      const int m = m0 + r, n = n0o + cv * 8;
      float s = 0.f, q = 0.f;
      if (m < M && n < Nout) {
        for (int i = 0; i < 8 && n + i < Nout; ++i) {
          float x = ep[r * LDE + cv * 8 + i];
          if (!GEGLU) {
            if (lnf) {
              const float2 st = ln_tab[r];
              x = st.y * (x - st.x * ln_cs[cv * 8 + i]);
            }
            if (bias) x += bias[n + i];
            if (rbias) x += rbias[(long long)(m / p.rows_per_group) * p.rowbias_ld + n + i];
            x = act_f(x, act);
          }
          if (R) x += (float)R[(long long)m * p.ldr + n + i];
          const TO o = (TO)x;
          C[(long long)m * p.ldc + n + i] = o;
          s += (float)o;
          q += (float)o * (float)o;
        }
      }
      if (lno) lnslot[r * VPR + cv] = make_float2(s, q);
    }
  }
  if (lno) {  // per-row partial over this tile's 160 columns, slots summed in column order
    __syncthreads();
    if (tid < BM && m0 + tid < M) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int c = 0; c < VPR; ++c) {
        const float2 v2 = lnslot[tid * VPR + c];
        s += v2.x;
        q += v2.y;
      }
      ((float2*)p.ln_out)[(long long)(m0 + tid) * (N / 160) + n0 / 160] = make_float2(s, q);
    }
  }
  if constexpr (GN4) {
    if (gn) gn_tile_write(gna, (float2*)(smem + LNC_OFF + LNC), tid, NTHR, VPR, gcpg, BNO, n0o, m0, p, 128);
  }
}

template <typename T, int BM, int BN, int WM, int WN, int NS, typename TO, int KS = 1>
static int launch_cfg(const fd_gemm_params* p, hipStream_t s, int swz) {
  const int tiles = ((p->M + BM - 1) / BM) * ((p->N + BN - 1) / BN);
  dim3 grid(tiles, 1, p->batch > 0 ? p->batch : 1), block(256 * KS);
  if (p->conv) {
    if (p->act == FD_ACT_GEGLU) return FD_ERR_ARG;
    hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WM, WN, NS, true, false, TO, KS>), grid, block, 0, s, *p, swz);
  } else if (p->act == FD_ACT_GEGLU) {
    if constexpr (WN % 32 == 0) {
      if (p->ln_in)
        hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WM, WN, NS, false, true, TO, KS, true>), grid, block, 0, s, *p,
                           swz);
      else
        hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WM, WN, NS, false, true, TO, KS>), grid, block, 0, s, *p, swz);
    } else {
      return FD_ERR_ARG;
    }
  } else if (p->ln_in) {
    hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WM, WN, NS, false, false, TO, KS, true>), grid, block, 0, s, *p, swz);
  } else {
    hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WM, WN, NS, false, false, TO, KS>), grid, block, 0, s, *p, swz);
  }
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// Tile choice: cost ~ ceil(tiles / (256 CUs x resident WGs per CU)) x per-tile time; a smaller tile is
// worth it only when it removes a partial wave.  Relative per-tile efficiencies are estimates.
// (256-row tiles live in gemm8.hip: 8 waves, register-double-buffered fragments, split-K.)
enum { CFG_128x128, CFG_64x160, CFG_128x64, CFG_64x64, CFG_AUTO_COUNT, CFG_COUNT = CFG_AUTO_COUNT };
static const int CFG_BM[] = {128, 64, 128, 64}, CFG_BN[] = {128, 160, 64, 64};

static int pick_cfg(const fd_gemm_params* p) {
  const long long b = p->batch > 0 ? p->batch : 1;
  const double eff[] = {1.00, 0.92, 0.85, 0.60};
  int best = CFG_128x128;
  double bestc = 1e30;
  for (int c = 0; c < CFG_AUTO_COUNT; ++c) {
    if (p->act == FD_ACT_GEGLU && c == CFG_64x160) continue;
    const long long tiles = b * ((p->M + CFG_BM[c] - 1) / CFG_BM[c]) * ((p->N + CFG_BN[c] - 1) / CFG_BN[c]);
    const long long waves = (tiles + 255) / 256;
    const double cost = waves * (double)(CFG_BM[c] * CFG_BN[c]) / eff[c];
    if (cost < bestc - 1e-9) { bestc = cost; best = c; }
  }
  return best;
}

// Tuning overrides (knob table, benchmarks only): FD_GEMM_CFG=<0..3> forces the tile, FD_GEMM_SWZ=<0|1> the tile
// order.  Ring depth: 4 stages (one workgroup per CU) when one round of tiles covers the launch and K >= 512, else 2;
// each K step split over two wave groups (KS = 2, 8 waves).  (Round 6: the knob-only 3-stage ring and KS = 1 forms,
// measured slower -- profiles/r04zl_gemm_ns_ab.txt, scripts/gemm_ks.sh history -- were removed.)

template <typename T, typename TO, int BM, int BN, int WM, int WN>
static int dispatch_ns(const fd_gemm_params* p, hipStream_t s, int ns, int swz) {
  constexpr int STAGE = (BM + BN) * 128;
  constexpr bool NS4 = 4 * STAGE <= 160 * 1024;
  if constexpr (std::is_same<T, TO>::value) {
    if constexpr (NS4) {
      if (ns == 4) return launch_cfg<T, BM, BN, WM, WN, 4, TO, 2>(p, s, swz);
    }
    return launch_cfg<T, BM, BN, WM, WN, 2, TO, 2>(p, s, swz);
  } else {
    return launch_cfg<T, BM, BN, WM, WN, 2, TO>(p, s, swz);
  }
}

// GroupNorm statistics from the 128 x 128 tiles (GN4): interior, image-aligned, group-aligned tiles only
static bool gn_ok4(const fd_gemm_params* p, int cfg) {
  if (!p->gn_part || cfg != CFG_128x128 || p->act == FD_ACT_GEGLU || p->ln_in || p->ln_out || p->batch > 1)
    return false;
  if (p->gn_groups <= 0 || p->gn_hw <= 0 || p->N % p->gn_groups) return false;
  const int cpg = p->N / p->gn_groups;
  if (cpg < 4 || 128 % cpg || p->N % 128 || p->M % 128 || p->gn_hw % 128 || p->M % p->gn_hw) return false;
  const unsigned long long al = (unsigned long long)p->C | (p->residual ? (unsigned long long)p->residual : 0) |
                                (p->bias ? (unsigned long long)p->bias : 0) | (p->rowbias ? (unsigned long long)p->rowbias : 0);
  return (al & 15) == 0 && p->ldc % 8 == 0 && (!p->residual || p->ldr % 8 == 0) &&
         (!p->rowbias || p->rowbias_ld % 4 == 0);
}

// Tile-row group height of the XCD-chunked walk (tile_coords): the ~tiles/8 tiles of one XCD chunk should touch as
// few A rows and B columns as possible (each XCD's L2 fetches its chunk's panels once).  Counted exactly on the
// first chunk's tiles for every power-of-two height; ties keep the smaller height.
static int plan_group_m(long long tiles_total, int tiles_m, int tiles_n, int bm, int bn) {
  if (!fd_knob(FDK_GEMM_GMP)) return 4;
  const int per_xcd = (int)((tiles_total + 7) / 8);
  if (per_xcd > 4096) return 4;
  int best = 4;
  long long bestc = -1;
  for (int g = 1; g <= tiles_m && g <= 64; g *= 2) {
    // rows / columns touched by pids [0, per_xcd) under tile_coords (the remap is bijective and chunk-contiguous)
    const int rows_seen = per_xcd >= g * tiles_n ? g * (int)((per_xcd + g * tiles_n - 1) / (g * tiles_n))
                                                 : g;
    const int cols_seen = per_xcd >= g * tiles_n ? tiles_n : (per_xcd + g - 1) / g;
    const long long c = (long long)(rows_seen < tiles_m ? rows_seen : tiles_m) * bm +
                        (long long)(cols_seen < tiles_n ? cols_seen : tiles_n) * bn;
    if (bestc < 0 || c < bestc) {
      bestc = c;
      best = g;
    }
  }
  return best;
}

template <typename T, typename TO>
static int dispatch_tiles(fd_gemm_params* p0, hipStream_t s) {
  const int g_cfg = fd_knob(FDK_GEMM_CFG);
  const int g_swz = fd_knob(FDK_GEMM_SWZ) | (fd_knob(FDK_GEMM_MODE) << 4);
  int cfg = g_cfg >= 0 && g_cfg < CFG_COUNT ? g_cfg : pick_cfg(p0);
  if (p0->ln_out) cfg = CFG_64x160;  // LN-fold producer: partials per 160 columns, whatever M (batch-invariant)
  if (p0->act == FD_ACT_GEGLU && cfg == CFG_64x160) cfg = CFG_128x128;
  fd_gemm_params q = *p0;  // the kernel's copy: gn_part kept only where the 128 x 128 tiles write the statistics
  if (!gn_ok4(p0, cfg)) q.gn_part = nullptr;
  const fd_gemm_params* p = &q;
  // ring depth: 4 stages (1 WG/CU) pays only on long K when one wave of tiles covers the launch; 2 stages
  // (2-3 co-resident WGs/CU) otherwise (scripts/gemm_sweep.py + in-situ traces)
  const long long tiles = (long long)(p->batch > 0 ? p->batch : 1) * ((p->M + CFG_BM[cfg] - 1) / CFG_BM[cfg]) *
                          ((p->N + CFG_BN[cfg] - 1) / CFG_BN[cfg]);
  // KS = 2 (8 waves, intra-WG split of each K step) measured >= KS = 1 on every UNet shape
  // (scripts/gemm_ks.sh: 2048x1280x5120 60 -> 42 us); the 4-deep ring pays whenever one wave of tiles
  // covers the launch (one WG per CU either way).
  const int ns = (tiles <= 256 && p->K >= 512) ? 4 : 2;
  const int tm_ = (p->M + CFG_BM[cfg] - 1) / CFG_BM[cfg], tn_ = (p->N + CFG_BN[cfg] - 1) / CFG_BN[cfg];
  const int swz = g_swz | (plan_group_m(tm_ * (long long)tn_, tm_, tn_, CFG_BM[cfg], CFG_BN[cfg]) << 8);
  int rc;
  switch (cfg) {
    case CFG_128x128: rc = dispatch_ns<T, TO, 128, 128, 64, 64>(p, s, ns, swz); break;
    case CFG_64x160: rc = dispatch_ns<T, TO, 64, 160, 32, 80>(p, s, ns, swz); break;
    case CFG_128x64: rc = dispatch_ns<T, TO, 128, 64, 64, 32>(p, s, ns, swz); break;
    default: rc = dispatch_ns<T, TO, 64, 64, 32, 32>(p, s, ns, swz);
  }
  if (rc == FD_OK && q.gn_part) p0->gn_done = 128;
  return rc;
}

// ------------------------------------------------------------------------------------------------ M <= 4
// Rows-of-a-few GEMM (the UNet's time / add-embedding MLPs and the per-resnet time_emb_proj at M = CFG rows = 2 per
// TLC tile, the text projection): a weight-streaming GEMV.  One wave per output column n streams W[n][0..K) in 16-B
// vectors (every lane a contiguous run of 8 k), multiplies by the rows of A four at a time in fp32, wave-reduces,
// and runs the fused epilogue (alpha, bias, activation, residual).  Chosen by the per-tile row count (m_ref <= 4),
// so a forward batching n tiles (M = 2n rows) takes the same kernel, and every row is summed in the same order
// whatever M is: batching stays bitwise.  The 64-row MFMA tile it replaces wasted 62 of 64 rows and covered
// N = 1280 with 20 workgroups (~18 us per launch for 3 MB of weights).
template <typename T, typename TO>
__global__ void __launch_bounds__(256) gemv_rows_kernel(const fd_gemm_params p) {
  typedef typename VecT<T>::v8 V8;
  constexpr int MR = 4;
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= p.N) return;
  const T* __restrict__ A = (const T*)p.A;
  const T* __restrict__ W = (const T*)p.B + (long long)n * p.ldb;
  const int nv = p.K / 8;
  for (int mb = 0; mb < p.M; mb += MR) {
    float acc[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) acc[m] = 0.f;
    for (int v = lane; v < nv; v += 64) {
      const V8 w = *(const V8*)(W + v * 8);
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        if (mb + m < p.M) {
          const V8 a = *(const V8*)(A + (long long)(mb + m) * p.lda + v * 8);
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[m] += (float)a[i] * (float)w[i];
        }
      }
    }
#pragma unroll
    for (int m = 0; m < MR; ++m) acc[m] = wave_sum(acc[m]);
    const int row = mb + lane;
    if (lane < MR && row < p.M) {
      float x = 0.f;
#pragma unroll
      for (int m = 0; m < MR; ++m)
        if (m == lane) x = acc[m];
      x *= p.alpha;
      if (p.bias) x += p.bias[n];
      x = act_f(x, p.act);
      if (p.residual) x += (float)((const TO*)p.residual)[(long long)row * p.ldr + n];
      ((TO*)p.C)[(long long)row * p.ldc + n] = (TO)x;
    }
  }
}

// Returns 1 when the GEMV took the launch, 0 when it does not apply.
template <typename T, typename TO>
static int try_gemv_rows(const fd_gemm_params* p, hipStream_t s) {
  const int on = fd_knob(FDK_GEMV);
  const int m_ref = p->m_ref > 0 ? p->m_ref : p->M;
  if (!on || m_ref > 4 || p->M > 4096 || p->conv || (p->batch > 1) || p->rowbias || p->ln_in || p->ln_out ||
      p->gn_part || p->act == FD_ACT_GEGLU || p->A2 || (p->K % 8) || (p->lda % 8) || (p->ldb % 8))
    return 0;
  if ((((unsigned long long)p->A) | ((unsigned long long)p->B)) & 15) return 0;
  dim3 grid((p->N + 3) / 4), block(256);
  hipLaunchKernelGGL((gemv_rows_kernel<T, TO>), grid, block, 0, s, *p);
  return hipGetLastError() == hipSuccess ? 1 : -1;
}

extern "C" int fd_gemm8_try(fd_gemm_params* p, void* stream);    // gemm8.hip
extern "C" int fd_gemm256_try(fd_gemm_params* p, void* stream);  // gemm256.hip

extern "C" int fd_gemm(fd_gemm_params* p, void* stream) {
  if (!p || !p->A || !p->B || !p->C) return FD_ERR_ARG;
  p->gn_done = 0;  // rows per partial block (256 / 128) when a kernel wrote the GroupNorm statistics (gn_part)
  if (p->M <= 0 || p->N <= 0 || p->K <= 0 || (p->K % 64) != 0) return FD_ERR_SHAPE;
  if (p->act == FD_ACT_GEGLU && (p->N % 32) != 0) return FD_ERR_SHAPE;
  if (p->rowbias && p->rows_per_group <= 0) return FD_ERR_ARG;
  if (p->rowbias && p->rowbias_rows < ((long long)p->M + p->rows_per_group - 1) / p->rows_per_group)
    return FD_ERR_SHAPE;  // the table must cover every row group of the launch (include/faithdiff_hip.h)
  if (p->residual) {
    if (p->ldr <= 0) return FD_ERR_SHAPE;
    const long long need = (long long)p->M + (p->batch > 1 ? (long long)(p->batch - 1) * ((p->strideR + p->ldr - 1) /
                                                                                            p->ldr) : 0);
    if (p->residual_rows < need) return FD_ERR_SHAPE;
  }
  if (p->batch_inner > 1 && (p->residual || p->rowbias || p->ln_out || p->ln_in || p->gn_part)) return FD_ERR_SHAPE;
  if (p->conv) {
    if (p->Cin % 64 || (p->C1 > 0 && (p->C1 % 64 || !p->A2)) || p->K != (p->up_phase ? 4 : 9) * p->Cin)
      return FD_ERR_SHAPE;
    if (p->M != p->nimg * p->Hout * p->Wout) return FD_ERR_SHAPE;
    if (p->stride != 1 && p->stride != 2) return FD_ERR_SHAPE;
    if (p->upsample && (p->stride != 1 || p->pad != 1 || p->Hout < p->Hin || p->Wout < p->Win)) return FD_ERR_SHAPE;
  }
  if (p->ln_out && (p->N % 160 || p->act == FD_ACT_GEGLU || p->batch > 1 || p->conv ||
                    (p->out_dtype != FD_BF16 && p->out_dtype != FD_F16)))
    return FD_ERR_SHAPE;
  if (p->ln_in && (p->K % 320 || p->K > 1280 || p->batch > 1 || p->conv || !p->ln_c)) return FD_ERR_SHAPE;
  const bool sm = p->act == FD_ACT_SOFTMAX;
  if (sm && (p->N % 160 || p->sm_group != 80 || p->sm_len < 1 || p->sm_len > 80 || p->residual || p->rowbias ||
             p->conv || p->batch > 1 || p->ln_out || p->gn_part || p->dtype == FD_F32 ||
             (p->out_dtype != FD_BF16 && p->out_dtype != FD_F16)))
    return FD_ERR_SHAPE;
  const bool bsel = p->bsel_rows > 0;
  if (bsel && (p->bsel_rows % 256 || p->batch > 1 || p->conv || p->bsel_mod < 0)) return FD_ERR_SHAPE;
  if (p->batch_inner > 1 && (p->batch <= 1 || p->batch % p->batch_inner || bsel)) return FD_ERR_SHAPE;
  if (sm || bsel) {  // the eight-wave kernels (softmax: only there), else the 4-wave kernel (bsel)
    const int r8 = fd_gemm8_try(p, stream);
    if (r8 < 0) return r8;
    if (r8 == 1) return FD_OK;
    if (sm) return FD_ERR_SHAPE;
    FD_DISPATCH_T(p->dtype, FD_DISPATCH_O(p->out_dtype, return dispatch_tiles<T, TO>(p, (hipStream_t)stream)));
  }
  if (p->conv) {  // 3x3 stride-1 convs: the halo-staged kernel where it applies (the only one taking gi_affine)
    const int rh = fd_conv_halo_try(p, stream);
    if (rh < 0) return rh;
    if (rh == 1) return FD_OK;
  } else if (p->gi_affine) {
    return FD_ERR_ARG;
  }
  if (!p->ln_out) {
    const int r256 = fd_gemm256_try(p, stream);  // large-M, N % 256 == 0: 256 x 256 tiles
    if (r256 < 0) return r256;
    if (r256 == 1) return FD_OK;
  }
  {
    const int r8 = fd_gemm8_try(p, stream);  // LN-fold producers only on its 160-column tiles (plan8)
    if (r8 < 0) return r8;
    if (r8 == 1) return FD_OK;
  }
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_T(p->dtype, FD_DISPATCH_O(p->out_dtype, {
    const int rv = try_gemv_rows<T, TO>(p, s);
    if (rv < 0) return FD_ERR_HIP;
    if (rv == 1) return FD_OK;
    return dispatch_tiles<T, TO>(p, s);
  }));
}
