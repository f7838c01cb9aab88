// Eight-wave, 256-row-tile MFMA GEMM / implicit-GEMM convolution for gfx950 with in-launch split-K.
//
// Why a second GEMM: at C2 (one 1024^2 tile, CFG pair) most of the UNet's FLOPs sit in GEMMs with
// M = 2048 (the 32^2 level: 2 x 1024 pixels) whose 128^2-tile launches cover only 64-160 of the 256 CUs,
// and each CU's operand stream from L2 (~70 GB/s per CU, MI355X_MICROARCH.md "Indexed rows") -- not the
// MFMA pipe -- bounds them.  This kernel raises the FLOP per operand byte (256 x 160 tile: 98 flop/B
// vs 64 for 128^2) and restores the CU count by splitting K across workgroups (S = 1..8), combining the
// fp32 partial tiles inside the same launch (last-arriving workgroup of a tile sums the S slabs in split
// order -- bitwise independent of arrival order -- and runs the fused epilogue).  S is chosen from
// (m_ref, N, K), where m_ref is the caller's per-tile row count, so batching TLC tiles into one forward
// does not change any output bit.
//
// Structure (cdna_hip_programming.md section 5): 512 threads = 8 waves (WAVES_M x WAVES_N), each wave a
// WM x WN sub-tile of v_mfma_f32_16x16x32; both operands K-contiguous ([rows][K]) staged global -> LDS by
// global_load_lds_dwordx4 into a 3-deep ring (two stages in flight across each barrier: counted
// s_waitcnt vmcnt, raw s_barrier); fragments are register double-buffered by K half, so the LDS reads
// of half h+1 overlap the MFMAs of half h, and the one barrier per 64-deep K step sits between the two
// MFMA halves.  XOR-swizzled 128-B LDS rows (source-side swizzle, rule 21).  Conv: im2col gather from
// NHWC with out-of-image taps on a zero page; nearest upsample and two-source skip concat folded in.
#include <stdlib.h>

#include "fd_common.h"

__device__ __attribute__((aligned(256))) unsigned char g_zero_page8[256];

typedef __attribute__((ext_vector_type(8))) int i32x8;

// Operand fragment of one MFMA: 8 x 16-bit (16x16x32) or, for e4m3 operands (T = uint8_t), 32 bytes (16x16x128)
// e4m3 operand tags: uint8_t = per-row scaled (fd_gemm_e4m3), mx8_t = OCP MX block-scaled (fd_gemm_mxe4m3)
struct mx8_t {
  uint8_t v;
};
template <typename T> struct Frag8 { typedef typename VecT<T>::v8 type; };
template <> struct Frag8<uint8_t> { typedef i32x8 type; };
template <> struct Frag8<mx8_t> { typedef i32x8 type; };
// e4m3 side arguments: per-row A scales (uint8_t operands), A block scales (mx8_t), output block scales (TO = uint8_t)
struct f8_args {
  const float* a_scale;
  const uint8_t* a_bs;
  long long a_bs_ld;
  uint8_t* o_bs;
  long long o_bs_ld;
};

__device__ __forceinline__ f32x4 mfma8(bf16x8 a, bf16x8 b, f32x4 c) { return mfma16x16x32(a, b, c); }
__device__ __forceinline__ f32x4 mfma8(f16x8 a, f16x8 b, f32x4 c) { return mfma16x16x32(a, b, c); }
// OCP e4m3 x e4m3 on the block-scaled MFMA with unit E8M0 scales (127 = 2^0); the per-row activation scale is
// applied in the epilogue (as gemm_fp8.hip's kernels, so both give the same bits)
__device__ __forceinline__ f32x4 mfma8(i32x8 a, i32x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}
// MX A operand: this lane's E8M0 byte (its row, its 32-element block) as the A scale; W unscaled (127)
__device__ __forceinline__ f32x4 mfma8s(i32x8 a, i32x8 b, f32x4 c, int sa) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, 127);
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

#ifndef FD_GEMM8_SCHED
#define FD_GEMM8_SCHED 1
#endif
#ifndef FD_GEMM8_DIAG
#define FD_GEMM8_DIAG 0
#endif
// timing build only (wrong results): 1 = the GEGLU epilogue multiplies by g instead of gelu(g)
#ifndef FD_GEGLU_DIAG
#define FD_GEGLU_DIAG 0
#endif

// BM x BN tile over NW waves (WAVES_M x WAVES_N).  Instances: 256 x 128 over 8 waves (the split-K kernel
// above) and 64 x 160 over 4 waves (one wave per SIMD, 32 x 80 each: the M = 2048 projections' 256-tile
// launches, where the previous 4-wave kernel split each K step over two waves and exposed the LDS-read
// latency in front of every MFMA group).
//
// T = uint8_t: OCP e4m3 operands (fd_gemm_e4m3, the use_fp8 model's transformer Linears).  A 128-byte K step then
// holds 128 elements and takes ONE v_mfma_scale_f32_16x16x128_f8f6f4 per 16x16 block (the cycles of the two
// 16x16x32 bf16 MFMAs it replaces, twice the FLOP); the two halves of a step split the wave's column blocks
// (half 0: ni < NH, half 1: the rest) instead of K.  a_scale[m] * alpha (= w_scale) replaces alpha per row.
// T = mx8_t: A carries E8M0 block scales ([M][K / 32] bytes): each stage also DMAs the tile's BM x 4 scale bytes
// (one dword per row) into LDS, and every MFMA takes its lane's byte as the A scale.  TO = uint8_t: the output is
// written as MX e4m3 (+ block scales f8.o_bs), each 32-column block's amax reduced over its 4 epilogue threads.
// Split-K hand-off health (fd_splitk_health): pairwise waits that timed out in this library's gemm8 launches, and
// a test hook that makes the publishing split skip its flag (forces the timeout path).
__device__ unsigned g_g8_sk_timeouts;
__device__ unsigned g_g8_sk_drop;

template <typename T, int BM, int BN, int NW, int WAVES_M, int NS, bool CONV, bool GEGLU, typename TO,
          bool LNF = false>
__global__ void __launch_bounds__(64 * NW) gemm8_kernel(const fd_gemm_params p, const int S, const int gm_mode,
                                                        float* __restrict__ slabs, unsigned* __restrict__ counters,
                                                        const f8_args f8) {
  typedef typename Frag8<T>::type V8;
  constexpr bool F8 = sizeof(T) == 1;
  constexpr bool MXI = __is_same(T, mx8_t);
  constexpr bool MXO = __is_same(TO, uint8_t);
  static_assert(!MXO || (F8 && !LNF && !CONV), "MX output from the e4m3 kernels only");
  static_assert(!F8 || (!CONV && !LNF), "e4m3: plain GEMM only");
  constexpr int KS = F8 ? 128 : 64;  // elements per 128-byte K step
  constexpr int CH = 16 / (int)sizeof(T);  // elements per 16-byte chunk
  constexpr bool SCHED = FD_GEMM8_SCHED;
  constexpr int NTHR = 64 * NW;
  static_assert(NS >= 3 && NS <= 5, "ring depth");
  constexpr int WAVES_N = NW / WAVES_M;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int MT = WM / 16, NT = WN / 16;
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  constexpr int A_I = BM / (8 * NW);       // A loads per wave per stage (8 rows x 128 B each)
  constexpr int B_TOT = BN / 8;            // B loads per stage over the NW waves
  constexpr int B_I = (B_TOT + NW - 1) / NW;  // ... at most this many per wave
  constexpr int B_LO = B_TOT / NW;         // waves >= B_TOT % NW issue only this many
  static_assert(A_I * 8 * NW == BM, "A rows per stage");
  // MX: every wave DMAs one dword (the 4 block scales of a K step) for each of 64 consecutive rows starting at its
  // RPW-row slice, all lanes active (an exec-masked LDS-DMA makes hipcc branch around it inside the main loop); the
  // slices of neighbouring waves overlap and write identical bytes.  Region per stage: (NW - 1) * RPW + 64 rows.
  constexpr int RPW = BM / NW;
  constexpr int SCR = ((NW - 1) * RPW + 64) * 4;
  constexpr int PER_HI = A_I + B_I + (MXI ? 1 : 0), PER_LO = A_I + B_LO + (MXI ? 1 : 0);
  constexpr int BNO = GEGLU ? BN / 2 : BN;
  constexpr int LDE = BNO + 4;
  // epilogue staged fp32 [EROWS][BNO+4] in the ring's LDS: the whole tile when it fits, else 128-row halves
  constexpr int EROWS = (BM * LDE * 4 <= NS * STAGE) ? BM : 128;
  constexpr int EPB = EROWS * LDE * 4;
  // LN-fold consumer (LNF): (mean, rstd) of the tile's rows and ln_c of its columns after the ring / staging
  // area, in the same LDS object (a second __shared__ array makes hipcc assume ds_reads may alias the
  // LDS-DMA targets and drain vmcnt(0) in front of them)
  constexpr int LNC_OFF = (NS * STAGE > EPB) ? NS * STAGE : EPB;
  // e4m3: the tile's per-row scales a_scale[m] * alpha (fp32) after that
  constexpr int SC_OFF = LNC_OFF + (LNF ? BM * 8 + BN * 4 : 0);
  constexpr int SCL_OFF = SC_OFF + (F8 && !MXI ? BM * 4 : 0);
  // MX: the ring's block-scale dwords (NS stages x BM rows) after that
  constexpr int SMX_END = SCL_OFF + (MXI ? NS * SCR : 0);
  // softmax epilogue (fd_gemm_params.sm_*, the cross-attention score GEMM): 160-column 16-bit plain tiles; the
  // tile's bias columns in LDS after that
  constexpr bool SMK = BN == 160 && !GEGLU && !CONV && !F8;
  constexpr int SMB_OFF = SMX_END;
  constexpr int SMEM = SMX_END + (SMK ? BN * 4 : 0);
  static_assert(SMEM <= 163840, "LDS");
  static_assert(!GEGLU || (WN % 32 == 0), "GEGLU pairs must not straddle waves");
  // GroupNorm output statistics (fd_gemm_params.gn_part): one 8-column chunk per thread, reduction scratch after the
  // epilogue staging
  constexpr int RED_OFF = ((EPB + 15) / 16) * 16;
  constexpr bool GN_OK = !GEGLU && !LNF && BM == 256 && (NTHR % (BNO / 8)) == 0 && RED_OFF + 16 * NTHR <= SMEM;
  // the 160-column tiles (the UNet's 10 / 20 / 40-channel groups divide 160, not 128): a thread's chunk changes
  // from row pass to row pass (NTHR % 20 != 0), so every chunk's two group sums go to an LDS slot per staged
  // half, then 32 threads per group fold them in a fixed order (fd_gemm_params.gn_part, same layout)
  constexpr bool GN160 = !GEGLU && !LNF && BM == 256 && BN == 160 && RED_OFF + EROWS * (BNO / 8) * 16 <= SMEM;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];
  float2* const ln_tab = (float2*)(smem + LNC_OFF);
  float* const ln_cs = (float*)(smem + LNC_OFF + BM * 8);
  float* const sc_tab = (float*)(smem + SC_OFF);
  float* const sm_bias = (float*)(smem + SMB_OFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WAVES_N, wn = w % WAVES_N;
  const int M = p.M, N = p.N, K = p.K;
  // diagnostic builds only (-DFD_GEMM8_DIAG=m; 0 in the product): 1 = no operand loads, 2 = no LDS reads /
  // MFMA, 4 = no epilogue stores.  Compile-time, so the product loop has no branches.
  constexpr int mode = FD_GEMM8_DIAG;
  const int group_m = gm_mode;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;

  // ---- block -> (tile, split): XCD-contiguous chunks (bijective remap), a tile's S splits adjacent
  // (same XCD: the reducer reads same-L2 slabs), tiles walked in groups of group_m tile rows.
  const int pid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = pid % S, tlin = pid / S;
  int tm, tn;
  {
    const int gsz_full = group_m * tiles_n;
    const int grp = tlin / gsz_full;
    const int first_m = grp * group_m;
    const int gsz = min(tiles_m - first_m, group_m);
    const int in_g = tlin - grp * gsz_full;
    tm = first_m + in_g % gsz;
    tn = in_g / gsz;
  }
  const int tile_id = tm * tiles_n + tn;
  const int m0 = tm * BM, n0 = tn * BN;
  // per-row-group B slot (bsel: each image row block multiplies its own prompt's matrices)
  const int bslot = p.bsel_rows > 0 ? (p.bsel_mod > 0 ? (m0 / p.bsel_rows) % p.bsel_mod : m0 / p.bsel_rows) : 0;
  const long long bsn = (long long)bslot * p.bsel_strideN;
  const bool sm = SMK && p.act == FD_ACT_SOFTMAX;
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
  float smbv = 0.f;  // softmax: this thread's bias column, staged in LDS with ln_cs
  if (SMK && sm && p.bias && tid < BN) smbv = p.bias[bsn + min(n0 + tid, p.N - 1)];
  float scv = 0.f;  // e4m3: this thread's row scale, requested ahead of the operand stages like the LN partials
  if (F8 && !MXI && tid < BM) scv = f8.a_scale[min(m0 + tid, M - 1)] * p.alpha;
  const int nk = K / KS;
  const int kb = (int)((long long)split * nk / S), ke = (int)((long long)(split + 1) * nk / S);
  const int nkl = ke - kb;

  const T* __restrict__ A = (const T*)p.A;
  const T* __restrict__ Bw = (const T*)p.B + bslot * p.bsel_strideB;
  const T* __restrict__ A2 = (const T*)p.A2;
  const int lrow = lane >> 3, slot = lane & 7;
  const bool hi = (B_TOT % NW == 0) || w < B_TOT % NW;  // this wave issues B_I (not B_LO) B loads

  // ---- per-lane load state (rows fixed over the K loop).  Conv: the output row; the im2col source pointers are
  // decoded once per tap in stage() (every Cin / 64 stages), not per stage
  const T* a_row[A_I];
  int a_m[A_I], a_chunk[A_I];
#pragma unroll
  for (int i = 0; i < A_I; ++i) {
    const int row = (w + NW * i) * 8 + lrow;
    const int m = m0 + row;
    const int mm = m < M ? m : M - 1;
    a_m[i] = m < M ? m : -1;
    a_chunk[i] = slot ^ ((row >> 1) & 7);
    a_row[i] = CONV ? nullptr : A + (long long)mm * p.lda + a_chunk[i] * CH;
  }
  const T* b_row[B_I];
#pragma unroll
  for (int i = 0; i < B_I; ++i) {
    const int row = (w + NW * i) * 8 + lrow;  // < BN for the loads this wave issues
    const int n = n0 + (row < BN ? row : 0);
    b_row[i] = Bw + (long long)(n < N ? n : N - 1) * p.ldb + (slot ^ ((row >> 1) & 7)) * CH;
  }
  const uint8_t* s_src = nullptr;  // MX: this lane's row of A block scales (row w * RPW + lane, clamped)
  if (MXI) s_src = f8.a_bs + (long long)min(m0 + w * RPW + lane, M - 1) * f8.a_bs_ld;
  const int Hl = p.upsample ? p.Hout : p.Hin, Wl = p.upsample ? p.Wout : p.Win;
  const bool up2 = p.upsample && Hl == 2 * p.Hin && Wl == 2 * p.Win;
  const int C1 = p.C1 > 0 ? p.C1 : p.Cin;

  int g_key = -1;        // conv: (tap, source) of g_base; stage() runs in K order within a split
  const T* g_base[A_I];  // per DMA row: this tap's source-pixel pointer (channel 0), nullptr = zero page
#pragma unroll
  for (int i = 0; i < A_I; ++i) g_base[i] = nullptr;
  auto stage = [&](int kt, int buf) {  // kt: global K step
    if (mode & 1) return;
    const int k0 = kt * KS;
    unsigned char* sa = smem + buf * STAGE;
    if (CONV) {
      const int tap = k0 / p.Cin;
      const int c0 = k0 - tap * p.Cin;
      const bool second = (A2 != nullptr) && (c0 >= C1);
      const int key = tap * 2 + (int)second;
      if (key != g_key) {  // uniform: the source pixels change only with the tap (and the concat source)
        g_key = key;
        const int ky = tap / 3, kx = tap - (tap / 3) * 3;
#pragma unroll
        for (int i = 0; i < A_I; ++i) {
          const int mm = a_m[i] < 0 ? 0 : a_m[i];
          const int hw = p.Hout * p.Wout;
          const int img = mm / hw;
          const int rem = mm - img * hw;
          const int oy = rem / p.Wout, ox = rem - (rem / p.Wout) * p.Wout;
          const int iy = oy * p.stride - p.pad + ky, ix = ox * p.stride - p.pad + kx;
          const bool ok = a_m[i] >= 0 && iy >= 0 && iy < Hl && ix >= 0 && ix < Wl;
          // exact x2 (every Upsample2D except diffusers' odd-size upsample_size path): a shift, not an integer
          // division
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
          const long long pix = ((long long)img * p.Hin + py) * p.Win + px;
          // pointer such that g_base + c0 addresses channel c0 of this tap's source pixel; nullptr = zero page
          g_base[i] = !ok ? nullptr
                          : second ? A2 + pix * (p.Cin - C1) - C1 + a_chunk[i] * 8 : A + pix * p.lda + a_chunk[i] * 8;
        }
      }
#pragma unroll
      for (int i = 0; i < A_I; ++i) {
        const void* s = g_base[i] ? (const void*)(g_base[i] + c0) : (const void*)g_zero_page8;
        __builtin_amdgcn_global_load_lds(s, LDS_PTR(sa + (w + NW * i) * 1024), 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_I; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(a_row[i] + k0), LDS_PTR(sa + (w + NW * i) * 1024), 16, 0, 0);
    }
    unsigned char* sb = sa + A_BYTES;
#pragma unroll
    for (int i = 0; i < B_I; ++i)
      if (i < B_LO || hi)
        __builtin_amdgcn_global_load_lds((const void*)(b_row[i] + k0), LDS_PTR(sb + (w + NW * i) * 1024), 16, 0, FD_WLD_AUX);
    if constexpr (MXI)  // the 4 block scales of this K step (128 elements = 4 blocks) of rows w * RPW .. + 63
      __builtin_amdgcn_global_load_lds((const void*)(s_src + kt * 4), LDS_PTR(smem + SCL_OFF + buf * SCR + w * RPW * 4),
                                       4, 0, 0);
  };
  // all but the youngest `ahead` stages of this wave's loads have landed
  auto wait_ahead = [&](int ahead) {  // ahead <= NS - 1 (the prologue); NS - 2 in the steady loop
    constexpr int P4 = NS >= 5 ? 4 : 0, P3 = NS >= 4 ? 3 : 0;
    if (NS >= 5 && ahead >= 4) {
      if (hi) vm_wait<P4 * PER_HI>(); else vm_wait<P4 * PER_LO>();
    } else if (NS >= 4 && ahead == 3) {
      if (hi) vm_wait<P3 * PER_HI>(); else vm_wait<P3 * PER_LO>();
    } else if (ahead == 2) {
      if (hi) vm_wait<2 * PER_HI>(); else vm_wait<2 * PER_LO>();
    } else if (ahead == 1) {
      if (hi) vm_wait<PER_HI>(); else vm_wait<PER_LO>();
    } else {
      vm_wait<0>();
    }
  };


  const int fr = lane & 15, fg = lane >> 4;
  auto read_frags = [&](int buf, int h, V8 (&af)[MT], V8 (&bf)[NT]) {
    if (mode & 2) return;
    const unsigned char* sa = smem + buf * STAGE;
    const unsigned char* sb = sa + A_BYTES;
    const int ch = h * 4 + fg;
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      const int r = wm * WM + mi * 16 + fr;
      af[mi] = *(const V8*)(sa + r * 128 + ((ch ^ ((r >> 1) & 7)) << 4));
    }
#pragma unroll
    for (int ni = 0; ni < NT; ++ni) {
      const int r = wn * WN + ni * 16 + fr;
      bf[ni] = *(const V8*)(sb + r * 128 + ((ch ^ ((r >> 1) & 7)) << 4));
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const V8 (&af)[MT], const V8 (&bf)[NT]) {
    if (mode & 2) return;
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) acc[mi][ni] = mfma8(af[mi], bf[ni], acc[mi][ni]);
  };

  // ---- main loop: ring of 3 stages; stage s lives in buffer s % 3.  The waits the compiler must see
  // (LDS reads retired before the barrier) use the builtin, so it does not re-wait them -- and with
  // them the next stage's fragment reads -- in front of the second MFMA half (an inline-asm lgkmcnt is
  // invisible to its waitcnt pass).  Only the LDS-DMA counts are inline asm (it does not track them).
#pragma unroll
  for (int s0 = 0; s0 < NS; ++s0)
    if (s0 < nkl) stage(kb + s0, s0);
  wait_ahead(min(nkl - 1, NS - 1));
  if (F8 && !MXI && tid < BM) sc_tab[tid] = scv;
  if (LNF && tid < BN) ln_cs[tid] = lncv;
  if (SMK && tid < BN) sm_bias[tid] = smbv;
  if (LNF && tid < BM) {  // (mean, rstd) per row, fp64 fold in a fixed order; written once stage 0 (issued after
    // the partials) has landed, so the 17 partial registers are not live across the K loop; read after its barriers
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
  __builtin_amdgcn_s_barrier();
  int buf = 0;
  if constexpr (!F8) {
  V8 a0[MT], b0[NT], a1[MT], b1[NT];
  read_frags(0, 0, a0, b0);
  // one K step: half-1 reads under the half-0 MFMAs, barrier, refill + next half-0 reads under the half-1
  // MFMAs.  The steady-state loop has no branches inside, so sched_group_barrier can interleave one read
  // (or LDS-DMA issue) between consecutive MFMAs within each of the two regions.
  auto step = [&](const bool refill, const int ahead, const int kt) {
    read_frags(buf, 1, a1, b1);
    mma(a0, b0);
    if (SCHED) {
#pragma unroll
      for (int i = 0; i < MT + NT; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, MT * NT - (MT + NT), 0);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the half-0 MFMAs on this side of the barrier
    wait_ahead(ahead);                   // stage kt+1 landed (kt+2 may still fly)
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's reads of stage kt retired
    __builtin_amdgcn_s_barrier();        // ... and every wave's; stage kt+1 visible to all
    if (refill) stage(kb + kt + NS, buf);
    buf = buf == NS - 1 ? 0 : buf + 1;
    read_frags(buf, 0, a0, b0);
    mma(a1, b1);
    if (SCHED) {
      if constexpr (PER_LO + MT + NT <= MT * NT) {
        if (refill) {
#pragma unroll
          for (int i = 0; i < PER_LO; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
            __builtin_amdgcn_sched_group_barrier(0x010, 1, 1);
          }
        }
#pragma unroll
        for (int i = 0; i < MT + NT; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        }
      } else {  // fewer MFMAs than loads + reads: one of each (while any remain) behind every MFMA
#pragma unroll
        for (int i = 0; i < MT * NT; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          if (refill && i < PER_LO) __builtin_amdgcn_sched_group_barrier(0x010, 1, 1);
          if (i < MT + NT) __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        }
      }
    }
  };
  int kt = 0;
  for (; kt < nkl - NS; ++kt) step(true, NS - 2, kt);
  for (; kt < nkl - 1; ++kt) step(false, min(NS - 2, nkl - 2 - kt), kt);
  read_frags(buf, 1, a1, b1);
  mma(a0, b0);
  mma(a1, b1);
  } else {
    // e4m3: half 0 = every A fragment + B column blocks ni < NH, half 1 = the others (A reused from a register
    // copy, since the next stage's half-0 reads overwrite a0 under the half-1 MFMAs)
    static_assert(NT >= 2, "column blocks per wave");
    constexpr int NH = NT / 2, NB1 = NT - NH;
    // The 8-bit 16x16x128 operand's K order (measured, probes/mx_diag2.py): a lane's 32 bytes are two 16-byte
    // halves at hardware k = 16 fg .. and 64 + 16 fg .., and the A scale of hardware block kb (k 32 kb ..) is taken
    // from lane row + 16 kb.  Per-row scaling only needs A and B to agree (chunks 2 fg, 2 fg + 1 of the 128-B
    // row); MX needs memory block kb = hardware block kb, so the lane reads chunks fg and 4 + fg.
    constexpr int C0 = MXI ? 1 : 2, C1 = MXI ? 4 : 1;
    auto frag = [&](const unsigned char* base, int r) {  // lane: row fr, 32 bytes of the 128-B K step
      const int sw = (r >> 1) & 7;
      const u32x4 lo = *(const u32x4*)(base + r * 128 + (((C0 * fg) ^ sw) << 4));
      const u32x4 hi = *(const u32x4*)(base + r * 128 + (((C0 * fg + C1) ^ sw) << 4));
      return V8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    };
    auto rd0 = [&](int b, V8 (&af)[MT], V8 (&bf)[NH], int (&sc)[MT]) {
      if (mode & 2) return;
      const unsigned char* sa = smem + b * STAGE;
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) af[mi] = frag(sa, wm * WM + mi * 16 + fr);
      if constexpr (MXI) {
#pragma unroll
        for (int mi = 0; mi < MT; ++mi)
          sc[mi] = (int)((*(const unsigned*)(smem + SCL_OFF + b * SCR + (wm * WM + mi * 16 + fr) * 4) >> (8 * fg)) & 255u);
      }
#pragma unroll
      for (int ni = 0; ni < NH; ++ni) bf[ni] = frag(sa + A_BYTES, wn * WN + ni * 16 + fr);
    };
    auto rd1 = [&](int b, V8 (&bf)[NB1]) {
      if (mode & 2) return;
      const unsigned char* sb = smem + b * STAGE + A_BYTES;
#pragma unroll
      for (int ni = 0; ni < NB1; ++ni) bf[ni] = frag(sb, wn * WN + (NH + ni) * 16 + fr);
    };
    auto mm0 = [&](const V8 (&af)[MT], const V8 (&bf)[NH], const int (&sc)[MT]) {
      if (mode & 2) return;
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NH; ++ni)
          acc[mi][ni] = MXI ? mfma8s(af[mi], bf[ni], acc[mi][ni], sc[mi]) : mfma8(af[mi], bf[ni], acc[mi][ni]);
    };
    auto mm1 = [&](const V8 (&af)[MT], const V8 (&bf)[NB1], const int (&sc)[MT]) {
      if (mode & 2) return;
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NB1; ++ni)
          acc[mi][NH + ni] = MXI ? mfma8s(af[mi], bf[ni], acc[mi][NH + ni], sc[mi])
                                 : mfma8(af[mi], bf[ni], acc[mi][NH + ni]);
    };
    V8 a0[MT], a1[MT], b0[NH], b1[NB1];
    int s0[MT], s1[MT];
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) s0[mi] = s1[mi] = 127;
    rd0(0, a0, b0, s0);
    auto step8 = [&](const bool refill, const int ahead, const int kt) {
      rd1(buf, b1);
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        a1[mi] = a0[mi];
        s1[mi] = s0[mi];
      }
      mm0(a0, b0, s0);
      if (SCHED) {  // the 2 * NB1 half-1 reads between the MT * NH half-0 MFMAs
        constexpr int R1 = 2 * NB1, M0 = MT * NH, RPM = (R1 + M0 - 1) / M0;
#pragma unroll
        for (int i = 0; i < M0; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
#pragma unroll
          for (int j = 0; j < RPM; ++j)
            if (i * RPM + j < R1) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      wait_ahead(ahead);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_s_barrier();
      if (refill) stage(kb + kt + NS, buf);
      buf = buf == NS - 1 ? 0 : buf + 1;
      rd0(buf, a0, b0, s0);
      mm1(a1, b1, s1);
      if (SCHED) {  // refill DMA + the next stage's 2 * (MT + NH) half-0 reads between the MT * NB1 MFMAs
        constexpr int R0 = 2 * (MT + NH), M1 = MT * NB1, RPM = (R0 + M1 - 1) / M1;
#pragma unroll
        for (int i = 0; i < M1; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          if (refill && i < PER_LO) __builtin_amdgcn_sched_group_barrier(0x010, 1, 1);
#pragma unroll
          for (int j = 0; j < RPM; ++j)
            if (i * RPM + j < R0) __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        }
      }
    };
    int kt = 0;
    for (; kt < nkl - NS; ++kt) step8(true, NS - 2, kt);
    for (; kt < nkl - 1; ++kt) step8(false, min(NS - 2, nkl - 2 - kt), kt);
    rd1(buf, b1);
    mm0(a0, b0, s0);
    mm1(a0, b1, s0);
  }
  constexpr bool lnf = LNF;

  // ---- split-K combine: each split stores its fp32 partial slab write-through (sc1) and drains it; one
  // lane then takes a ticket on the tile's counter (agent-scope atomic).  The last arriver reads all S
  // slabs with sc1 loads (no L1/L2 flush or invalidate needed: cdna_hip_programming.md section 5,
  // "Projection GEMM" item 2, sc1 form), sums them in split order and runs the epilogue; the others exit.
  if (S == 2) {
    // Pairwise combine: the first split to finish publishes its partial (sc1 stores, drained, then an sc1
    // flag); the second waits for the flag, adds the partial to its own and runs the epilogue.  Half the
    // slab traffic of the S-way form, and the sum a + b is bitwise the same whichever split came first.
    // The waiting split only ever waits on one that has already taken its ticket (it is running), so
    // no co-residency assumption is needed.
    constexpr int SLAB = MT * NT * NTHR * 16;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((char*)slabs + (long long)tile_id * SLAB, (short)0, SLAB, 0x00020000);
    unsigned* flag = counters + 32768 + tile_id;
    __syncthreads();  // every wave is past its last LDS read: smem[0] is free
    if (tid == 0) {
      const unsigned tk = __hip_atomic_fetch_add(counters + tile_id, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *(volatile unsigned*)smem = tk;
    }
    __syncthreads();
    const unsigned tk = *(volatile unsigned*)smem;
    if (tk == 0) {
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NT; ++ni)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[mi][ni]), rs,
                                                 ((mi * NT + ni) * NTHR + tid) * 16, 0, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0 && !__hip_atomic_load(&g_g8_sk_drop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if (tid == 0) {
      // bounded: a lost flag poisons the tile (NaN) instead of hanging the GPU, and counts a timeout in
      // g_g8_sk_timeouts.  The flag and the counter are reset only after the partner's flag was seen, so after a
      // timeout this tile's slot is stale (a late flag could be taken by a later launch): the host checks the count
      // at its sync points (fd_splitk_health, ops.split_k_health) and re-zeroes every workspace's counters.
      unsigned got = 0u;
      for (int it = 0; it < (1 << 24) && !got; ++it) {
        got = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!got) __builtin_amdgcn_s_sleep(2);
      }
      if (got) {
        __hip_atomic_store(flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(counters + tile_id, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        __hip_atomic_fetch_add(&g_g8_sk_timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      ((volatile unsigned*)smem)[1] = got;
    }
    __syncthreads();
    const bool partner_ok = ((volatile unsigned*)smem)[1] != 0u;
    f32x4 part[MT][NT];
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni)
        part[mi][ni] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ((mi * NT + ni) * NTHR + tid) * 16, 0, 16));
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) acc[mi][ni] += part[mi][ni];
    if (!partner_ok) {
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NT; ++ni) acc[mi][ni] = f32x4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
    }
  } else if (S > 1) {
    constexpr int SLAB = MT * NT * NTHR * 16;  // bytes per split of one tile
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((char*)slabs + (long long)tile_id * S * SLAB, (short)0, S * SLAB, 0x00020000);
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[mi][ni]), rs,
                                               split * SLAB + ((mi * NT + ni) * NTHR + tid) * 16, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const unsigned tk = __hip_atomic_fetch_add(counters + tile_id, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *(volatile unsigned*)smem = tk;
    }
    __syncthreads();
    const unsigned tk = *(volatile unsigned*)smem;
    if (tk != (unsigned)(S - 1)) return;
    if (tid == 0) __hip_atomic_store(counters + tile_id, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni)
        acc[mi][ni] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ((mi * NT + ni) * NTHR + tid) * 16, 0, 16));
    for (int q = 1; q < S; ++q) {
      f32x4 part[MT][NT];
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NT; ++ni)
          part[mi][ni] = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, q * SLAB + ((mi * NT + ni) * NTHR + tid) * 16, 0, 16));
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NT; ++ni) acc[mi][ni] += part[mi][ni];
    }
  }

  if (mode & 4) {
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) asm volatile("" ::"v"(acc[mi][ni]));
    return;
  }
  // ---- epilogue in BM / EROWS passes.  Phase 1: accumulators -> LDS fp32 [128][LDE] (alpha applied;
  // GEGLU pairs (h, g) are combined here, their bias loaded once per lane up front).  Phase 2: each thread
  // owns 8 consecutive columns of a row: bias, row-group bias (time embedding), activation and residual
  // with 16-B vector loads issued together, one 16-B store.  With one workgroup per CU nothing hides a
  // stalled epilogue, so no per-element branches or loads.
  TO* __restrict__ C = (TO*)p.C;
  const TO* __restrict__ R = (const TO*)p.residual;
  const float* __restrict__ bias = p.bias ? p.bias + bsn : nullptr;
  const float* __restrict__ rbias = p.rowbias;
  const int Nout = GEGLU ? N / 2 : N;
  const int n0o = GEGLU ? n0 / 2 : n0;
  const float alpha = p.alpha;
  const int act = p.act;
  float* ep = (float*)smem;
  constexpr int VPR = BNO / 8;
  // row-phase iterations whose loads are issued together
  // (1 for the 256 x 160 plain / conv tiles: five batched iterations push them past 256 VGPRs)
  constexpr int ITER = (BN == 160 && BM == 256 && !GEGLU) ? 1
                       : (EROWS * VPR) % (NTHR * 4) == 0 ? 4 : (EROWS * VPR) % (NTHR * 5) == 0 ? 5 : 1;
  static_assert(EROWS * VPR % (NTHR * ITER) == 0, "epilogue iterations");
  float gbh[GEGLU ? NT / 2 : 1], gbg[GEGLU ? NT / 2 : 1];
  if (GEGLU) {
#pragma unroll
    for (int q = 0; q < NT / 2; ++q) {
      const int np = min(n0 + wn * WN + 2 * q * 16 + fr, N - 17);
      gbh[q] = bias ? bias[np] : 0.f;
      gbg[q] = bias ? bias[np + 16] : 0.f;
    }
  }
  const bool vec = (Nout % 8 == 0) && (p.ldc % 8 == 0) && ((((unsigned long long)C) & 15) == 0) &&
                   (!R || ((p.ldr % 8 == 0) && ((((unsigned long long)R) & 15) == 0))) &&
                   (GEGLU || !bias || ((((unsigned long long)bias) & 15) == 0)) &&
                   (GEGLU || !rbias || ((p.rowbias_ld % 4 == 0) && ((((unsigned long long)rbias) & 15) == 0)));
  const bool interior = vec && (m0 + BM <= M) && (n0o + BNO <= Nout);
  typedef __attribute__((ext_vector_type(8))) TO TO8;
  // GroupNorm statistics: this thread's chunk (tid % VPR) is the same in every row pass (NTHR % VPR == 0);
  // gsplit = its columns in the chunk's first group (the host only asks for interior, group-aligned tiles)
  const bool gn = GN_OK && p.gn_part != nullptr;
  const int gcpg = (gn || (GN160 && p.gn_part != nullptr)) ? p.N / p.gn_groups : 8;
  const int gsplit = (((tid % VPR) * 8) / gcpg + 1) * gcpg - (tid % VPR) * 8;
  GnTile gna;
  const bool gn160 = GN160 && p.gn_part != nullptr;
  f32x4* const gslot = (f32x4*)(smem + RED_OFF);
  float g16s = 0.f, g16q = 0.f;  // this thread's group (tid / 32) sums over its rows, both halves
  // LN-fold producer (fd_gemm_params.ln_out) on the 160-column tiles: per-row (sum, sumsq) of the values as stored,
  // over the tile's 160 columns -- the partial layout of the 4-wave 64 x 160 producer (gemm.hip), which the
  // consumers read -- summed 8-column chunk by chunk in column order.  Chunk slots after the epilogue staging.
  constexpr bool LNO_OK = (BN == 160) && !GEGLU && !CONV && (EPB + EROWS * VPR * 8 <= SMEM) && EROWS <= NTHR;
  const bool lno = LNO_OK && p.ln_out != nullptr;
  float2* const lnslot = (float2*)(smem + EPB);
#pragma unroll 1
  for (int half = 0; half < BM / EROWS; ++half) {
    __syncthreads();  // ring (half 0) / previous half's staging (half 1) fully consumed
    if ((wm * WM) / EROWS == half) {
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int rl = wm * WM + mi * 16 + fg * 4 - half * EROWS;
        float rsc[4];  // alpha, or for e4m3 the row's a_scale * alpha
#pragma unroll
        for (int j = 0; j < 4; ++j) rsc[j] = (F8 && !MXI) ? sc_tab[rl + j + half * EROWS] : alpha;
        if (GEGLU) {
          // LN-fold operands read into registers ahead of the staging stores (same LDS object: hipcc would
          // otherwise re-read them after every store)
          float2 st[LNF ? 4 : 1];
          float lcn[LNF ? NT : 1];
          if (LNF) {
#pragma unroll
            for (int j = 0; j < (LNF ? 4 : 1); ++j) st[j] = ln_tab[rl + j + half * EROWS];
#pragma unroll
            for (int ni = 0; ni < (LNF ? NT : 1); ++ni) lcn[ni] = ln_cs[wn * WN + ni * 16 + fr];
          }
#pragma unroll
          for (int ni = 0; ni < NT; ni += 2) {
            const int col = (wn * WN) / 2 + (ni / 2) * 16 + fr;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float hv = acc[mi][ni][j] * rsc[j], g = acc[mi][ni + 1][j] * rsc[j];
              if (F8) {  // explicit fma (contraction would otherwise be the compiler's choice): gemm_fp8.hip's form
                hv = __builtin_fmaf(acc[mi][ni][j], rsc[j], gbh[ni / 2]);
                g = __builtin_fmaf(acc[mi][ni + 1][j], rsc[j], gbg[ni / 2]);
                ep[(rl + j) * LDE + col] = hv * (FD_GEGLU_DIAG ? g : gelu_f(g));
                continue;
              }
              if (LNF) {
                hv = st[j & (LNF ? 3 : 0)].y * (hv - st[j & (LNF ? 3 : 0)].x * lcn[ni % (LNF ? NT : 1)]);
                g = st[j & (LNF ? 3 : 0)].y * (g - st[j & (LNF ? 3 : 0)].x * lcn[(ni + 1) % (LNF ? NT : 1)]);
              }
              hv += gbh[ni / 2];
              g += gbg[ni / 2];
              ep[(rl + j) * LDE + col] = hv * (FD_GEGLU_DIAG ? g : gelu_f(g));
            }
          }
        } else {
#pragma unroll
          for (int ni = 0; ni < NT; ++ni) {
            const int col = wn * WN + ni * 16 + fr;
#pragma unroll
            for (int j = 0; j < 4; ++j) ep[(rl + j) * LDE + col] = acc[mi][ni][j] * rsc[j];
          }
        }
      }
    }
    __syncthreads();
    if constexpr (SMK) {
      if (sm) {
        // softmax over each row's two 80-column head groups: 4 lanes per (row, group), 20 columns each; the LayerNorm
        // fold and the bias are applied here (phase 2 only rounds and stores); columns >= sm_len become 0
        const int sl = p.sm_len;
#pragma unroll 1
        for (int e = tid; e < EROWS * 8; e += NTHR) {
          const int r = e >> 3, g = (e >> 2) & 1, q = e & 3;
          const int c0 = g * 80 + q * 20;
          float v[20];
#pragma unroll
          for (int i = 0; i < 5; ++i) *(f32x4*)&v[4 * i] = *(const f32x4*)(ep + r * LDE + c0 + 4 * i);
          float mu = 0.f, rs = 1.f;
          if (lnf) {
            const float2 st = ln_tab[half * EROWS + r];
            mu = st.x;
            rs = st.y;
          }
          float mx = -INFINITY;
#pragma unroll
          for (int i = 0; i < 20; ++i) {
            float x = v[i];
            if (lnf) x = rs * (x - mu * ln_cs[c0 + i]);
            x += sm_bias[c0 + i];
            v[i] = q * 20 + i < sl ? x : -INFINITY;
            mx = fmaxf(mx, v[i]);
          }
          mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
          mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
          float sum = 0.f;
#pragma unroll
          for (int i = 0; i < 20; ++i) {
            v[i] = q * 20 + i < sl ? __expf(v[i] - mx) : 0.f;
            sum += v[i];
          }
          sum += __shfl_xor(sum, 1, 64);
          sum += __shfl_xor(sum, 2, 64);
          const float inv = 1.0f / sum;
#pragma unroll
          for (int i = 0; i < 20; ++i) v[i] *= inv;
#pragma unroll
          for (int i = 0; i < 5; ++i) *(f32x4*)(ep + r * LDE + c0 + 4 * i) = *(const f32x4*)&v[4 * i];
        }
        __syncthreads();
      }
    }
    if (interior) {
#pragma unroll 1
    for (int e0 = 0; e0 < EROWS * VPR; e0 += NTHR * ITER) {
      float v[ITER][8], bv[ITER][8], rv[ITER][8];
      TO8 res[ITER];
#pragma unroll
      for (int it = 0; it < ITER; ++it) {
        const int e = e0 + tid + it * NTHR;
        const int r = e / VPR, cv = e % VPR;
        const int m = m0 + half * EROWS + r, n = n0o + cv * 8;
        *(f32x4*)&v[it][0] = *(const f32x4*)(ep + r * LDE + cv * 8);
        *(f32x4*)&v[it][4] = *(const f32x4*)(ep + r * LDE + cv * 8 + 4);
        if (!GEGLU && !sm && bias) {
          *(f32x4*)&bv[it][0] = *(const f32x4*)(bias + n);
          *(f32x4*)&bv[it][4] = *(const f32x4*)(bias + n + 4);
        }
        if (!GEGLU && rbias) {
          const float* rb = rbias + (long long)(m / p.rows_per_group) * p.rowbias_ld + n;
          *(f32x4*)&rv[it][0] = *(const f32x4*)rb;
          *(f32x4*)&rv[it][4] = *(const f32x4*)(rb + 4);
        }
        if (R) res[it] = *(const TO8*)(R + (long long)m * p.ldr + n);
      }
#pragma unroll
      for (int it = 0; it < ITER; ++it) {
        const int e = e0 + tid + it * NTHR;
        const int r = e / VPR, cv = e % VPR;
        const int m = m0 + half * EROWS + r, n = n0o + cv * 8;
        if (!GEGLU && !sm) {
          if (lnf) {
            const float2 st = ln_tab[half * EROWS + r];
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
        if constexpr (MXO) {  // 32-column block = 4 consecutive threads (VPR % 4 == 0, n0o % 32 == 0)
          float am = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) am = fmaxf(am, fabsf(v[it][i]));
          am = fmaxf(am, __shfl_xor(am, 1, 64));
          am = fmaxf(am, __shfl_xor(am, 2, 64));
          const int E = mx_exp(am);
          *(u32x2*)((uint8_t*)p.C + (long long)m * p.ldc + n) =
              u32x2{mx_pack4(v[it][0], v[it][1], v[it][2], v[it][3], E), mx_pack4(v[it][4], v[it][5], v[it][6], v[it][7], E)};
          if ((cv & 3) == 0) f8.o_bs[(long long)m * f8.o_bs_ld + n / 32] = (uint8_t)(E + 127);
          continue;
        }
        TO8 o;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (TO)v[it][i];
        st_out16((TO8*)(C + (long long)m * p.ldc + n), o);
        if (gn) gna.add(o, gsplit);
        if (GN160 && gn160) {
          const int gs = ((cv * 8) / gcpg + 1) * gcpg - cv * 8;
          float s0 = 0.f, q0 = 0.f, s1 = 0.f, q1 = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float f = (float)o[i];
            if (i < gs) {
              s0 += f;
              q0 += f * f;
            } else {
              s1 += f;
              q1 += f * f;
            }
          }
          gslot[e] = (f32x4){s0, q0, s1, q1};
        }
        if (LNO_OK && lno) {
          float ls = 0.f, lq = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float f = (float)o[i];
            ls += f;
            lq += f * f;
          }
          lnslot[e] = make_float2(ls, lq);
        }
      }
    }
    } else if constexpr (!MXO) {  // edge tiles / unaligned operands: scalar, bounds-checked (MX: host-checked interior)
      for (int e = tid; e < EROWS * VPR; e += NTHR) {
        const int r = e / VPR, cv = e % VPR;
        const int m = m0 + half * EROWS + r, n = n0o + cv * 8;
        if (m >= M || n >= Nout) {
          if (LNO_OK && lno) lnslot[e] = make_float2(0.f, 0.f);
          continue;
        }
        float ls = 0.f, lq = 0.f;
        for (int i = 0; i < 8 && n + i < Nout; ++i) {
          float x = ep[r * LDE + cv * 8 + i];
          if (!GEGLU && !sm) {
            if (lnf) {
              const float2 st = ln_tab[half * EROWS + r];
              x = st.y * (x - st.x * ln_cs[cv * 8 + i]);
            }
            if (bias) x += bias[n + i];
            if (rbias) x += rbias[(long long)(m / p.rows_per_group) * p.rowbias_ld + n + i];
            x = act_f(x, act);
          }
          if (R) x += (float)R[(long long)m * p.ldr + n + i];
          const TO o1 = (TO)x;
          C[(long long)m * p.ldc + n + i] = o1;
          ls += (float)o1;
          lq += (float)o1 * (float)o1;
        }
        if (LNO_OK && lno) lnslot[e] = make_float2(ls, lq);
      }
    }
    if (GN160 && gn160) {  // this half's chunk slots: thread (g, j) folds rows j, j + 32, ... of group g
      __syncthreads();
      const int g = tid >> 5, j = tid & 31;
      if (g < BNO / gcpg) {
        const int c0 = (g * gcpg) / 8, c1 = ((g + 1) * gcpg - 1) / 8;
        for (int r = j; r < EROWS; r += 32)
          for (int c = c0; c <= c1; ++c) {
            const f32x4 v4 = gslot[r * VPR + c];
            const bool first = (c * 8) / gcpg == g;
            g16s += first ? v4[0] : v4[2];
            g16q += first ? v4[1] : v4[3];
          }
      }
    }
    if (LNO_OK && lno) {  // this half's rows: 20 chunk slots each, summed in column order
      __syncthreads();
      const int mr = m0 + half * EROWS + tid;
      if (tid < EROWS && mr < M) {
        float ls = 0.f, lq = 0.f;
#pragma unroll
        for (int c = 0; c < VPR; ++c) {
          const float2 v2 = lnslot[tid * VPR + c];
          ls += v2.x;
          lq += v2.y;
        }
        ((float2*)p.ln_out)[(long long)mr * (N / 160) + n0 / 160] = make_float2(ls, lq);
      }
    }
  }
  if constexpr (GN_OK) {
    if (gn) gn_tile_write(gna, (float2*)(smem + RED_OFF), tid, NTHR, VPR, gcpg, BNO, n0o, m0, p);
  }
  if constexpr (GN160) {
    if (gn160) {  // 32-lane butterfly (fixed order), lane 0 of each group writes the tile's (sum, sumsq)
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) {
        g16s += __shfl_xor(g16s, o, 64);
        g16q += __shfl_xor(g16q, o, 64);
      }
      const int g = tid >> 5;
      if ((tid & 31) == 0 && g < BNO / gcpg) {
        const long long blk = (long long)(m0 / p.gn_hw) * (p.gn_hw / 256) + (m0 % p.gn_hw) / 256;
        ((float2*)p.gn_part)[blk * p.gn_groups + n0o / gcpg + g] = make_float2(g16s, g16q);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------ host
namespace {

struct Plan8 {
  int bm, bn, nw, waves_m, ns, S, group_m, tiles;
};

// Split count from the per-tile row count m_ref (not the batched M).  Measured on MI355X (scripts/gemm8_sweep.sh,
// profiles/r01_gemm8_sweep.txt): one 147 KiB workgroup per CU streams ~40-70 GB/s of operands, so a 256x128 tile
// K step costs ~1.1-1.4 us whatever the tile count, while the split-K slab round trip (write-through fp32 slabs
// + the reducer's reads) costs ~S * tiles * 256 KiB at HBM speed (~15 us at 2048 x 1280).  Splitting therefore
// pays only for long K (the 3x3 convs of the 32^2 level, K = 9 * 1280 and up).  Returns 0 when the 4-wave
// kernel is the better choice (few tiles and short K, or N not a multiple of the 128-column tile).
int choose_split(int m_ref, int N, int K, int bn) {
  const int nk = K / 64;
  const long long tiles = (long long)((m_ref + 255) / 256) * ((N + bn - 1) / bn);
  if (N % bn != 0) return 0;
  if (tiles >= 192) return 1;
  // mid K on the 32^2 level (ff out 2048 x 1280 x 5120, the K = 5760 conv): three splits of 80 tiles beat the
  // 4-wave 64 x 160 kernel with cold weights, 47.1 -> 41.1 us / 61.2 -> 45.0 us, and stay ahead when 13 TLC tiles
  // share the launch (C3: 520 -> 454 us); N = 640 at 64^2 (160 tiles) gains nothing (profiles/r02e_ksplit.jsonl)
  const int midk = fd_knob(FDK_GEMM8_MIDK);  // 0 = off (A/B), else the split count
  if (midk > 0 && K >= 4096 && K < 8192 && N >= 1280 && tiles <= 96) return midk;
  if (K < 8192) return 0;
  int s = (int)(256 / tiles);
  if (s > nk / 8) s = nk / 8;
  if (s > 8) s = 8;
  return s < 1 ? 1 : s;
}

template <typename T, typename TO, int BM, int BN, int NW, int WAVES_M, int NS>
int launch8(const fd_gemm_params* p, const Plan8& pl, hipStream_t s) {
  dim3 grid(pl.tiles * pl.S), block(64 * NW);
  float* slabs = (float*)((char*)p->ws + 65536 * sizeof(unsigned));
  unsigned* cnt = (unsigned*)p->ws;
  if constexpr (BM < 256) {
    // 128 / 64-row tiles: plan8 gives them only the LN-fold producers (plain) and the cross-attention score GEMMs
    // (plain, or LN-fold consumers: the attn2 LayerNorm is folded into the score GEMM)
    if (p->conv || p->act == FD_ACT_GEGLU) return FD_ERR_ARG;
    if (p->ln_in)
      hipLaunchKernelGGL((gemm8_kernel<T, BM, BN, NW, WAVES_M, NS, false, false, TO, true>), grid, block, 0, s, *p,
                         pl.S, pl.group_m, slabs, cnt, f8_args{});
    else
      hipLaunchKernelGGL((gemm8_kernel<T, BM, BN, NW, WAVES_M, NS, false, false, TO>), grid, block, 0, s, *p, pl.S,
                         pl.group_m, slabs, cnt, f8_args{});
  } else if (p->conv) {
    hipLaunchKernelGGL((gemm8_kernel<T, BM, BN, NW, WAVES_M, NS, true, false, TO>), grid, block, 0, s, *p, pl.S,
                       pl.group_m, slabs, cnt, f8_args{});
  } else if (p->act == FD_ACT_GEGLU) {
    if constexpr ((BN / (NW / WAVES_M)) % 32 == 0) {
      if (p->ln_in)
        hipLaunchKernelGGL((gemm8_kernel<T, BM, BN, NW, WAVES_M, NS, false, true, TO, true>), grid, block, 0, s, *p,
                           pl.S, pl.group_m, slabs, cnt, f8_args{});
      else
        hipLaunchKernelGGL((gemm8_kernel<T, BM, BN, NW, WAVES_M, NS, false, true, TO>), grid, block, 0, s, *p, pl.S,
                           pl.group_m, slabs, cnt, f8_args{});
    } else {
      return FD_ERR_ARG;
    }
  } else if (p->ln_in) {
    hipLaunchKernelGGL((gemm8_kernel<T, BM, BN, NW, WAVES_M, NS, false, false, TO, true>), grid, block, 0, s, *p, pl.S,
                       pl.group_m, slabs, cnt, f8_args{});
  } else {
    hipLaunchKernelGGL((gemm8_kernel<T, BM, BN, NW, WAVES_M, NS, false, false, TO>), grid, block, 0, s, *p, pl.S,
                       pl.group_m, slabs, cnt, f8_args{});
  }
  FD_LAUNCH_CHECK();
  return FD_OK;
}

}  // namespace

// Plan for one launch (0 = not eligible -> the 4-wave kernel).  Shared by fd_gemm8_ws_bytes and fd_gemm8.
// Every decision reads m_ref (rows per TLC tile), never the batched M, so batching tiles changes no bit:
// the 4-wave kernel sums each K step's two halves in separate waves, these kernels in one accumulator,
// and any tile shape of the same kernel family gives the same k order.
static int plan8(const fd_gemm_params* p, Plan8* pl) {
  const int enabled = fd_knob(FDK_GEMM8), force_s = fd_knob(FDK_GEMM8_S), force_gm = fd_knob(FDK_GEMM8_GM);
  const int w160 = fd_knob(FDK_GEMM8_W160);  // bit 0: 256 x 160 tiles where faster; bit 1: also take N = 320
  const int m_ref = p->m_ref > 0 ? p->m_ref : p->M;
  if (!enabled || p->batch > 1 || p->K < 128) return 0;
  // (round 6: the variants measured slower and kept only as knobs were removed -- the 64 x 160 one-wave-per-SIMD
  // instance, the pairwise 128-row split at M = 2048, the 4-deep 128 x 160 ring, the 128-channel convs on the 4-wave
  // kernel, the split cross-attention score GEMM, the 256 x 160 S-way and large-M LN-fold producers, and the four-wave
  // 128 x 160 tile; their measurements are in DESIGN.md section 5 and git history)
  Plan8 q;
  if (p->act == FD_ACT_SOFTMAX) {
    // the attention-score GEMM: 160-column tiles (two 80-column head groups): the tile with the fewest operand bytes
    // per CU, rounds on 256 CUs x (BM + BN); FD_XATTN_SPLIT: the 128 x 160 form with K split in two (pairwise
    // combine, softmax after it) -- 320 half-K workgroups instead of 160 full ones at M = 2048 (measured slower)
    if (p->N % 160) return 0;
    // one K pass: every tile shape gives the same bits, so the batched M may choose (C3's 13 tiles: 256 x 160)
    const int m_plan = p->M;
    int best = 0;
    long long bc = 0;
    for (int bm = 256; bm >= 64; bm /= 2) {
      const long long tiles = (long long)((m_plan + bm - 1) / bm) * (p->N / 160);
      const long long c = (tiles + 255) / 256 * (bm + 160);
      if (!best || c < bc) {
        best = bm;
        bc = c;
      }
    }
    q.bm = best;
    q.bn = 160;
    q.nw = best >= 128 ? 8 : 4;  // 128 x 160: eight waves of 32 x 80 (two per SIMD)
    q.waves_m = best == 256 ? 8 : best == 128 ? 4 : 2;
    q.ns = 3;
    q.S = 1;
    goto planned;
  }
  if (p->ln_out) {
    // LN-fold producer: only a 160-column tile writes the partial layout the consumers read.  Long K (the ff out
    // of the 32^2 level, 2048 x 1280 x 5120 at C2): 128 x 160 tiles with K split in two (pairwise combine),
    // 0.64x the operand bytes per CU of the 4-wave 64 x 160 producer (probe with cold weights 47.1 -> 40.6 us,
    // profiles/r02e_m2048_split.jsonl); anything else stays on that producer (return 0).
    const int lnp = fd_knob(FDK_GEMM8_LNP);
    // K >= 4096 (the ff outs); shorter producers (attention out-projections, proj_in) stay on the 4-wave 64 x 160 tile
    if (!lnp || p->act == FD_ACT_GEGLU || p->conv || p->N % 160 || p->K < 4096 || m_ref < 128) return 0;
    if ((long long)((m_ref + 63) / 64) * (p->N / 160) > 256) return 0;
    q.bm = 128;
    q.bn = 160;
    // eight waves of 32 x 80 (two per SIMD: one wave's fragment reads under the other's MFMAs)
    q.nw = 8;
    q.waves_m = 4;
    q.ns = 3;
    q.S = 2;
    goto planned;
  }
  // 256 x 128 tiles (4 x 2 waves of 64 x 64).  256 x 160 (98 vs 85 flop/B) spills at the 256-VGPR cap of
  // two waves per SIMD with register-double-buffered fragments; kept out until it fits.
  q.bm = 256;
  q.bn = 128;
  q.nw = 8;
  q.waves_m = 4;
  q.ns = 3;
  q.S = (m_ref >= 256 && p->N >= 128) ? (force_s > 0 ? force_s : choose_split(m_ref, p->N, p->K, q.bn)) : 0;
  if (w160 && m_ref >= 256 && p->N % 160 == 0 && force_s <= 0) {
    // 256 x 160 tiles (8 waves of 32 x 160) when they finish in less time on 256 CUs: time ~ rounds x
    // (columns per workgroup) / S.  2048 x 10240 GEGLU: 640 -> 512 tiles (3 -> 2 rounds); 8192 x 1280 conv:
    // 320 -> 256 tiles; 8192 x 640 long-K conv: 160 tiles S = 1 -> 128 tiles S = 2; N = 320 at 128^2.
    const long long tm = (m_ref + 255) / 256;
    const int s160 = choose_split(m_ref, p->N, p->K, 160);
    if (s160 > 0) {
      const double t160 = (double)((tm * (p->N / 160) * s160 + 255) / 256) * 160.0 / s160;
      const double t128 = q.S > 0 ? (double)((tm * ((p->N + 127) / 128) * q.S + 255) / 256) * 128.0 / q.S : 1e30;
      const bool narrow = q.S <= 0 && !(w160 & 2);  // the 4-wave kernel holds N = 320 unless FD_GEMM8_W160 & 2
      if (!narrow && t160 < 0.9 * t128) {
        q.bn = 160;
        q.waves_m = 8;
        q.S = s160;
      }
    }
  }
  if (q.S <= 0) return 0;  // few tiles and short K: the 4-wave kernel (gemm.hip)
planned:
  if (q.S > p->K / 64) q.S = p->K / 64;
  const int tiles_m = (p->M + q.bm - 1) / q.bm, tiles_n = (p->N + q.bn - 1) / q.bn;
  q.tiles = tiles_m * tiles_n;
  if (q.S > 1 && q.tiles > (q.S == 2 ? 32768 : 65536)) return 0;
  // group_m: per-XCD chunk of tiles/8 tiles; pick the tile-row group height minimising that chunk's
  // unique A rows + B columns (both stream K bytes each)
  int gm = 1;
  {
    const long long per_xcd = ((long long)q.tiles + 7) / 8;
    double bestc = 1e30;
    for (int g = 1; g <= tiles_m; g *= 2) {
      const long long cols = per_xcd < g ? 1 : (per_xcd + g - 1) / g;
      const long long rows = per_xcd < g ? per_xcd : g;
      const double c = rows * (double)q.bm + (cols < tiles_n ? cols : tiles_n) * (double)q.bn;
      if (c < bestc - 1e-9) { bestc = c; gm = g; }
    }
  }
  q.group_m = force_gm > 0 ? force_gm : gm;
  *pl = q;
  return 1;
}

extern "C" long long fd_conv_halo_ws_bytes(const fd_gemm_params* p);

extern "C" long long fd_gemm_ws_bytes(const fd_gemm_params* p) {
  if (p && p->conv) {  // the halo-staged conv takes it (its own split-K slabs, or none)
    const long long hb = fd_conv_halo_ws_bytes(p);
    if (hb >= 0) return hb;
  }
  Plan8 pl;
  if (!p || !plan8(p, &pl) || pl.S <= 1) return 0;
  const long long slab = (long long)pl.bm * pl.bn * 4;
  return 65536LL * sizeof(unsigned) + (long long)pl.tiles * pl.S * slab;
}

// GroupNorm output statistics (fd_gemm_params.gn_part) from the 256 x 128 instance's vector epilogue: every
// tile interior, inside one image and a whole number of groups wide.
static bool gn_ok8(const fd_gemm_params* p, const Plan8& pl) {
  if (!p->gn_part || pl.bm != 256 || (pl.bn != 128 && pl.bn != 160) || p->act == FD_ACT_GEGLU || p->ln_in ||
      p->ln_out)
    return false;
  if (p->gn_groups <= 0 || p->gn_hw <= 0 || p->N % p->gn_groups) return false;
  const int cpg = p->N / p->gn_groups;
  // 128-column tiles: one chunk per thread, cpg >= 4; 160-column tiles: <= 16 groups per tile (32 folding
  // threads each), so cpg >= 10
  if (pl.bn == 128 ? (cpg < 4 || 128 % cpg) : (cpg < 10 || 160 % cpg)) return false;
  if (p->N % pl.bn || p->M % 256 || p->gn_hw % 256 || p->M % p->gn_hw) return false;
  const unsigned long long al = (unsigned long long)p->C | (p->residual ? (unsigned long long)p->residual : 0) |
                                (p->bias ? (unsigned long long)p->bias : 0) | (p->rowbias ? (unsigned long long)p->rowbias : 0);
  return (al & 15) == 0 && p->ldc % 8 == 0 && (!p->residual || p->ldr % 8 == 0) &&
         (!p->rowbias || p->rowbias_ld % 4 == 0);
}

// Returns 1 and launches when the eight-wave kernel takes this GEMM, 0 when it does not apply, < 0 on error.
extern "C" int fd_gemm8_try(fd_gemm_params* p0, void* stream) {
  Plan8 pl;
  if (!plan8(p0, &pl)) return 0;
  fd_gemm_params q = *p0;  // the kernel's copy: gn_part kept only where this instance writes the statistics
  if (!gn_ok8(p0, pl)) q.gn_part = nullptr;
  const fd_gemm_params* p = &q;
  if (pl.S > 1) {
    const long long need = 65536LL * sizeof(unsigned) + (long long)pl.tiles * pl.S * pl.bm * pl.bn * 4;
    if (!p->ws || p->ws_bytes < need) return FD_ERR_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  int rc;
#define FD_G8(BM_, BN_, NW_, WM_, NS_) \
  FD_DISPATCH_T(p->dtype, FD_DISPATCH_O(p->out_dtype, rc = (launch8<T, TO, BM_, BN_, NW_, WM_, NS_>(p, pl, s))))
  if (pl.bm == 256 && pl.bn == 160) {
    FD_G8(256, 160, 8, 8, 3);
  } else if (pl.bm == 256) {
    FD_G8(256, 128, 8, 4, 3);
  } else if (pl.bm == 128) {
    FD_G8(128, 160, 8, 4, 3);
  } else {
    FD_G8(64, 160, 4, 2, 3);  // the 64-row score-GEMM tile (M <= 64 per launch)
  }
#undef FD_G8
  if (rc == FD_OK) p0->gn_done = q.gn_part != nullptr ? 256 : 0;
  return rc == FD_OK ? 1 : rc;
}

// ------------------------------------------------------------------------------------ e4m3 (fd_gemm_e4m3 / _mxe4m3)
namespace {
template <typename T, typename TO, int BM, int BN, int NW, int WAVES_M>
int launch8_e4m3(const fd_gemm_params* p, const Plan8& pl, const f8_args& f8, hipStream_t s) {
  dim3 grid(pl.tiles), block(64 * NW);
  if (p->act == FD_ACT_GEGLU) {
    if constexpr ((BN / (NW / WAVES_M)) % 32 == 0)
      hipLaunchKernelGGL((gemm8_kernel<T, BM, BN, NW, WAVES_M, 3, false, true, TO>), grid, block, 0, s, *p, 1,
                         pl.group_m, nullptr, nullptr, f8);
    else
      return FD_ERR_ARG;
  } else {
    hipLaunchKernelGGL((gemm8_kernel<T, BM, BN, NW, WAVES_M, 3, false, false, TO>), grid, block, 0, s, *p, 1,
                       pl.group_m, nullptr, nullptr, f8);
  }
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// Tile plan for the e4m3 kernels.  No split-K: every output is one accumulator over K in order, so the tile shape --
// chosen from (M, N, K) -- never changes a bit (batched TLC tiles stay bitwise).  Least rounds x per-tile time on
// 256 CUs, the per-tile time a + b * K / 1280 us fitted per shape to the graph-timed launches of
// profiles/r03_f8_tiles.jsonl (K = 640 .. 5120; the fixed part -- prologue, epilogue, launch ramp -- is 40-60 % of a
// K = 1280 tile); FD_F8_TILE = 256160 / 256128 / 128160 / 64160 forces one (A/B, tests).  mx_out: only tiles whose
// output columns are whole 32-column blocks and lie inside M / N_out (the MX epilogue has no edge path).
int plan_e4m3(const fd_gemm_params* p, bool mx_out, Plan8* pl) {
  const int force = fd_knob(FDK_F8_TILE);  // tests compare the shapes in one process
  struct Cand { int bm, bn, nw, wm; double a, b; };
  static const Cand cands[4] = {{256, 160, 8, 8, 10.6, 10.2}, {256, 128, 8, 4, 7.5, 7.9},
                                {128, 160, 4, 2, 7.4, 6.0}, {64, 160, 4, 2, 5.65, 4.42}};
  const bool geglu = p->act == FD_ACT_GEGLU;
  const int nout = geglu ? p->N / 2 : p->N;
  int best = -1;
  double bt = 1e30;
  bool ok128 = false;
  for (int c = 0; c < 4; ++c) {
    const Cand& q = cands[c];
    if (geglu && (q.bn / (q.nw / q.wm)) % 32) continue;
    if (force && force != q.bm * 1000 + q.bn) continue;
    const int bno = geglu ? q.bn / 2 : q.bn;
    if (mx_out && (bno % 32 || nout % bno || p->M % q.bm)) continue;
    if (c == 1) ok128 = true;
    const long long tiles = (long long)((p->M + q.bm - 1) / q.bm) * ((p->N + q.bn - 1) / q.bn);
    // the 256 x 160 GEGLU tile stores 80 columns: its fixed part is relatively smaller (fit: 0.9x)
    const double t = (double)((tiles + 255) / 256) * (q.a + q.b * p->K / 1280.0) * (geglu && c == 0 ? 0.9 : 1.0);
    if (t < bt * 0.999) { bt = t; best = c; }
  }
  // M >= 16384 (the tiled C4 forwards: 25 tiles = 51200 / 204800 rows): many rounds per launch, where the model's
  // per-tile fit (C2 shapes, M <= 8192) no longer ranks the tiles -- every launch on 256 x 128 measured 72.56 vs
  // 71.32 tile-steps/s for the modelled mix (profiles/r05am_f8_tile_c4_ab.txt).  C2's e4m3 launches stay as planned.
  if (!force && p->M >= 16384 && ok128) best = 1;
  if (best < 0) return 0;
  pl->bm = cands[best].bm;
  pl->bn = cands[best].bn;
  pl->nw = cands[best].nw;
  pl->waves_m = cands[best].wm;
  if (pl->bm == 128) {  // eight waves of 32 x 80 (as the 16-bit 128 x 160 tiles)
    pl->nw = 8;
    pl->waves_m = 4;
  }
  pl->ns = 3;
  pl->S = 1;
  const int tiles_m = (p->M + pl->bm - 1) / pl->bm, tiles_n = (p->N + pl->bn - 1) / pl->bn;
  pl->tiles = tiles_m * tiles_n;
  const long long per_xcd = ((long long)pl->tiles + 7) / 8;  // group_m as plan8
  double bestc = 1e30;
  int gm = 1;
  for (int g = 1; g <= tiles_m; g *= 2) {
    const long long cols = per_xcd < g ? 1 : (per_xcd + g - 1) / g;
    const long long rows = per_xcd < g ? per_xcd : g;
    const double c = rows * (double)pl->bm + (cols < tiles_n ? cols : tiles_n) * (double)pl->bn;
    if (c < bestc - 1e-9) { bestc = c; gm = g; }
  }
  pl->group_m = gm;
  return 1;
}

template <typename T>
int launch_e4m3(const fd_gemm_params* p, const Plan8& pl, const f8_args& f8, int out_dtype, hipStream_t s) {
  int rc = FD_ERR_DTYPE;
#define FD_G8F(TO_)                                                                            \
  if (pl.bm == 256 && pl.bn == 160) rc = launch8_e4m3<T, TO_, 256, 160, 8, 8>(p, pl, f8, s);   \
  else if (pl.bm == 256) rc = launch8_e4m3<T, TO_, 256, 128, 8, 4>(p, pl, f8, s);              \
  else if (pl.bm == 128) rc = launch8_e4m3<T, TO_, 128, 160, 8, 4>(p, pl, f8, s);              \
  else rc = launch8_e4m3<T, TO_, 64, 160, 4, 2>(p, pl, f8, s);
  if (out_dtype == FD_BF16) {
    FD_G8F(bf16)
  } else if (out_dtype == FD_F16) {
    FD_G8F(f16)
  } else if (out_dtype == FD_F32) {
    FD_G8F(float)
  } else if (out_dtype == FD_MXE4M3) {
    FD_G8F(uint8_t)
  }
#undef FD_G8F
  return rc;
}
}  // namespace

// The e4m3 GEMM of fd_gemm_e4m3 on the eight-wave kernel family (p->A / p->B e4m3 bytes, p->alpha = w_scale,
// a_scale[M] per-row activation scales).  Returns 1 when launched, 0 when not applicable (ragged K, batch,
// alignment), < 0 on error.
extern "C" int fd_gemm8_e4m3_try(fd_gemm_params* p, const float* a_scale, void* stream) {
  if (p->batch > 1 || p->conv || p->ln_in || p->ln_out || p->rowbias || p->K % 128) return 0;
  if (((unsigned long long)p->A | (unsigned long long)p->B) & 15 || p->lda % 16 || p->ldb % 16) return 0;
  Plan8 pl;
  if (!plan_e4m3(p, false, &pl)) return 0;
  fd_gemm_params q = *p;
  q.gn_part = nullptr;
  f8_args f8{a_scale, nullptr, 0, nullptr, 0};
  const int rc = launch_e4m3<uint8_t>(&q, pl, f8, q.out_dtype, (hipStream_t)stream);
  return rc == FD_OK ? 1 : rc;
}

extern "C" int fd_gemm_mxe4m3(const void* A8, long long lda, const void* a_bs, long long ldas, const void* W8,
                              long long ldw, float w_scale, void* C, long long ldc, void* c_bs, long long ldcs, int M,
                              int N, int K, const float* bias, const void* residual, long long ldr, int act,
                              int out_dtype, void* stream) {
  if (!A8 || !a_bs || !W8 || !C) return FD_ERR_ARG;
  if (act < FD_ACT_NONE || act > FD_ACT_GEGLU) return FD_ERR_ARG;
  const int nout = act == FD_ACT_GEGLU ? N / 2 : N;
  if (M <= 0 || N <= 0 || K <= 0 || K % 128 || lda % 16 || ldw % 16 || lda < K || ldw < K || ldc < nout)
    return FD_ERR_SHAPE;
  if (act == FD_ACT_GEGLU && (N % 32)) return FD_ERR_SHAPE;
  if (ldas % 4 || ldas < K / 32 || ((unsigned long long)a_bs & 3)) return FD_ERR_SHAPE;
  if ((((unsigned long long)A8) | ((unsigned long long)W8)) & 15) return FD_ERR_ARG;
  if (out_dtype != FD_BF16 && out_dtype != FD_F16 && out_dtype != FD_F32 && out_dtype != FD_MXE4M3) return FD_ERR_DTYPE;
  const bool mx_out = out_dtype == FD_MXE4M3;
  if (residual && (ldr < nout || out_dtype == FD_F32 || mx_out)) return FD_ERR_SHAPE;
  // an MX output is written only by the interior 16-B vector epilogue: C (and the bias it reads as vectors unless
  // GEGLU) must be 16-B aligned, or a tile would be planned that writes nothing
  if (mx_out && (!c_bs || ldcs < nout / 32 || ldc % 16 || ((unsigned long long)C & 15) ||
                 (act != FD_ACT_GEGLU && bias && ((unsigned long long)bias & 15))))
    return FD_ERR_SHAPE;
  fd_gemm_params p{};
  p.A = A8;
  p.B = W8;
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
  Plan8 pl;
  if (!plan_e4m3(&p, mx_out, &pl)) return FD_ERR_SHAPE;
  f8_args f8{nullptr, (const uint8_t*)a_bs, ldas, (uint8_t*)c_bs, ldcs};
  return launch_e4m3<mx8_t>(&p, pl, f8, out_dtype, (hipStream_t)stream);
}

// Split-K hand-off health of this translation unit (fd_splitk_health in knobs.hip sums the units): adds the timed-out
// pairwise waits to *timeouts; reset: zero the count; drop >= 0: set the test hook (1: publishers skip their flag).
int g8_splitk_health(unsigned* timeouts, int reset, int drop) {
  unsigned v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_g8_sk_timeouts), sizeof(v)) != hipSuccess) return FD_ERR_HIP;
  if (timeouts) *timeouts += v;
  const unsigned z = 0u, d = (unsigned)drop;
  if (reset && hipMemcpyToSymbol(HIP_SYMBOL(g_g8_sk_timeouts), &z, sizeof(z)) != hipSuccess) return FD_ERR_HIP;
  if (drop >= 0 && hipMemcpyToSymbol(HIP_SYMBOL(g_g8_sk_drop), &d, sizeof(d)) != hipSuccess) return FD_ERR_HIP;
  return FD_OK;
}
