// 256 x 256-tile MFMA GEMM / implicit-GEMM convolution for gfx950, for the large-M launches (the VAE decoder's and
// encoders' 256- and 512-channel convs at 256^2..1024^2, the upsample convs): one workgroup per CU.
//
// Why: the 256 x 128 eight-wave kernel (gemm8.hip) is bound by the per-CU operand stream into LDS, not by the
// MFMA pipe (scripts/diag_probe.sh: its load-only build takes 70-90 % of the full time, its compute-only build
// ~50 %).  A 256 x 256 tile needs 32 KB of operands per 4.2 MFLOP (131 flop/B) instead of 48 KB (85 flop/B).
//
// Structure: 512 threads = 8 waves (4 x 2), each a 64 x 128 sub-tile of v_mfma_f32_16x16x32 (32 accumulators),
// in two groups of four that ping-pong (group 1 one barrier behind group 0, so on every SIMD one wave computes while
// its partner reads fragments / issues LDS-DMA).  Two 64 KB K tiles of 64 in LDS as 128-B rows with a source-side
// XOR swizzle (16-B chunk ^ ((row >> 1) & 7)): the 16-row ds_read_b128 fragments are conflict-free.  K is summed in
// 32-deep halves in order, the same order as gemm8's two 32-deep halves per 64-deep step, so both kernels give the
// same bits.  Conv: im2col gather from NHWC with out-of-image taps on a zero page, exact-x2 / diffusers upsample and
// two-source channel concat folded in.
// Epilogue: the 256 x 256 fp32 tile in two 128-row passes through the drained ring (phase 1 accumulators -> LDS,
// phase 2 eight columns per thread: bias / row bias / activation / residual with 16-B loads, one 16-B store).
#include <stdlib.h>

#include "fd_common.h"

__device__ __attribute__((aligned(256))) unsigned char g_zero_page256[256];

// diagnostic builds only (-DFD_G256_DIAG=m; 0 in the product): 1 = no operand loads, 2 = no LDS reads / MFMA,
// 4 = no epilogue stores (scripts/g256_diag.sh)
#ifndef FD_G256_DIAG
#define FD_G256_DIAG 0
#endif

namespace {

template <typename T, typename TO, bool CONV, int NW>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(1, 2)))
gemm256_kernel(const fd_gemm_params p, const int group_m) {
  // 8 waves (4 x 2) of 64 x 128: group 0 = waves 0-3 = tile rows [0, 128), group 1 = waves 4-7 = rows [128, 256);
  // wave w and w + 4 share a SIMD
  static_assert(NW == 8, "ping-pong needs two groups of four waves");
  typedef typename VecT<T>::v8 V8;
  constexpr int BM = 256, BN = 256, NTHR = 64 * NW, WAVES_N = 2, WAVES_M = NW / WAVES_N;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N, MT = WM / 16, NT = WN / 16;
  constexpr int NBUF = 2;                // K tiles of 64 in LDS
  constexpr int STAGE = (BM + BN) * 128;  // 64 KB: 512 rows of 64 k (128 B)
  constexpr int A_BYTES = BM * 128;
  constexpr int AI = BM / (8 * NW);      // 8-row DMA pieces of A (and of B) per wave per K tile
  constexpr int LDE = BN + 4;
  constexpr int EROWS = 128;
  constexpr int RED_OFF = ((EROWS * LDE * 4 + 15) / 16) * 16;  // GroupNorm statistics scratch (gn_part)
  constexpr int SMEM = 163840;
  static_assert(NBUF * STAGE <= SMEM && RED_OFF + 16 * NTHR <= SMEM, "LDS");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WAVES_N, wn = w % WAVES_N;
  const int M = p.M, N = p.N, K = p.K;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = N / BN;

  // block -> tile: XCD-contiguous chunks (bijective remap), tiles walked in groups of group_m tile rows
  const int pid = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  {
    const int gsz_full = group_m * tiles_n;
    const int grp = pid / gsz_full;
    const int first_m = grp * group_m;
    const int gsz = min(tiles_m - first_m, group_m);
    const int in_g = pid - grp * gsz_full;
    tm = first_m + in_g % gsz;
    tn = in_g / gsz;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = K / 64;

  const T* __restrict__ A = (const T*)p.A;
  const T* __restrict__ Bw = (const T*)p.B;
  const T* __restrict__ A2 = (const T*)p.A2;
  // this lane's 16 B of a DMA piece: row (lane >> 3) of an 8-row piece, LDS chunk (lane & 7) holding the source
  // chunk (lane & 7) ^ ((row >> 1) & 7).  Piece w + 8 i starts at row 8 (w + 8 i), so the tile row's bits 0-2 are
  // lane >> 3 and its bit 3 is w & 1, the same for all of this lane's pieces.
  const int lrow = lane >> 3, chunk = (lane & 7) ^ (((lrow >> 1) | ((w & 1) << 2)) & 7);

  // A rows of this lane's DMA pieces: plain GEMM -> row pointers; conv -> the output pixel (decoded per tap)
  const T* a_row[AI];
  int a_m[AI];  // conv: output row, -1 past M
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int m = m0 + (w + NW * i) * 8 + lrow;
    const int mm = m < M ? m : M - 1;
    a_m[i] = m < M ? m : -1;
    a_row[i] = CONV ? nullptr : A + (long long)mm * p.lda + chunk * 8;
  }
  int b_off[AI];  // element offsets of this lane's B rows (32-bit: fd_gemm256_try checks N * ldb < 2^31)
#pragma unroll
  for (int i = 0; i < AI; ++i) b_off[i] = (n0 + (w + NW * i) * 8 + lrow) * p.ldb + chunk * 8;
  const int Hl = p.upsample ? p.Hout : p.Hin, Wl = p.upsample ? p.Wout : p.Win;
  const bool up2 = p.upsample && Hl == 2 * p.Hin && Wl == 2 * p.Win;
  const int C1 = p.C1 > 0 ? p.C1 : p.Cin;

  constexpr int mode = FD_G256_DIAG;
  int g_key = -1;         // conv: (tap, source) of the gather offsets below; stage() runs in K order
  constexpr int ZP = -0x7fffffff - 1;  // g_off sentinel: the zero page (a real offset can be negative: A2 - C1)
  int g_off[AI];          // per DMA row: source pixel's channel-0 element offset for this tap, ZP = zero page
#pragma unroll
  for (int i = 0; i < AI; ++i) g_off[i] = ZP;
  auto stage = [&](int t) {  // K tile t = k [64 t, 64 t + 64) into buffer t % 2
    if (mode & 1) return;
    const int k0 = t * 64;
    unsigned char* sa = smem + (t & 1) * STAGE;
    if (CONV) {
      const int tap = k0 / p.Cin;
      const int c0 = k0 - tap * p.Cin;
      const bool second = (A2 != nullptr) && (c0 >= C1);
      const int key = tap * 2 + (int)second;
      if (key != g_key) {  // the im2col source rows change only with the tap (every Cin / 64 tiles): uniform
        g_key = key;
        const int ky = tap / 3, kx = tap - (tap / 3) * 3;
#pragma unroll
        for (int i = 0; i < AI; ++i) {
          const int mm = a_m[i] < 0 ? 0 : a_m[i];
          const int hw = p.Hout * p.Wout;
          const int img = mm / hw;
          const int rem = mm - img * hw;
          const int oy = rem / p.Wout, ox = rem - (rem / p.Wout) * p.Wout;
          const int iy = oy * p.stride - p.pad + ky, ix = ox * p.stride - p.pad + kx;
          const bool ok = a_m[i] >= 0 && iy >= 0 && iy < Hl && ix >= 0 && ix < Wl;
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
          const int pix = (img * p.Hin + py) * p.Win + px;
          // offset such that src + g_off + c0 addresses channel c0 of this tap's source pixel (32-bit:
          // fd_gemm256_try checks the image sizes)
          g_off[i] = ok ? (second ? pix * (p.Cin - C1) - C1 + chunk * 8 : pix * (int)p.lda + chunk * 8) : ZP;
        }
      }
      const T* srcb = second ? A2 : A;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const void* s_ = g_off[i] != ZP ? (const void*)(srcb + (g_off[i] + c0)) : (const void*)g_zero_page256;
        __builtin_amdgcn_global_load_lds(s_, LDS_PTR(sa + (w + NW * i) * 1024), 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < AI; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(a_row[i] + k0), LDS_PTR(sa + (w + NW * i) * 1024), 16, 0, 0);
    }
    unsigned char* sb = sa + A_BYTES;
#pragma unroll
    for (int i = 0; i < AI; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(Bw + (b_off[i] + k0)), LDS_PTR(sb + (w + NW * i) * 1024), 16, 0,
                                       FD_WLD_AUX);
  };

  const int fr = lane & 15, fg = lane >> 4;
  auto read_frags = [&](int t, int h, V8 (&af)[MT], V8 (&bf)[NT]) {
    if (mode & 2) return;
    const unsigned char* sa = smem + (t & 1) * STAGE;
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
      for (int ni = 0; ni < NT; ++ni) acc[mi][ni] = mfma16x16x32(af[mi], bf[ni], acc[mi][ni]);
  };

  // ---- ping-pong main loop (probes/gemm_pp.hip, 256 x 256 BK 64: 1453 TF at 4096^3 vs 1061 for the five-slot
  // single-group loop).  Every wave runs, per 32-deep K half, a LOAD segment (its fragment ds_reads; in the first
  // half its share of K tile t + 1 into the buffer tile t - 1 used; in the second half the wait for tile t + 1) and
  // a COMPUTE segment (lgkmcnt(0) + 32 MFMAs), each closed by a raw s_barrier; group 1 starts one barrier late, so
  // on every SIMD one wave's MFMAs run beside its partner's loads.  Buffer hazards: tile t - 1's buffer is last read
  // by group 1 in the load segment closed by the barrier that opens group 0's first load segment of tile t; tile
  // t + 1 has landed for every wave before the barrier closing group 1's second load segment of tile t, which
  // precedes group 0's first read of it.  K is summed in 32-deep halves in order, as before (and as gemm8): the
  // same bits.
  if (nk > 0) stage(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  const int grp = w >> 2;
  if (grp == 1) __builtin_amdgcn_s_barrier();  // the stagger
  V8 af[MT], bfr[NT];
  for (int t = 0; t < nk; ++t) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      read_frags(t, h, af, bfr);
      if (h == 0 && t + 1 < nk) stage(t + 1);
      if (h == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t + 1 landed (this wave's part)
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this half's fragments
      mma(af, bfr);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // re-align the groups

  // ---- epilogue: two 128-row passes through the drained ring
  if (mode & 4) {
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) asm volatile("" ::"v"(acc[mi][ni]));
    return;
  }
  __syncthreads();
  TO* __restrict__ C = (TO*)p.C;
  const TO* __restrict__ R = (const TO*)p.residual;
  const float* __restrict__ bias = p.bias;
  const float* __restrict__ rbias = p.rowbias;
  const float alpha = p.alpha;
  const int act = p.act;
  float* ep = (float*)smem;
  constexpr int VPR = BN / 8;
  constexpr int ITER = 2;  // batched row-phase loads (4 spills: the second pass's accumulators are still live)
  static_assert((EROWS * VPR) % (NTHR * ITER) == 0, "epilogue iterations");
  const bool vec = (p.ldc % 8 == 0) && ((((unsigned long long)C) & 15) == 0) &&
                   (!R || ((p.ldr % 8 == 0) && ((((unsigned long long)R) & 15) == 0))) &&
                   (!bias || ((((unsigned long long)bias) & 15) == 0)) &&
                   (!rbias || ((p.rowbias_ld % 4 == 0) && ((((unsigned long long)rbias) & 15) == 0)));
  const bool interior = vec && (m0 + BM <= M);
  typedef __attribute__((ext_vector_type(8))) TO TO8;
  // GroupNorm statistics (fd_gemm_params.gn_part; host: interior, group-aligned tiles): chunk tid % VPR per thread
  const bool gn = p.gn_part != nullptr;
  const int gcpg = gn ? p.N / p.gn_groups : 8;
  const int gsplit = (((tid % VPR) * 8) / gcpg + 1) * gcpg - (tid % VPR) * 8;
  GnTile gna;
#pragma unroll 1
  for (int half = 0; half < BM / EROWS; ++half) {
    if (half) __syncthreads();  // the previous half's staging fully consumed
    if ((wm * WM) / EROWS == half) {
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int rl = wm * WM + mi * 16 + fg * 4 - half * EROWS;
#pragma unroll
        for (int ni = 0; ni < NT; ++ni) {
          const int col = wn * WN + ni * 16 + fr;
#pragma unroll
          for (int j = 0; j < 4; ++j) ep[(rl + j) * LDE + col] = acc[mi][ni][j] * alpha;
        }
      }
    }
    __syncthreads();
    if (interior) {
#pragma unroll 1
      for (int e0 = 0; e0 < EROWS * VPR; e0 += NTHR * ITER) {
        float v[ITER][8], bv[ITER][8], rv[ITER][8];
        TO8 res[ITER];
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
          const int e = e0 + tid + it * NTHR;
          const int r = e / VPR, cv = e % VPR;
          const int m = m0 + half * EROWS + r, n = n0 + cv * 8;
          *(f32x4*)&v[it][0] = *(const f32x4*)(ep + r * LDE + cv * 8);
          *(f32x4*)&v[it][4] = *(const f32x4*)(ep + r * LDE + cv * 8 + 4);
          if (bias) {
            *(f32x4*)&bv[it][0] = *(const f32x4*)(bias + n);
            *(f32x4*)&bv[it][4] = *(const f32x4*)(bias + n + 4);
          }
          if (rbias) {
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
          const int m = m0 + half * EROWS + r, n = n0 + cv * 8;
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
          if (R) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[it][i] += (float)res[it][i];
          }
          TO8 o;
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = (TO)v[it][i];
          st_out16((TO8*)(C + (long long)m * p.ldc + n), o);
          if (gn) gna.add(o, gsplit);
        }
      }
    } else {  // ragged last row tile / unaligned operands: scalar, bounds-checked
      for (int e = tid; e < EROWS * VPR; e += NTHR) {
        const int r = e / VPR, cv = e % VPR;
        const int m = m0 + half * EROWS + r, n = n0 + cv * 8;
        if (m >= M) continue;
        for (int i = 0; i < 8; ++i) {
          float x = ep[r * LDE + cv * 8 + i];
          if (bias) x += bias[n + i];
          if (rbias) x += rbias[(long long)(m / p.rows_per_group) * p.rowbias_ld + n + i];
          x = act_f(x, act);
          if (R) x += (float)R[(long long)m * p.ldr + n + i];
          C[(long long)m * p.ldc + n + i] = (TO)x;
        }
      }
    }
  }
  if (gn) gn_tile_write(gna, (float2*)(smem + RED_OFF), tid, NTHR, VPR, gcpg, BN, n0, m0, p);
}

}  // namespace

// Whether fd_gemm256_try takes this launch (also asked by the halo-staged conv's planner, which leaves these convs
// to this kernel).
int gemm256_takes(const fd_gemm_params* p) {
  const int min_tiles = fd_knob(FDK_GEMM256_MIN_TILES);
  const int enabled = fd_knob(FDK_GEMM256);  // tests compare against gemm8 in one process
  if (!enabled || p->batch > 1 || p->act == FD_ACT_GEGLU || p->ln_in || p->ln_out || p->N % 256 || p->K % 32 ||
      p->bsel_rows > 0 || p->act == FD_ACT_SOFTMAX)
    return 0;
  if (p->conv && (p->Cin % 32 || (p->C1 > 0 && p->C1 % 32))) return 0;
  const int m_ref = p->m_ref > 0 ? p->m_ref : p->M;
  if ((long long)((m_ref + 255) / 256) * (p->N / 256) < min_tiles) return 0;
  if (p->K % 64 || (p->conv && (p->Cin % 64 || (p->C1 > 0 && p->C1 % 64)))) return 0;  // 64-deep K tiles
  // 32-bit element offsets inside the kernel (B rows; conv source pixels)
  if ((long long)p->N * p->ldb >= (1LL << 31)) return 0;
  if (p->conv && (long long)p->nimg * p->Hin * p->Win * (p->lda > p->Cin ? p->lda : p->Cin) >= (1LL << 31)) return 0;
  return 1;
}

// Returns 1 and launches when this kernel takes the GEMM, 0 when it does not apply, < 0 on error.  Taken for
// N % 256 == 0, no GEGLU / LayerNorm fold / batching, and at least 192 tiles of 256 x 256 counted from the
// per-TLC-tile row count m_ref (so batching tiles never changes the kernel choice: bitwise batch-invariant).
// Knob FD_GEMM256 = 0 disables it (tests: the bitwise gemm8 comparison).
extern "C" int fd_gemm256_try(fd_gemm_params* p0, void* stream) {
  fd_gemm_params q = *p0;  // the kernel's copy: gn_part kept only where the statistics can be written
  {
    const fd_gemm_params* p = p0;
    bool ok = p->gn_part && p->gn_groups > 0 && p->gn_hw > 0 && p->N % p->gn_groups == 0;
    if (ok) {
      const int cpg = p->N / p->gn_groups;
      const unsigned long long al = (unsigned long long)p->C | (p->residual ? (unsigned long long)p->residual : 0) |
                                    (p->bias ? (unsigned long long)p->bias : 0) |
                                    (p->rowbias ? (unsigned long long)p->rowbias : 0);
      ok = cpg >= 4 && 256 % cpg == 0 && p->M % 256 == 0 && p->gn_hw % 256 == 0 && p->M % p->gn_hw == 0 &&
           (al & 15) == 0 && p->ldc % 8 == 0 && (!p->residual || p->ldr % 8 == 0) &&
           (!p->rowbias || p->rowbias_ld % 4 == 0);
    }
    if (!ok) q.gn_part = nullptr;
  }
  const fd_gemm_params* p = &q;
  if (!gemm256_takes(p)) return 0;
  const int tiles_m = (p->M + 255) / 256, tiles_n = p->N / 256;
  const long long tiles = (long long)tiles_m * tiles_n;
  if (tiles > 0x7fffffff) return FD_ERR_SHAPE;
  // group_m: per-XCD chunk of tiles/8; the tile-row group height minimising that chunk's A rows + B columns
  int gm = 1;
  {
    const long long per_xcd = (tiles + 7) / 8;
    double bestc = 1e30;
    for (int g = 1; g <= tiles_m; g *= 2) {
      const long long cols = per_xcd < g ? 1 : (per_xcd + g - 1) / g;
      const long long rows = per_xcd < g ? per_xcd : g;
      const double c = rows * 256.0 + (cols < tiles_n ? cols : tiles_n) * 256.0;
      if (c < bestc - 1e-9) {
        bestc = c;
        gm = g;
      }
    }
  }
  hipStream_t s = (hipStream_t)stream;
  // eight waves: the 4-wave (one 128 x 128 wave per SIMD) instance measured 1.3-1.4x slower on the convs
  dim3 grid((unsigned)tiles), block(512);
  int rc = FD_OK;
  FD_DISPATCH_T(p->dtype, FD_DISPATCH_O(p->out_dtype, {
    if (p->conv)
      hipLaunchKernelGGL((gemm256_kernel<T, TO, true, 8>), grid, block, 0, s, *p, gm);
    else
      hipLaunchKernelGGL((gemm256_kernel<T, TO, false, 8>), grid, block, 0, s, *p, gm);
  }));
  FD_LAUNCH_CHECK();
  if (rc == FD_OK) p0->gn_done = q.gn_part != nullptr ? 256 : 0;
  return rc == FD_OK ? 1 : rc;
}
