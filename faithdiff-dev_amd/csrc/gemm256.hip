// 256 x 256-tile MFMA GEMM / implicit-GEMM convolution for gfx950, for the large-M launches (the VAE decoder's and
// encoders' 256- and 512-channel convs at 256^2..1024^2, the upsample convs): one workgroup per CU.
//
// Why: the 256 x 128 eight-wave kernel (gemm8.hip) is bound by the per-CU operand stream into LDS, not by the
// MFMA pipe (scripts/diag_probe.sh: its load-only build takes 70-90 % of the full time, its compute-only build
// ~50 %).  A 256 x 256 tile needs 32 KB of operands per 4.2 MFLOP (131 flop/B) instead of 48 KB (85 flop/B).
// The ring holds K slots of 32 (256 + 256 rows x 64 B = 32 KB per slot), five slots = all 160 KiB of LDS, so up to
// four slots (128 KB) are in flight while one is read -- more bytes in flight than gemm8's two 48 KB stages.
//
// Structure: 512 threads = 8 waves (4 x 2), each a 64 x 128 sub-tile of v_mfma_f32_16x16x32 (32 accumulators);
// per slot one counted s_waitcnt vmcnt (the next slot has landed) + one raw s_barrier, then the next
// slot's LDS-DMA refill and the next slot's fragment reads under this slot's 32 MFMAs (register double-buffered
// fragments).  64-B LDS rows with a source-side XOR swizzle (16-B chunk ^ ((row >> 2) & 3)): the 16-row
// ds_read_b128 fragments are conflict-free.  K is summed in 32-deep slots in order, the same order as gemm8's
// two 32-deep halves per 64-deep step, so both kernels give the same bits.  Conv: im2col gather from NHWC with
// out-of-image taps on a zero page, exact-x2 / diffusers upsample and two-source channel concat folded in.
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

template <int N>
__device__ __forceinline__ void vm_wait256() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <typename T, typename TO, bool CONV, int NW>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(1, NW == 4 ? 1 : 2)))
gemm256_kernel(const fd_gemm_params p, const int group_m) {
  // NW = 8: 4 x 2 waves of 64 x 128, two waves per SIMD; NW = 4: 2 x 2 waves of 128 x 128, one wave per SIMD
  // (a third fewer fragment bytes read from LDS per slot; 512-VGPR waves)
  typedef typename VecT<T>::v8 V8;
  constexpr int BM = 256, BN = 256, NTHR = 64 * NW, WAVES_N = 2, WAVES_M = NW / WAVES_N;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N, MT = WM / 16, NT = WN / 16;
  constexpr int AI = 16 / NW;            // 16-row DMA blocks of A (and of B) per wave per slot
  constexpr int NSL = 5;                 // ring slots
  constexpr int SLOT = (BM + BN) * 64;   // 32 KB: 512 rows of 32 k
  constexpr int A_BYTES = BM * 64;
  constexpr int PER = 2 * AI;            // LDS-DMA instructions per wave per slot (A + B, 16 rows each)
  constexpr int LDE = BN + 4;
  constexpr int EROWS = 128;
  static_assert(EROWS * LDE * 4 <= NSL * SLOT, "epilogue staging");
  constexpr int RED_OFF = ((EROWS * LDE * 4 + 15) / 16) * 16;  // GroupNorm statistics scratch (gn_part)
  static_assert(RED_OFF + 16 * NTHR <= NSL * SLOT, "GroupNorm reduction scratch");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NSL * SLOT];

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
  const int nsl = K / 32;

  const T* __restrict__ A = (const T*)p.A;
  const T* __restrict__ Bw = (const T*)p.B;
  const T* __restrict__ A2 = (const T*)p.A2;
  // this lane's 16 B of a DMA instruction: row (lane >> 2) of a 16-row block, LDS chunk (lane & 3) holding the
  // source chunk (lane & 3) ^ ((row >> 2) & 3) = (lane & 3) ^ (lane >> 4)
  const int lrow = lane >> 2, chunk = (lane & 3) ^ (lane >> 4);

  // A rows of this lane's DMA pieces: plain GEMM -> row pointers; conv -> the output pixel (decoded per tap)
  const T* a_row[AI];
  int a_m[AI];  // conv: output row, -1 past M
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int m = m0 + (w + NW * i) * 16 + lrow;
    const int mm = m < M ? m : M - 1;
    a_m[i] = m < M ? m : -1;
    a_row[i] = CONV ? nullptr : A + (long long)mm * p.lda + chunk * 8;
  }
  int b_off[AI];  // element offsets of this lane's B rows (32-bit: fd_gemm256_try checks N * ldb < 2^31)
#pragma unroll
  for (int i = 0; i < AI; ++i) b_off[i] = (n0 + (w + NW * i) * 16 + lrow) * p.ldb + chunk * 8;
  const int Hl = p.upsample ? p.Hout : p.Hin, Wl = p.upsample ? p.Wout : p.Win;
  const bool up2 = p.upsample && Hl == 2 * p.Hin && Wl == 2 * p.Win;
  const int C1 = p.C1 > 0 ? p.C1 : p.Cin;

  constexpr int mode = FD_G256_DIAG;
  int g_key = -1;         // conv: (tap, source) of the gather offsets below; stage() runs in slot order
  constexpr int ZP = -0x7fffffff - 1;  // g_off sentinel: the zero page (a real offset can be negative: A2 - C1)
  int g_off[AI];          // per DMA row: source pixel's channel-0 element offset for this tap, ZP = zero page
#pragma unroll
  for (int i = 0; i < AI; ++i) g_off[i] = ZP;
  auto stage = [&](int s, int buf) {  // slot s = k [32 s, 32 s + 32)
    if (mode & 1) return;
    const int k0 = s * 32;
    unsigned char* sa = smem + buf * SLOT;
    if (CONV) {
      const int tap = k0 / p.Cin;
      const int c0 = k0 - tap * p.Cin;
      const bool second = (A2 != nullptr) && (c0 >= C1);
      const int key = tap * 2 + (int)second;
      if (key != g_key) {  // the im2col source rows change only with the tap (every Cin / 32 slots): uniform
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
                                       0);
  };
  // all but this wave's youngest `ahead` slots have landed (ahead <= NSL - 1)
  auto wait_ahead = [&](int ahead) {
    if (ahead >= 4) vm_wait256<4 * PER>();
    else if (ahead == 3) vm_wait256<3 * PER>();
    else if (ahead == 2) vm_wait256<2 * PER>();
    else if (ahead == 1) vm_wait256<PER>();
    else vm_wait256<0>();
  };

  const int fr = lane & 15, fg = lane >> 4;
  const int rd_off = fr * 64 + ((fg ^ (fr >> 2)) << 4);  // row fr of a 16-row block, logical chunk fg
  auto read_frags = [&](int buf, V8 (&af)[MT], V8 (&bf)[NT]) {
    if (mode & 2) return;
    const unsigned char* sa = smem + buf * SLOT + rd_off;
    const unsigned char* sb = sa + A_BYTES;
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) af[mi] = *(const V8*)(sa + (wm * WM + mi * 16) * 64);
#pragma unroll
    for (int ni = 0; ni < NT; ++ni) bf[ni] = *(const V8*)(sb + (wn * WN + ni * 16) * 64);
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

  // prologue: slots 0..NSL-1 in flight, slot 0 landed and visible, its fragments read
#pragma unroll
  for (int s0 = 0; s0 < NSL; ++s0)
    if (s0 < nsl) stage(s0, s0);
  wait_ahead(min(nsl - 1, NSL - 1));
  __builtin_amdgcn_s_barrier();
  V8 a0[MT], b0[NT], a1[MT], b1[NT];
  read_frags(0, a0, b0);
  // slot s (its fragments already in registers): wait for slot s+1 (this wave's DMA; slots s+2..s+4 may fly) and
  // for this wave's reads of slot s; barrier (slot s+1 visible, every wave done reading slot s); refill slot s's
  // buffer with slot s+NSL (four slots in flight); slot s+1's fragment reads under slot s's MFMAs.
  auto step = [&](int s, V8 (&ac)[MT], V8 (&bc)[NT], V8 (&an)[MT], V8 (&bn)[NT]) {
    if (s + 1 < nsl) {
      wait_ahead(min(NSL - 2, nsl - 2 - s));
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's reads of slot s retired
      __builtin_amdgcn_s_barrier();
      if (s + NSL < nsl) stage(s + NSL, s % NSL);
      read_frags((s + 1) % NSL, an, bn);
    } else {
      __builtin_amdgcn_s_waitcnt(0xc07f);
    }
    mma(ac, bc);
#pragma unroll
    for (int i = 0; i < MT + NT; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, MT * NT - (MT + NT), 0);
  };
  int s = 0;
  for (; s + 1 < nsl; s += 2) {
    step(s, a0, b0, a1, b1);
    step(s + 1, a1, b1, a0, b0);
  }
  if (s < nsl) step(s, a0, b0, a1, b1);

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
          *(TO8*)(C + (long long)m * p.ldc + n) = o;
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

int env256(const char* n, int d) {
  const char* v = getenv(n);
  return v ? atoi(v) : d;
}

}  // namespace

// Returns 1 and launches when this kernel takes the GEMM, 0 when it does not apply, < 0 on error.  Taken for
// N % 256 == 0, no GEGLU / LayerNorm fold / batching, and at least 192 tiles of 256 x 256 counted from the
// per-TLC-tile row count m_ref (so batching tiles never changes the kernel choice: bitwise batch-invariant).
// FD_GEMM256=0 disables it (A/B timing).
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
  static int min_tiles = -1;
  if (min_tiles < 0) min_tiles = env256("FD_GEMM256_MIN_TILES", 192);
  const int enabled = env256("FD_GEMM256", 1);  // read per call: tests compare against gemm8 in one process
  if (!enabled || p->batch > 1 || p->act == FD_ACT_GEGLU || p->ln_in || p->ln_out || p->N % 256 || p->K % 32)
    return 0;
  if (p->conv && (p->Cin % 32 || (p->C1 > 0 && p->C1 % 32))) return 0;
  const int m_ref = p->m_ref > 0 ? p->m_ref : p->M;
  if ((long long)((m_ref + 255) / 256) * (p->N / 256) < min_tiles) return 0;
  // 32-bit element offsets inside the kernel (B rows; conv source pixels)
  if ((long long)p->N * p->ldb >= (1LL << 31)) return 0;
  if (p->conv && (long long)p->nimg * p->Hin * p->Win * (p->lda > p->Cin ? p->lda : p->Cin) >= (1LL << 31)) return 0;
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
  if (rc == FD_OK) p0->gn_done = q.gn_part != nullptr;
  return rc == FD_OK ? 1 : rc;
}
