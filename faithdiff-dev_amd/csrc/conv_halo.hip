// 3x3 stride-1 convolution on a halo-staged input patch, with the consumer GroupNorm (+ SiLU) applied in the
// staging pass (gfx950).
//
// Why: the implicit-GEMM conv (gemm8 / gemm256) gathers its A operand per tap, so every input pixel crosses the
// CU's L2 -> LDS path 9 times (once per tap) -- at the UNet's 128^2 / 64^2 levels and in the VAE that stream, not the
// MFMA pipe, bounds the convs (conv counter traffic ~2.3x the activations + weights) -- and the
// GroupNorm (+ SiLU) in front of every resnet conv is a separate read + write pass of the activation.  Here a
// workgroup owns a TH x 16 output-pixel tile and BN output channels; per 64-channel chunk it stages the
// (TH + 2) x 18 input patch into LDS ONCE (1.27x / 1.41x the tile's pixels instead of 9x), applies the GroupNorm
// affine (+ SiLU) to the staged values in place (once per element per workgroup, not per tap and wave), and runs
// the chunk's 9 taps as 9 MFMA K steps that read shifted windows of the patch.  Weights stream through a 3-deep
// LDS ring of (tap, chunk) stages as in gemm8.
//
// Roles: waves 0-3 DMA the weight stages (global_load_lds, counted vmcnt); waves 4-7 DMA the patches (two patch
// buffers: chunk c + 2 is issued right after the last read of chunk c, waited for 8 steps later); all 8 waves
// compute (4 x 2 waves of (TH * 4) x (BN / 2)).  Out-of-image pixels come from a zero page and are written as zero
// by the affine pass (the reference pads the normalised activation, not the raw one).
//
// Numerics: the staged values are exactly the bf16 / fp16 values fd_group_norm would store (same fma, SiLU and
// rounding), and the sum over K runs chunk by chunk, tap by tap inside the chunk -- per output element the same
// order whatever the tile shape (TH 16 or 8, BN 160 or 128), so tile choices never change a bit; it differs from
// the implicit GEMM's tap-major order (not bitwise equal to gemm8, tested against fp32).
#include <type_traits>
#include <utility>

#include "fd_common.h"

__device__ __attribute__((aligned(256))) unsigned char g_zero_halo[256];
// split-K hand-off health of the channel-split form (as gemm8.hip: timed-out pairwise waits, test hook)
__device__ unsigned g_halo_sk_timeouts;
__device__ unsigned g_halo_sk_drop;

#ifndef FD_HALO_CT
#define FD_HALO_CT 1
#endif
// diagnostic builds only (-DFD_HALO_DIAG=m, wrong answers; 0 in the product), CT K loop: 1 = no DMA waits, 2 = no
// MFMAs (fragments still read), 4 = no DMA issued after the prologue, 8 = no barriers, 16 = no fragment reads,
// 32 = no K loop at all (prologue DMA + wait, epilogue)
#ifndef FD_HALO_DIAG
#define FD_HALO_DIAG 0
#endif
// ping-pong K loop (build-time A/B): first tap of the GroupNorm transform pieces; s_setprio(1) for waves 4-7
#ifndef FD_HALO_PP_TR
#define FD_HALO_PP_TR 5
#endif
#ifndef FD_HALO_PP_PRIO
#define FD_HALO_PP_PRIO 0
#endif

namespace {

template <int... I, typename F>
__device__ __forceinline__ void halo_static_for(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>()), ...);
}

template <int N>
__device__ __forceinline__ void hvm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

constexpr int PW = 18;  // patch width: 16 output columns + halo
// Patch LDS layout: pixel pix = py * PW + px at pix * 128 B, its 16-B channel chunk j at chunk slot j ^ ((px >> 1) & 7).
// The XOR depends on the pixel's COLUMN only (PW * 128 B = 9 x 256 B, so the row never changes the bank): a fragment
// read for tap (ky, kx) is then a per-lane offset of (kx, K half) plus an immediate (row, chunk buffer), with no
// address arithmetic in the K loop (the per-step LDS address VALU had made the loop VALU-issue-bound, r05).
constexpr int TR = 4;   // tap of chunk c at which chunk c + 1's patch is waited for
constexpr int NPART = 8 - TR;  // ... and transformed in NPART pieces at taps TR .. 7 (published by tap 8's barrier)

// LDS-only workgroup barrier: this wave's LDS operations retired, then s_barrier.  Unlike __syncthreads() it does
// not drain vector memory, so LDS-DMA and stores issued before it stay in flight (the PT epilogue relies on that).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// PT (persistent tiles): one workgroup per CU walks a strided list of tiles inside its XCD's contiguous share; the
// epilogue stages 32-row passes in an LDS region of its own past the ring, so the next tile's weight stages and
// patches are DMA'd while this tile's outputs are written (the non-PT form waits for its patches at the start of
// every tile and stores at the end with nothing to overlap either: at the VAE's 1024^2 level that was ~1/3 of the
// conv).  The per-element K order, the stored values and the GroupNorm partials are bit for bit the non-PT ones.
//
// PH (the nearest x2 upsample conv, Upsample2D, in four phases): output pixel (2i + a, 2j + b) of conv3x3(up2(x))
// reads only source rows i + a - 1 + {0, 1} and columns j + b - 1 + {0, 1}, so each phase (a, b) is a 2 x 2 conv
// of the LOW-resolution x with weights summed over the taps that land on the same source pixel
// (pack_conv3x3_up2: [4 * Cout][4 * Cin]) -- 16 taps per 2 x 2 output pixels instead of 36.  The tiles cover the
// low-resolution grid; the combined N = 4 * Cout is phase-major (an N tile never straddles two phases); a tile's
// 4 taps read the window at rows a + {0, 1}, columns b + {0, 1} of its (TH + 2) x 18 patch, and its epilogue writes
// the strided output pixels.  GroupNorm partials: one block per (image, phase, tile) -- 256 output pixels each.
//
// PP (ping-pong K loop, every form but PT): the 8 waves run as two groups of four -- group 0 = waves 0-3 = the
// tile's rows [0, BM / 2), group 1 = waves 4-7 = rows [BM / 2, BM); waves w and w + 4 share a SIMD -- and group 1
// starts one barrier late, so on every SIMD one wave issues its MFMAs while its partner reads fragments, issues
// LDS-DMA and transforms the next chunk's patch (the gemm256 scheme).  Per K step (one tap of one chunk) a wave runs
// a LOAD segment (both halves' fragments of the step) and a COMPUTE segment (the step's MFMAs, half 0 then half 1),
// each closed by a raw s_barrier.  Same per-element K order as the one-barrier loop: the same bits.
template <typename T, int TH, int BN, bool GNI, bool SK, int NS, bool PT, bool PH, bool PP>
__global__ void __launch_bounds__(512) conv_halo_kernel(const fd_gemm_params p, float* __restrict__ slabs,
                                                          unsigned* __restrict__ counters) {
  typedef typename VecT<T>::v8 V8;
  typedef __attribute__((ext_vector_type(8))) T TO8;
  constexpr int BM = TH * 16;
  constexpr int PIX = (TH + 2) * PW;
  constexpr int PIXR = (PIX + 7) / 8 * 8;
  constexpr int PATCH = PIXR * 128;
  constexpr int AFF = GNI ? 1024 : 0;  // the chunk's 64 affine pairs (512 B, DMA'd as 1 KB) after each patch
  constexpr int PBUF = PATCH + AFF;
  static_assert(NS >= 3 && NS <= 5, "weight ring depth");
  constexpr int STAGE = BN * 128;
  constexpr int RING = 2 * PBUF;
  constexpr int SMEM_MAIN = RING + NS * STAGE;
  constexpr int WM = BM / 4, WN = BN / 2;
  constexpr int MT = WM / 16, NT = WN / 16;
  constexpr int B_TOT = BN / 8, PER_B = B_TOT / 4;
  static_assert(B_TOT % 4 == 0, "B stage split over 4 waves");
  constexpr int P_TOT = PIXR / 8, P_I = (P_TOT + 3) / 4;
  constexpr int EROWS = 128, LDE = BN + 4, EPB = EROWS * LDE * 4, VPR = BN / 8;
  constexpr int SLOT = EPB, RED = SLOT + EROWS * VPR * 16;
  constexpr int SMEM_EPI = RED + 512 * 8;
  constexpr int PER = 32;  // PT epilogue pass: 32 rows x BN fp32 + their GroupNorm slots, past the ring
  constexpr int PT_EP = SMEM_MAIN, PT_SLOT = PT_EP + PER * LDE * 4, PT_END = PT_SLOT + PER * VPR * 16;
  static_assert(!PH || (!GNI && !SK && !PT), "phase form: plain tiles only");
  static_assert(!(PP && PT), "ping-pong loop: per-tile forms");
  constexpr int NTAP = PH ? 4 : 9;
  // lane-constant LDS read bases in the K loop (below): every tile form but the persistent and the phase ones
  constexpr bool CT = !PH && FD_HALO_CT;
  static_assert(!PT || (!SK && BN == 128 && TH == 16 && PER * VPR == 512 && PT_END <= 163840 &&
                        PER * LDE * 4 >= 512 * 8),
                "PT layout: one 8-column vector per thread per pass, red[] in the pass buffer");
  constexpr int SMEM = PT ? PT_END : (SMEM_MAIN > SMEM_EPI ? SMEM_MAIN : SMEM_EPI);
  static_assert(SMEM <= 163840, "LDS");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const int Ho = p.Hout, Wo = p.Wout, Cin = p.Cin, N = p.N;
  const int Hg = PH ? p.Hin : Ho, Wg = PH ? p.Win : Wo;  // the tiled (and patch) grid
  const int tiles_x = (Wg + 15) / 16, tiles_y = (Hg + TH - 1) / TH;
  const int nsp = p.nimg * tiles_y * tiles_x;
  // tile order: XCD-contiguous chunks (bijective remap), output-channel tiles outer, so the ~32 workgroups an XCD
  // runs at once share one weight panel in its L2; SK: the two channel halves of a tile adjacent (same XCD)
  const int pid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = SK ? (pid & 1) : 0, tlin = SK ? (pid >> 1) : pid;
  // this workgroup's tiles: tl, tl + tl_step, ... < tl_hi (non-PT: the one tile tlin).  PT: workgroups b and b + 8
  // share an XCD (blocks are dealt round-robin), so XCD b % 8 takes the contiguous eighth [lo, hi) of the tile
  // order and its gx workgroups stride it -- the ~32 tiles an XCD holds at once are neighbours sharing halo rows
  int tl = tlin, tl_hi = tlin + 1, tl_step = 1;
  if constexpr (PT) {
    const int total = ((PH ? 4 : 1) * N / BN) * nsp, xcd = blockIdx.x & 7;
    tl = (int)((long long)xcd * total / 8) + (blockIdx.x >> 3);
    tl_hi = (int)((long long)(xcd + 1) * total / 8);
    tl_step = gridDim.x >> 3;
    if (tl >= tl_hi) return;
  }
  // input-channel chunks of this workgroup: all, or (SK) one half of them, combined pairwise after the K loop
  const int nch_all = Cin / 64;
  const int cb = SK && split ? nch_all / 2 : 0, ce = SK && !split ? nch_all / 2 : nch_all;
  const int nsteps = NTAP * (ce - cb);
  const T* __restrict__ A = (const T*)p.A;
  const T* __restrict__ Bw = (const T*)p.B;
  const bool up2 = p.upsample && Ho == 2 * p.Hin && Wo == 2 * p.Win;
  const bool ups = !PH && p.upsample;  // nearest resize folded into the patch gather (PH: the patch is low-res)

  // ---- per-tile coordinates and DMA sources.  Weight stages (waves 0-3): rows n0 + (w + 4 i) * 8 + lane / 8,
  // source-side XOR swizzle of 128-B rows; patch pixels (waves 4-7): this lane's source 16-B chunk at channel 0,
  // nullptr = outside the image.  Non-PT: computed once into registers.  PT: recomputed at each DMA issue from the
  // (wave-uniform) tile coordinates, which keeps ~30 VGPRs of pointers out of the epilogue, and rows past the patch
  // (j >= P_TOT) re-load row P_TOT - 1 (the same bytes to the same LDS address), so every patch wave issues exactly
  // P_I loads per chunk and the epilogue's counted waits hold
  int img = 0, spi = 0, y0 = 0, x0 = 0, n0 = 0, nb = 0, pha = 0, phb = 0;  // nb: B row base (PH: phase-major)
  const T* b_row[PT ? 1 : PER_B];
  // PSRC_RE: patch sources recomputed at each DMA issue instead of held in 2 * P_I VGPRs across the K loop (PT)
  constexpr bool PSRC_RE = PT;
  const T* p_src[PSRC_RE ? 1 : P_I];
  const float* __restrict__ aff = nullptr;
  auto b_src = [&] __attribute__((always_inline)) (int i) {
    int row = (w + 4 * i) * 8 + (lane >> 3);
    if constexpr (PT) asm volatile("" : "+v"(row));
    return Bw + (long long)(nb + row) * p.ldb + (((lane & 7) ^ ((row >> 1) & 7)) * 8);
  };
  auto p_row = [&] __attribute__((always_inline)) (int i) { return PT ? min((w - 4) + 4 * i, P_TOT - 1) : (w - 4) + 4 * i; };
  auto p_src_at = [&] __attribute__((always_inline)) (int i, int img_, int y0_, int x0_) -> const T* {
    const int j = p_row(i);
    int pix = j * 8 + (lane >> 3);
    if constexpr (PSRC_RE) asm volatile("" : "+v"(pix));  // recomputed at each issue, never hoisted out of the loops
    const int py = pix / PW, px = pix - (pix / PW) * PW;
    const int iy = y0_ - 1 + py, ix = x0_ - 1 + px;
    const bool ok = j < P_TOT && pix < PIX && iy >= 0 && iy < Hg && ix >= 0 && ix < Wg;
    int sy = iy, sx = ix;
    if (ups) {
      sy = up2 ? (iy >> 1) : (iy * p.Hin) / Ho;
      sx = up2 ? (ix >> 1) : (ix * p.Win) / Wo;
    }
    return ok ? A + ((long long)(img_ * p.Hin + sy) * p.Win + sx) * p.lda + (((lane & 7) ^ ((px >> 1) & 7)) * 8)
              : nullptr;
  };
  auto p_src_of = [&] __attribute__((always_inline)) (int i) -> const T* { return p_src_at(i, img, y0, x0); };
  auto setup = [&] __attribute__((always_inline)) (int tile) {
    // tile order: output-channel tiles outer (the ~32 workgroups an XCD holds share one weight panel in its L2).
    // PH: the 4 x Cout / BN column tiles come in groups of G whose weight panels fit together in ~2 MB of L2, the
    // G tiles of one group and spatial tile adjacent -- the low-resolution patch is then fetched once per group
    // instead of once per column tile (the 1024^2 upsample conv: 8 column tiles, all in one group)
    int nt, sp;
    if constexpr (PH) {
      const int ntn = 4 * N / BN;
      const long long panel = (long long)BN * p.K * 2;
      int g = (int)min((long long)ntn, max(1LL, (2LL << 20) / panel));
      while (ntn % g) --g;
      const int ntg = tile / (nsp * g), rem = tile - ntg * (nsp * g);
      sp = rem / g;
      nt = ntg * g + (rem - sp * g);
    } else {
      nt = tile / nsp;
      sp = tile - nt * nsp;
    }
    img = sp / (tiles_y * tiles_x);
    spi = sp - img * (tiles_y * tiles_x);
    const int tyt = spi / tiles_x, txt = spi - tyt * tiles_x;
    y0 = tyt * TH;
    x0 = txt * 16;
    nb = nt * BN;
    const int ph = PH ? nb / N : 0;
    pha = ph >> 1;
    phb = ph & 1;
    n0 = nb - ph * N;
    if constexpr (!PT) {
      if (w < 4) {
#pragma unroll
        for (int i = 0; i < PER_B; ++i) b_row[i] = b_src(i);
      } else if constexpr (!PSRC_RE) {
#pragma unroll
        for (int i = 0; i < P_I; ++i) p_src[i] = p_src_of(i);
      }
    }
    if (GNI) aff = (const float*)p.gi_affine + (long long)img * Cin * 2;
  };

  auto stage_b = [&] __attribute__((always_inline)) (int s, int rb) {  // s: this workgroup's step (chunk cb + s / 9, tap s % 9)
    const int c = cb + s / NTAP, t = s - (s / NTAP) * NTAP;
    const int off = t * Cin + c * 64;
    unsigned char* dst = smem + RING + rb * STAGE;
#pragma unroll
    for (int i = 0; i < PER_B; ++i)
      __builtin_amdgcn_global_load_lds((const void*)((PT ? b_src(i) : b_row[PT ? 0 : i]) + off),
                                       LDS_PTR(dst + (w + 4 * i) * 1024), 16, 0, FD_WLD_AUX);
  };
  // patch of chunk c of the tile at (img_, y0_, x0_) into buffer c & 1 (+ its affine table; aff_: that tile's image)
  auto stage_p_at = [&] __attribute__((always_inline)) (int c, int img_, int y0_, int x0_, const float* aff_) {
    unsigned char* dst = smem + (c & 1) * PBUF;
#pragma unroll
    for (int i = 0; i < P_I; ++i) {
      const int j = p_row(i);
      if (PT || j < P_TOT) {
        const T* src = PSRC_RE ? p_src_at(i, img_, y0_, x0_) : p_src[PSRC_RE ? 0 : i];
        const void* s = src ? (const void*)(src + c * 64) : (const void*)g_zero_halo;
        __builtin_amdgcn_global_load_lds(s, LDS_PTR(dst + j * 1024), 16, 0, 0);
      }
    }
    // 64 channels x (scale, shift) = 512 B; the upper half of the 1 KB is never read.  PT: every patch wave loads it
    // (identical bytes), for the uniform DMA count
    if (GNI && (PT || w == 4))
      __builtin_amdgcn_global_load_lds((const void*)(aff_ + (long long)c * 128 + lane * 4), LDS_PTR(dst + PATCH), 16, 0,
                                       0);
  };
  auto stage_p = [&] __attribute__((always_inline)) (int c) { stage_p_at(c, img, y0, x0, aff); };
  // GroupNorm affine (+ SiLU) in place on patch buffer c & 1: y = silu(fma(x, a, b)) rounded to T (fd_group_norm's
  // bits), zero outside the image.  Each thread keeps one logical 8-channel slot (tid % 8) for every pixel.  Piece
  // `part` of `nparts` covers pixels [part * PIX / nparts, (part + 1) * PIX / nparts): the main loop transforms the
  // next chunk's patch a piece per tap, issued behind that tap's MFMAs so the VALU work runs under them.
  auto transform = [&] __attribute__((always_inline)) (int c, int part, auto npc) {
    constexpr int NP = decltype(npc)::value;
    unsigned char* buf = smem + (c & 1) * PBUF;
    const int lc = tid & 7;
    const float* ab = (const float*)(buf + PATCH) + lc * 16;
    float a[8], b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[i] = ab[2 * i];
      b[i] = ab[2 * i + 1];
    }
    const bool silu = p.gi_silu != 0;
    const int e0 = ((part * PIX) / NP) * 8, e1 = (((part + 1) * PIX) / NP) * 8;
    constexpr int IT = (((PIX + NP - 1) / NP + 1) * 8 + 511) / 512;
    V8 xs[IT];  // every read issued before the first write (one LDS round trip, not IT)
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int e = e0 + tid + it * 512;
      const int pix = e >> 3;
      const int pxs = pix - (pix / PW) * PW;
      if (e < e1) xs[it] = *(const V8*)(buf + pix * 128 + ((lc ^ ((pxs >> 1) & 7)) << 4));
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int e = e0 + tid + it * 512;
      const int pix = e >> 3;
      if (e < e1) {
        const int py = pix / PW, px = pix - (pix / PW) * PW;
        const int iy = y0 - 1 + py, ix = x0 - 1 + px;
        const bool ok = iy >= 0 && iy < Ho && ix >= 0 && ix < Wo;
        V8 y;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float f = __builtin_fmaf((float)xs[it][i], a[i], b[i]);
          if (silu) f = silu_f(f);
          y[i] = ok ? (T)f : (T)0.f;
        }
        *(V8*)(buf + pix * 128 + ((lc ^ ((px >> 1) & 7)) << 4)) = y;
      }
    }
  };
  auto read_frags = [&] __attribute__((always_inline)) (int c, int t, int rb, int h, V8 (&af)[MT], V8 (&bf)[NT]) {
    const unsigned char* pa = smem + (c & 1) * PBUF;
    const unsigned char* sb = smem + RING + rb * STAGE;
    const int ky = PH ? pha + (t >> 1) : t / 3, kx = PH ? phb + (t & 1) : t - (t / 3) * 3;
    const int ch = h * 4 + fg;
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      const int pix = (wm * MT + mi + ky) * PW + fr + kx;
      af[mi] = *(const V8*)(pa + pix * 128 + ((ch ^ (((fr + kx) >> 1) & 7)) << 4));
    }
#pragma unroll
    for (int ni = 0; ni < NT; ++ni) {
      const int r = wn * WN + ni * 16 + fr;
      bf[ni] = *(const V8*)(sb + r * 128 + ((ch ^ ((r >> 1) & 7)) << 4));
    }
  };
  f32x4 acc[MT][NT];
  auto mma =[&](const V8 (&af)[MT], const V8 (&bf)[NT]) {
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) acc[mi][ni] = mfma16x16x32(af[mi], bf[ni], acc[mi][ni]);
  };
  // B-waves: all but the youngest `ahead` weight stages landed (ahead <= NS - 1)
  auto wait_b = [&] __attribute__((always_inline)) (int ahead) {
    if (NS >= 5 && ahead >= 4) hvm<(NS >= 5 ? 4 : 0) * PER_B>();
    else if (NS >= 4 && ahead >= 3) hvm<(NS >= 4 ? 3 : 0) * PER_B>();
    else if (ahead >= 2) hvm<2 * PER_B>();
    else if (ahead == 1) hvm<PER_B>();
    else hvm<0>();
  };

  // ---- prologue DMA: weight stages 0..NS-1, patches of chunks 0 (unless skip0: already in flight) and 1
  auto prologue_dma = [&] __attribute__((always_inline)) (bool skip0) {
    if (w < 4) {
#pragma unroll
      for (int s0 = 0; s0 < NS; ++s0)
        if (s0 < nsteps) stage_b(s0, s0);
    } else {
      if (!skip0) stage_p(cb);
      if (cb + 1 < ce) stage_p(cb + 1);
    }
  };
  // PT: the next tile's coordinates, so its chunk-0 patch can be DMA'd inside this tile's K loop (into patch buffer 0
  // once this tile's last chunk pair has started: an even chunk count) -- at the VAE's 1024^2 level the patch comes
  // from HBM, and fetched under the epilogue (the round-4 PT form) it still made every tile start on an HBM round
  // trip in lockstep with every other CU (r05 diagnostics: prologue + epilogue alone 175 of 381 us)
  constexpr int PCNT = P_I + (GNI ? 1 : 0);  // DMA instructions per patch wave and chunk (PT: uniform)
  auto tile_xy = [&] __attribute__((always_inline)) (int tile, int& img_, int& y0_, int& x0_) {
    const int nt_ = tile / nsp, sp_ = tile - nt_ * nsp;
    img_ = sp_ / (tiles_y * tiles_x);
    const int spi_ = sp_ - img_ * (tiles_y * tiles_x), ty_ = spi_ / tiles_x;
    y0_ = ty_ * TH;
    x0_ = (spi_ - ty_ * tiles_x) * 16;
  };
  setup(tl);
  prologue_dma(false);
  bool pf_prev = false;  // PT: this tile's chunk 0 was DMA'd inside the previous tile's K loop
  for (bool first = true;; first = false) {
  int nx_img = 0, nx_y0 = 0, nx_x0 = 0;
  const bool pf_next = PT && !SK && tl + tl_step < tl_hi && ce % 2 == 0;
  if (PT && pf_next) tile_xy(tl + tl_step, nx_img, nx_y0, nx_x0);
  // PT after the first tile: the weight stages and chunk 1 went out after the previous tile's epilogue stores; a
  // chunk 0 prefetched inside the previous K loop is older than those 8 stores (one per pass)
  if (PT && !first) {
    if (w < 4) hvm<(NS - 1) * PER_B>();
    else if (pf_prev) hvm<PCNT + 8>();
    else hvm<PCNT>();
  } else if (w < 4) wait_b(min(nsteps, NS) - 1);
  else hvm<0>();
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  __builtin_amdgcn_s_barrier();
  if (GNI) {
    transform(cb, 0, std::integral_constant<int, 1>());
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_barrier();
  }

  V8 a0[MT], b0[NT], a1[MT], b1[NT];
  if constexpr (PP) {
    // ---- ping-pong K loop.  Interval i (between barriers i - 1 and i): group 0 runs segment i, group 1 segment
    // i - 1; segment 2s = LOAD(s), 2s + 1 = COMPUTE(s).  So step s's fragments are read in intervals 2s (group 0)
    // and 2s + 1 (group 1).  Hazards:
    //  * weight stage s + NS - 1 is DMA'd by group 0 in LOAD(s) (interval 2s) into slot (s - 1) % NS, whose last
    //    reader (group 1, step s - 1) finished in interval 2s - 1; group 0 waits for stage s + 1 at the end of
    //    COMPUTE(s) (interval 2s + 1), before either group reads it (intervals 2s + 2, 2s + 3);
    //  * chunk c + 2's patch is DMA'd by group 1 at the end of COMPUTE(chunk c, tap 8) (interval 2(9c + 8) + 2) into
    //    buffer c & 1, whose last readers were group 0's and group 1's LOAD(chunk c, tap 8) (intervals 2(9c + 8) and
    //    + 1); group 1 waits for it at the end of LOAD(chunk c + 1, tap TW): before the first transform piece (GNI,
    //    tap PTR) or the first read of chunk c + 2;
    //  * GNI: each group transforms its threads' share of chunk c + 1's patch a piece per tap PTR .. 8 in its LOAD
    //    segments (under the partner's MFMAs); every LOAD ends with lgkmcnt(0), so the last piece (group 1,
    //    interval 2(9c + 8) + 1) is visible before group 0 reads chunk c + 1 (interval 2(9c + 9)).
    const int grp = w >> 2;
    // the next chunk's patch: DMA'd at the end of the last COMPUTE of chunk c - 1 (buffer (c + 1) & 1 is free once
    // both groups' LOAD of chunk c - 1's last tap is behind them), waited for by group 1 at the end of LOAD(tap TW)
    // of chunk c, transformed (GNI) in pieces at taps PTR .. NTAP - 1 -- the last piece (group 1, tap 8) still lands
    // an interval before group 0's first read of chunk c + 1
    constexpr int PTR = FD_HALO_PP_TR, PNP = NTAP - PTR > 0 ? NTAP - PTR : 1;
    constexpr int TW = GNI ? PTR - 1 : NTAP - 1;
    static_assert(!GNI || (PTR >= 1 && PTR < NTAP), "ping-pong transform taps");
    const int rr = wn * WN + fr;
    const int lb0 = RING + rr * 128 + (((0 * 4 + fg) ^ ((rr >> 1) & 7)) << 4);
    const int lb1 = RING + rr * 128 + (((1 * 4 + fg) ^ ((rr >> 1) & 7)) << 4);
    // fragment (mi, tap (ky, kx), K half h): the lane's column base la(kx, h) plus wave-uniform row offsets (the
    // column-only patch swizzle, as in the one-barrier loop below); PH: the tap's 2 x 2 window at (pha, phb)
    auto rd = [&] __attribute__((always_inline)) (int c, int t, int rb, auto hcc, V8 (&af)[MT], V8 (&bf)[NT]) {
      constexpr int H = decltype(hcc)::value;
      const int ky = PH ? pha + (t >> 1) : t / 3, kx = PH ? phb + (t & 1) : t - (t / 3) * 3;  // wave-uniform
      const int px = fr + kx;
      const int la = px * 128 + (((H * 4 + fg) ^ ((px >> 1) & 7)) << 4);
      const unsigned char* pa = smem + ((c & 1) * PBUF + (wm * MT + ky) * (PW * 128)) + la;
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) af[mi] = *(const V8*)(pa + mi * (PW * 128));
      const unsigned char* sb = smem + rb * STAGE + (H ? lb1 : lb0);
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) bf[ni] = *(const V8*)(sb + ni * 2048);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    if (grp == 1) {
      __builtin_amdgcn_s_barrier();  // the stagger
      if (FD_HALO_PP_PRIO) __builtin_amdgcn_s_setprio(1);  // the younger half wins VALU arbitration (guide item 4)
    }
    int c = cb, t = 0, rb = 0;
    for (int s = 0; s < nsteps; ++s) {
      // LOAD(s)
      rd(c, t, rb, I0(), a0, b0);
      rd(c, t, rb, I1(), a1, b1);
      if (w < 4) {
        if (s >= 1 && s + NS - 1 < nsteps) stage_b(s + NS - 1, rb == 0 ? NS - 1 : rb - 1);
      } else if (t == TW && c + 1 < ce) {
        hvm<0>();  // chunk c + 1's patch (the only patch DMA in flight)
      }
      if constexpr (GNI) {
        if (t >= PTR && c + 1 < ce) transform(c + 1, t - PTR, std::integral_constant<int, PNP>());
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this step's fragments, the transform's LDS writes
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      // COMPUTE(s)
      mma(a0, b0);
      mma(a1, b1);
      if (w < 4) wait_b(min(NS - 2, nsteps - 2 - s));  // weight stage s + 1 landed
      else if (t == NTAP - 1 && c + 2 < ce) stage_p(c + 2);  // buffer c & 1: both groups' last reads are behind
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      rb = rb == NS - 1 ? 0 : rb + 1;
      if (t == NTAP - 1) {
        ++c;
        t = 0;
      } else {
        ++t;
      }
    }
    if (grp == 0) __builtin_amdgcn_s_barrier();  // re-align the groups
    else if (FD_HALO_PP_PRIO) __builtin_amdgcn_s_setprio(0);
  } else if constexpr (CT) {
    // ---- the K loop with cheap LDS read addresses.  With the column-only patch swizzle, fragment (mi, tap (ky, kx),
    // K half h) sits at  la(kx, h) + [chunk buffer + (wm * MT + ky) * PW * 128] + mi * PW * 128  with
    //   la(kx, h) = (fr + kx) * 128 + chunk slot ((h * 4 + fg) ^ ((fr + kx) >> 1 & 7))
    // and the weights at lb(h) + rb * STAGE + ni * 2048 (r = wn * WN + fr; ni * 16 rows keep r >> 1 & 7): per half
    // step one lane base (five VALU), two adds of a wave-uniform offset, and immediates -- the generic read_frags spends
    // ~50 VALU per half step on the swizzled addresses, which made the loop VALU-issue-bound (r05 counters:
    // 132 VALU per 32 MFMAs).  Same schedule, waits, DMA and GroupNorm pieces, same per-element K order.
    // (the A lane base is recomputed per half step from the wave-uniform kx -- five VALU: a select among held bases
    // is turned by the compiler into a lookup table in scratch, whose vmcnt wait would also wait out the DMA)
    const int rr = wn * WN + fr;
    const int lb0 = RING + rr * 128 + (((0 * 4 + fg) ^ ((rr >> 1) & 7)) << 4);
    const int lb1 = RING + rr * 128 + (((1 * 4 + fg) ^ ((rr >> 1) & 7)) << 4);
    auto rd = [=] __attribute__((always_inline)) (int c, int t, int rb, auto hcc, V8 (&af)[MT], V8 (&bf)[NT]) {
      constexpr int H = decltype(hcc)::value;
      if constexpr ((FD_HALO_DIAG & 16) != 0) {
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) asm volatile("v_mov_b32 %0, 0" : "=v"(af[mi][0]));
#pragma unroll
        for (int ni = 0; ni < NT; ++ni) asm volatile("v_mov_b32 %0, 0" : "=v"(bf[ni][0]));
        return;
      }
      const int ky = t / 3, kx = t - (t / 3) * 3;  // wave-uniform
      const int px = fr + kx;
      const int la = px * 128 + (((H * 4 + fg) ^ ((px >> 1) & 7)) << 4);
      const int lboff_h = H ? lb1 : lb0;
      const unsigned char* pa = smem + ((c & 1) * PBUF + (wm * MT + ky) * (PW * 128)) + la;
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) af[mi] = *(const V8*)(pa + mi * (PW * 128));
      const unsigned char* sb = smem + rb * STAGE + lboff_h;
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) bf[ni] = *(const V8*)(sb + ni * 2048);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    constexpr int DG = FD_HALO_DIAG;
    auto mmd = [&] __attribute__((always_inline)) (const V8 (&af)[MT], const V8 (&bf)[NT]) {
      if constexpr (DG & 2) {
#pragma unroll
        for (int i = 0; i < MT; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
        for (int i = 0; i < NT; ++i) asm volatile("" ::"v"(bf[i]));
      } else {
        mma(af, bf);
      }
    };
    rd(cb, 0, 0, I0(), a0, b0);
    int c = cb, t = 0, rb = 0;
    for (int s = 0; s < ((DG & 32) ? 0 : nsteps - 1); ++s) {
      rd(c, t, rb, I1(), a1, b1);
      mmd(a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(DG & 1)) {
        if (w < 4) wait_b(min(NS - 2, nsteps - 2 - s));  // stage s + 1 landed
        else if (t == TR && c + 1 < ce) hvm<0>();        // chunk c + 1's patch landed
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      if constexpr (!(DG & 8)) __builtin_amdgcn_s_barrier();
      if constexpr (!(DG & 4)) {
        if (w < 4) {
          if (s + NS < nsteps) stage_b(s + NS, rb);
        } else if (t == NTAP - 1 && c + 2 < ce) {
          stage_p(c + 2);  // buffer c & 1: its last reads (this step's half 1) are behind the barrier
        } else if (PT && pf_next && t == NTAP - 1 && c + 2 == ce) {
          // the next tile's chunk 0 into buffer 0 (c even): waited for at that tile's start
          stage_p_at(0, nx_img, nx_y0, nx_x0, GNI ? (const float*)p.gi_affine + (long long)nx_img * Cin * 2 : nullptr);
        }
      }
      const int tc = (GNI && t >= TR && t < NTAP - 1 && c + 1 < ce) ? c + 1 : -1, tp = t - TR;
      rb = rb == NS - 1 ? 0 : rb + 1;
      if (t == NTAP - 1) {
        ++c;
        t = 0;
      } else {
        ++t;
      }
      rd(c, t, rb, I0(), a0, b0);
      mmd(a1, b1);
      if (GNI && tc >= 0) {
        __builtin_amdgcn_sched_barrier(0);
        transform(tc, tp, std::integral_constant<int, NPART>());
      }
    }
    rd(c, t, rb, I1(), a1, b1);
    mmd(a0, b0);
    mmd(a1, b1);
    if constexpr ((DG & 1) != 0) hvm<0>();  // nothing in flight past the loop
  } else {
  read_frags(cb, 0, 0, 0, a0, b0);
  int c = cb, t = 0, rb = 0;
  for (int s = 0; s < nsteps - 1; ++s) {
    read_frags(c, t, rb, 1, a1, b1);
    mma(a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    if (w < 4) wait_b(min(NS - 2, nsteps - 2 - s));  // stage s + 1 landed
    else if (t == (PH ? NTAP - 1 : TR)) hvm<0>();     // chunk c + 1's patch landed
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_barrier();
    if (w < 4) {
      if (s + NS < nsteps) stage_b(s + NS, rb);
    } else if (t == NTAP - 1 && c + 2 < ce) {
      stage_p(c + 2);  // buffer c & 1: its last reads (this step's half 1) are behind the barrier
    }
    // chunk c + 1's patch: a piece per tap TR .. 7 behind this step's half-1 MFMAs (below); visible to the readers
    // after step (c, 8)'s barrier
    const int tc = (GNI && t >= TR && t < NTAP - 1 && c + 1 < ce) ? c + 1 : -1, tp = t - TR;
    rb = rb == NS - 1 ? 0 : rb + 1;
    if (t == NTAP - 1) {
      ++c;
      t = 0;
    } else {
      ++t;
    }
    read_frags(c, t, rb, 0, a0, b0);
    mma(a1, b1);
    if (GNI && tc >= 0) {
      __builtin_amdgcn_sched_barrier(0);
      transform(tc, tp, std::integral_constant<int, NPART>());
    }
  }
  read_frags(c, t, rb, 1, a1, b1);
  mma(a0, b0);
  mma(a1, b1);
  }  // generic K loop

  if constexpr (PT) {
    // ---- PT epilogue: thread tid owns the 8-column vector cv of row rr of each 32-row pass.  This tile's bias and
    // residual go into registers first (older than the next tile's DMA, so the compiler's counted waits on them do
    // not wait for it), then -- every wave past its last ring / patch read -- the next tile's DMA is issued, then
    // the passes run on the PT region only.  Stores, GroupNorm slots and the fixed-order fold as in the 128-row
    // epilogue below (the fold visits rows gj, gj + TPG, ... in the same order, so the partials are the same bits).
    constexpr int NPASS = BM / PER;
    const int rr = tid >> 4, cv = tid & 15, n = n0 + cv * 8;
    const T* __restrict__ R = (const T*)p.residual;
    float bv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) bv[i] = 0.f;
    if (p.bias) {
      *(f32x4*)&bv[0] = *(const f32x4*)(p.bias + n);
      *(f32x4*)&bv[4] = *(const f32x4*)(p.bias + n + 4);
    }
    const long long m0 = ((long long)img * Ho + y0) * Wo + x0;  // output row of the tile's pixel (0, 0)
    TO8 res[NPASS];
    if (R) {
#pragma unroll
      for (int k = 0; k < NPASS; ++k) {
        const int rt = k * PER + rr;
        res[k] = *(const TO8*)(R + (m0 + (long long)(rt >> 4) * Wo + (rt & 15)) * p.ldr + n);
      }
    }
    const int cimg = img, cspi = spi, cn0 = n0;
    lds_barrier();
    const int tl_next = tl + tl_step;
    T* __restrict__ C = (T*)p.C;
    float* ep = (float*)(smem + PT_EP);
    f32x4* const slots = (f32x4*)(smem + PT_SLOT);
    const bool gn = p.gn_part != nullptr;
    const int cpg = gn ? N / p.gn_groups : 8;
    const int G = BN / cpg, TPG = gn ? 512 / G : 512;
    const int gg = tid / TPG, gj = tid - (tid / TPG) * TPG;
    float gs = 0.f, gq = 0.f;
#pragma unroll 1
    for (int k = 0; k < NPASS; ++k) {
      if (k) lds_barrier();  // the previous pass's ep / slot reads done
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        if (wm * WM + mi * 16 >= k * PER && wm * WM + mi * 16 < (k + 1) * PER) {
          const int rl = wm * WM + mi * 16 + fg * 4 - k * PER;
#pragma unroll
          for (int ni = 0; ni < NT; ++ni) {
            const int col = wn * WN + ni * 16 + fr;
#pragma unroll
            for (int j = 0; j < 4; ++j) ep[(rl + j) * LDE + col] = acc[mi][ni][j] * p.alpha;
          }
        }
      }
      lds_barrier();
      float v[8];
      *(f32x4*)&v[0] = *(const f32x4*)(ep + rr * LDE + cv * 8);
      *(f32x4*)&v[4] = *(const f32x4*)(ep + rr * LDE + cv * 8 + 4);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] += bv[i];
      if (p.act != FD_ACT_NONE) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = act_f(v[i], p.act);
      }
      if (R) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] += (float)res[k][i];
      }
      TO8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (T)v[i];
      const int rt = k * PER + rr;
      st_out16((TO8*)(C + (m0 + (long long)(rt >> 4) * Wo + (rt & 15)) * p.ldc + n), o);
      if (gn) {
        const int sp8 = ((cv * 8) / cpg + 1) * cpg - cv * 8;
        float s0 = 0.f, q0 = 0.f, s1 = 0.f, q1 = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float f = (float)o[i];
          if (i < sp8) {
            s0 += f;
            q0 += f * f;
          } else {
            s1 += f;
            q1 += f * f;
          }
        }
        slots[tid] = (f32x4){s0, q0, s1, q1};
        lds_barrier();
        const int cc0 = (gg * cpg) / 8, cc1 = ((gg + 1) * cpg - 1) / 8;
        const int r0 = ((gj - (k * PER) % TPG) % TPG + TPG) % TPG;  // first row of this pass that is = gj mod TPG
        for (int r = r0; r < PER; r += TPG)
          for (int cc = cc0; cc <= cc1; ++cc) {
            const f32x4 v4 = slots[r * VPR + cc];
            const bool fst = (cc * 8) / cpg == gg;
            gs += fst ? v4[0] : v4[2];
            gq += fst ? v4[1] : v4[3];
          }
      }
    }
    if (gn) {  // red[] in the pass buffer: its last readers passed the fold barrier above
      float2* red = (float2*)ep;
      red[tid] = make_float2(gs, gq);
      lds_barrier();
      if (tid < G) {
        float S = 0.f, Q = 0.f;
        for (int k = 0; k < TPG; ++k) {
          const float2 v2 = red[tid * TPG + k];
          S += v2.x;
          Q += v2.y;
        }
        const long long blk = (long long)cimg * (tiles_y * tiles_x) + cspi;
        ((float2*)p.gn_part)[blk * p.gn_groups + cn0 / cpg + tid] = make_float2(S, Q);
      }
    }
    // the next tile's weight stages and chunk 1 (chunk 0 too unless the K loop prefetched it) only now: DMA issued
    // before the passes made the compiler's waits for this tile's bias / residual registers wait for it as well
    // (round 4: PT 2.3x slower on the residual convs)
    if (tl_next < tl_hi) {
      setup(tl_next);
      prologue_dma(pf_next);
    }
    pf_prev = pf_next;
    tl = tl_next;
    if (tl >= tl_hi) return;
    continue;
  }
  break;
  }  // tile loop (one pass unless PT)

  // ---- SK: pairwise combine (gemm8's S = 2 form): the first half to finish publishes its fp32 accumulators with
  // write-through (sc1) stores and an sc1 flag; the second waits for the flag, adds them to its own (a + b: the
  // same bits whichever half came first) and runs the epilogue.  It only ever waits on a workgroup that already
  // took its ticket (running), so no co-residency is assumed; the wait is bounded.
  if constexpr (SK) {
    constexpr int SLAB = MT * NT * 512 * 16;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((char*)slabs + (long long)tlin * SLAB, (short)0, SLAB, 0x00020000);
    unsigned* flag = counters + 32768 + tlin;
    __syncthreads();  // every wave past its last LDS read: smem[0] is free
    if (tid == 0) {
      const unsigned tk = __hip_atomic_fetch_add(counters + tlin, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
                                                 ((mi * NT + ni) * 512 + tid) * 16, 0, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0 && !__hip_atomic_load(&g_halo_sk_drop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if (tid == 0) {
      // bounded: a lost flag poisons the tile (NaN) instead of hanging the GPU and counts a timeout (the host
      // checks it and re-zeroes the counters: gemm8.hip's pairwise form has the same protocol)
      unsigned got = 0u;
      for (int it = 0; it < (1 << 24) && !got; ++it) {
        got = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!got) __builtin_amdgcn_s_sleep(2);
      }
      if (got) {
        __hip_atomic_store(flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(counters + tlin, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        __hip_atomic_fetch_add(&g_halo_sk_timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ((mi * NT + ni) * 512 + tid) * 16, 0, 16));
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) acc[mi][ni] = split == 0 ? acc[mi][ni] + part[mi][ni] : part[mi][ni] + acc[mi][ni];
    if (!partner_ok) {
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NT; ++ni) acc[mi][ni] = f32x4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
    }
  }

  // ---- epilogue: two (TH = 16) or one 128-row passes through LDS fp32 [128][BN + 4]; each thread then owns 8
  // consecutive columns of a row: bias, per-image row bias (time embedding), activation, residual, one 16-B store;
  // GroupNorm output statistics (gn_part) folded per group in a fixed order.
  T* __restrict__ C = (T*)p.C;
  const T* __restrict__ R = (const T*)p.residual;
  const float* __restrict__ bias = p.bias;
  const float* __restrict__ rbias = p.rowbias;
  const float alpha = p.alpha;
  const int act = p.act;
  float* ep = (float*)smem;
  f32x4* const slots = (f32x4*)(smem + SLOT);
  const bool gn = p.gn_part != nullptr;
  const int cpg = gn ? N / p.gn_groups : 8;
  const int G = BN / cpg, TPG = gn ? 512 / G : 512;
  const int gg = tid / TPG, gj = tid - (tid / TPG) * TPG;
  float gs = 0.f, gq = 0.f;
  // the residual rows of the whole tile requested before the first staging barrier: their memory round trip (HBM at
  // the VAE's 1024^2 level) overlaps the staging instead of being paid once per 512-vector pass (the passes were a
  // run-time loop, each waiting for its own loads; r05).  Only the VAE's 256 x 128 tiles: on the UNet's 160-column
  // tiles the unrolled passes measured 1-2 % slower, so those keep the run-time loop and load in place.
  constexpr int EIT = (EROWS * VPR + 511) / 512, NHALF = BM / EROWS;
  constexpr bool EPF = TH == 16 && BN == 128;
  constexpr int EU_H = EPF ? NHALF : 1, EU_I = EPF ? EIT : 1;
  auto epi_row = [&] __attribute__((always_inline)) (int half, int e, int& cv, bool& ok, long long& m) {
    const int r = e / VPR;
    cv = e - r * VPR;
    const int rt = half * EROWS + r;
    const int oy = y0 + (rt >> 4), ox = x0 + (rt & 15);
    ok = oy < Hg && ox < Wg;
    m = PH ? ((long long)img * Ho + 2 * oy + pha) * Wo + 2 * ox + phb : ((long long)img * Ho + oy) * Wo + ox;
  };
  TO8 resv[EU_H][EU_I];
  if (EPF && R) {
#pragma unroll
    for (int hh = 0; hh < NHALF; ++hh)
#pragma unroll
      for (int it = 0; it < EIT; ++it) {
        const int e = tid + it * 512;
        if ((EROWS * VPR) % 512 == 0 || e < EROWS * VPR) {
          int cv;
          bool ok;
          long long m;
          epi_row(hh, e, cv, ok, m);
          if constexpr (EPF) {
            if (ok) resv[hh][it] = *(const TO8*)(R + m * p.ldr + n0 + cv * 8);
          }
        }
      }
  }
#pragma unroll EU_H
  for (int half = 0; half < NHALF; ++half) {
    __syncthreads();  // the ring / patches (half 0) or the previous half's staging (half 1) fully consumed
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
#pragma unroll EU_I
    for (int it = 0; it < EIT; ++it) {
      const int e = tid + it * 512;
      if ((EROWS * VPR) % 512 != 0 && e >= EROWS * VPR) break;
      const int r = e / VPR;
      int cv;
      bool ok;
      long long m;
      epi_row(half, e, cv, ok, m);
      const int n = n0 + cv * 8;
      float v[8], bv[8], rv[8];
      TO8 res;
      *(f32x4*)&v[0] = *(const f32x4*)(ep + r * LDE + cv * 8);
      *(f32x4*)&v[4] = *(const f32x4*)(ep + r * LDE + cv * 8 + 4);
      if (bias) {
        *(f32x4*)&bv[0] = *(const f32x4*)(bias + n);
        *(f32x4*)&bv[4] = *(const f32x4*)(bias + n + 4);
      }
      // rows outside the image (ragged tiles) are never stored and must not read either: past the last image
      // m / rows_per_group indexes a row-bias row that does not exist (an out-of-bounds read that faulted when the
      // allocator placed the time-embedding buffer at the end of a mapping)
      if (rbias && ok) {
        const float* rr = rbias + (long long)(m / p.rows_per_group) * p.rowbias_ld + n;
        *(f32x4*)&rv[0] = *(const f32x4*)rr;
        *(f32x4*)&rv[4] = *(const f32x4*)(rr + 4);
      }
      if (R && ok) {
        if constexpr (EPF) res = resv[half][it];
        else res = *(const TO8*)(R + m * p.ldr + n);
      }
      if (bias) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] += bv[i];
      }
      if (rbias && ok) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] += rv[i];
      }
      if (act != FD_ACT_NONE) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = act_f(v[i], act);
      }
      if (R && ok) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] += (float)res[i];
      }
      TO8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (T)v[i];
      if (ok) st_out16((TO8*)(C + m * p.ldc + n), o);
      if (gn) {  // (sum, sumsq) of the stored values, split at the group boundary inside the chunk
        const int split = ((cv * 8) / cpg + 1) * cpg - cv * 8;
        float s0 = 0.f, q0 = 0.f, s1 = 0.f, q1 = 0.f;
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
        slots[e] = (f32x4){s0, q0, s1, q1};
      }
    }
    if (gn) {  // thread (group gg, j) folds rows j, j + TPG, ... of its group, chunks in column order
      __syncthreads();
      const int cc0 = (gg * cpg) / 8, cc1 = ((gg + 1) * cpg - 1) / 8;
      for (int r = gj; r < EROWS; r += TPG)
        for (int cc = cc0; cc <= cc1; ++cc) {
          const f32x4 v4 = slots[r * VPR + cc];
          const bool first = (cc * 8) / cpg == gg;
          gs += first ? v4[0] : v4[2];
          gq += first ? v4[1] : v4[3];
        }
    }
  }
  if (gn) {
    float2* red = (float2*)(smem + RED);
    red[tid] = make_float2(gs, gq);
    __syncthreads();
    if (tid < G) {
      float S = 0.f, Q = 0.f;
      for (int k = 0; k < TPG; ++k) {
        const float2 v2 = red[tid * TPG + k];
        S += v2.x;
        Q += v2.y;
      }
      const long long blk = ((long long)img * (PH ? 4 : 1) + (PH ? pha * 2 + phb : 0)) * (tiles_y * tiles_x) + spi;
      ((float2*)p.gn_part)[blk * p.gn_groups + n0 / cpg + tid] = make_float2(S, Q);
    }
  }
}

struct HaloPlan {
  int th, bn, tiles, sk, ns;  // tiles: output tiles (workgroups = tiles * (1 + sk)); ns: weight ring depth
  int pt;                     // persistent workgroups (PT form), 0 = one workgroup per tile
  int ph;                     // the phase form of a nearest x2 upsample conv (fd_gemm_params.up_phase)
};

// Compute units of the current device (cached per device id).
int cu_count() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    cache[dev] = v;
  }
  return cache[dev];
}

// The PT form: 256-row x 128-column tiles over whole images (every tile full: one store per thread and pass), at
// least two chunks of input channels (the prologue DMA count the epilogue waits rely on), no per-image row bias,
// and at least two tiles per CU (below that there is no next tile to overlap).  Returns its workgroup count.
// FD_CONV_HALO_PT = 3 (default, "auto"): only the GroupNorm-folded convs without a residual -- the VAE 1024^2 resnet
// conv1s, 470 -> 431 us with the next tile's chunk-0 patch DMA'd inside the K loop; the residual convs run 2.3x
// slower in this form and the plain ones ~2 % slower (profiles/r05k_*)
int halo_pt_grid(const fd_gemm_params* p, int th, int bn, int sk, long long tiles) {
  const int mode = fd_knob(FDK_CONV_HALO_PT);
  if (!mode || (mode == 3 && (!p->gi_affine || p->residual))) return 0;
  if (th != 16 || bn != 128 || sk || p->Cin < 128 || p->rowbias) return 0;
  if (p->Hout % 16 || p->Wout % 16) return 0;
  const int cus = cu_count();
  if (tiles < 2LL * cus || cus < 8) return 0;
  return cus & ~7;
}

// Eligibility and tile plan, from per-image quantities only (m_ref: rows of one TLC tile's forward), so batching
// tiles never moves a launch between this kernel and the implicit GEMM (bitwise batch invariance).
// The phase form (up_phase): always this kernel (no other takes the [4 Cout][4 Cin] weights); tiles over the
// low-resolution grid, 256-row tiles while there are enough of them, else 128-row.
int halo_plan_phase(const fd_gemm_params* p, HaloPlan* pl) {
  if (!p->conv || !p->upsample || p->batch > 1 || p->stride != 1 || p->pad != 1 || p->A2 || p->gi_affine) return 0;
  if (p->Hout != 2 * p->Hin || p->Wout != 2 * p->Win || p->K != 4 * p->Cin || p->Cin % 64) return 0;
  if (p->lda < p->Cin || p->lda % 8 || p->ldb % 8 || p->ldc % 8 || p->ldb < 4 * p->Cin) return 0;
  if (p->act == FD_ACT_GEGLU || p->ln_in || p->ln_out || p->dtype != p->out_dtype || p->dtype == FD_F32) return 0;
  if ((p->residual && p->ldr % 8) || (p->rowbias && p->rowbias_ld % 4)) return 0;
  const unsigned long long al = (unsigned long long)p->A | (unsigned long long)p->B | (unsigned long long)p->C |
                                (unsigned long long)(p->residual ? p->residual : nullptr) |
                                (unsigned long long)(p->bias ? p->bias : nullptr) |
                                (unsigned long long)(p->rowbias ? p->rowbias : nullptr);
  if (al & 15) return 0;
  const int bn = p->N % 160 == 0 ? 160 : (p->N % 128 == 0 ? 128 : 0);
  if (!bn || p->Win < 16 || p->Hin < 8) return 0;
  const long long hw = (long long)p->Hout * p->Wout;
  const int m_ref = p->m_ref > 0 ? p->m_ref : p->M;
  const long long nimg_ref = m_ref / hw > 0 ? m_ref / hw : 1;
  const long long t16 = nimg_ref * ((p->Hin + 15) / 16) * ((p->Win + 15) / 16) * (4 * p->N / bn);
  const int th = (t16 >= fd_knob(FDK_CONV_HALO_MIN_TILES) && p->Hin >= 16) ? 16 : 8;
  pl->th = th;
  pl->bn = bn;
  pl->sk = 0;
  pl->pt = 0;
  pl->ns = 3;
  pl->ph = 1;
  pl->tiles = (int)(p->nimg * ((p->Hin + th - 1) / th) * ((p->Win + 15) / 16) * (4 * p->N / bn));
  return 1;
}

int halo_plan(const fd_gemm_params* p, HaloPlan* pl) {
  if (p->up_phase) return halo_plan_phase(p, pl);
  pl->ph = 0;
  // FD_CONV_HALO: 0 off; 1 on, except the convs the 256 x 256 kernel takes (the VAE's 256 / 512-channel levels at
  // 256^2 - 512^2 and the upsample convs: its intake beats the 128 / 160-column halo tile there even with the
  // GroupNorm pass, probes/conv_ab.py); 2 on wherever eligible
  const int mode = fd_knob(FDK_CONV_HALO);
  if (!mode) return 0;
  const bool g256 = mode == 1 && gemm256_takes(p);
  if (g256 && fd_knob(FDK_CONV_HALO_PT) != 2) return 0;
  if (!p->conv || p->batch > 1 || p->stride != 1 || p->pad != 1 || p->A2 || p->K != 9 * p->Cin) return 0;
  if (p->Cin % 64 || p->lda < p->Cin || p->lda % 8 || p->ldb % 8 || p->ldc % 8) return 0;
  if (p->act == FD_ACT_GEGLU || p->ln_in || p->ln_out || p->dtype != p->out_dtype || p->dtype == FD_F32) return 0;
  if (p->residual && p->ldr % 8) return 0;
  if (p->rowbias && p->rowbias_ld % 4) return 0;
  const unsigned long long al = (unsigned long long)p->A | (unsigned long long)p->B | (unsigned long long)p->C |
                                (unsigned long long)(p->residual ? p->residual : nullptr) |
                                (unsigned long long)(p->bias ? p->bias : nullptr) |
                                (unsigned long long)(p->rowbias ? p->rowbias : nullptr) |
                                (unsigned long long)(p->gi_affine ? p->gi_affine : nullptr);
  if (al & 15) return 0;
  if (p->upsample == 0 && (p->Hin != p->Hout || p->Win != p->Wout)) return 0;
  const int bn = p->N % 160 == 0 ? 160 : (p->N % 128 == 0 ? 128 : 0);
  if (!bn) return 0;
  const long long hw = (long long)p->Hout * p->Wout;
  const int m_ref = p->m_ref > 0 ? p->m_ref : p->M;
  const long long nimg_ref = m_ref / hw > 0 ? m_ref / hw : 1;
  auto tiles = [&](int th) { return nimg_ref * ((p->Hout + th - 1) / th) * ((p->Wout + 15) / 16) * (p->N / bn); };
  const int min_tiles = fd_knob(FDK_CONV_HALO_MIN_TILES);
  int th = 0, sk = 0;
  if (tiles(16) >= min_tiles) th = 16;
  // 256-row tiles with the input channels split over two workgroups before 128-row tiles: half the weight bytes per
  // MFMA flop (the UNet's 64^2 level, whose 128-row tiles are bound by the weight stream into LDS, r05 diagnostics);
  // from 640 input channels (K >= 5760): below that the pairwise hand-off costs more than it saves (320 -> 640:
  // 42.7 -> 49.0 us; 1920 -> 640: 160 -> 145 us, profiles/r05i_conv_ab_split16_*.jsonl)
  else if (fd_knob(FDK_CONV_HALO_SPLIT16) && p->Cin >= 640 && 2 * tiles(16) >= min_tiles) th = 16, sk = 1;
  else if (tiles(8) >= min_tiles) th = 8;
  else if (fd_knob(FDK_CONV_HALO_SPLIT) && p->Cin >= 128 && 2 * tiles(8) >= min_tiles) th = 8, sk = 1;
  if (!th || p->Wout < 16 || p->Hout < th) return 0;
  pl->th = th;
  pl->bn = bn;
  pl->sk = sk;
  pl->tiles = (int)(p->nimg * ((p->Hout + th - 1) / th) * ((p->Wout + 15) / 16) * (p->N / bn));
  if (sk && pl->tiles > 32768) return 0;  // one split-K counter / flag per tile
  pl->pt = halo_pt_grid(p, th, bn, sk, pl->tiles);
  // a 128-row tile's K step is half the MFMA work of a 256-row one: its weight stages need a deeper ring to cover
  // the L2 latency (the 256-row tile's LDS holds 3 stages at 160 columns, 4 at 128)
  pl->ns = th == 8 ? 3 : (bn == 128 && !pl->pt && !sk ? fd_knob(FDK_CONV_HALO_NS16) : 3);
  if (g256 && !pl->pt) return 0;  // FD_CONV_HALO_PT = 2 takes a gemm256 conv only in the PT form
  return 1;
}

constexpr int slab_bytes(int th, int bn) { return (th * 4 / 16) * (bn / 32) * 512 * 16; }

template <typename T>
int launch_halo(const fd_gemm_params* p, const HaloPlan& pl, hipStream_t s) {
  const bool gi = p->gi_affine != nullptr;
  float* slabs = pl.sk ? (float*)((char*)p->ws + 65536 * sizeof(unsigned)) : nullptr;
  unsigned* cnt = pl.sk ? (unsigned*)p->ws : nullptr;
  const dim3 grid(pl.pt ? pl.pt : pl.tiles * (1 + pl.sk));
  // ping-pong loop for the 256-row tiles (per-tile forms); the 128-row tiles' 10-20 MFMAs per half step measured
  // slower split in two segments (profiles/r06a_conv_ab_pp*.jsonl)
  const bool pp = fd_knob(FDK_CONV_HALO_PP) != 0 && pl.th == 16;
  if (pl.ph) {
    if (gi || pl.sk || pl.pt || pl.ns != 3) return FD_ERR_ARG;
#define FD_HALO_PH(TH_, BN_)                                                                                          \
    if (pl.th == TH_ && pl.bn == BN_) {                                                                              \
      if (pp)                                                                                                        \
        hipLaunchKernelGGL((conv_halo_kernel<T, TH_, BN_, false, false, 3, false, true, true>), grid, dim3(512), 0, s, \
                           *p, slabs, cnt);                                                                          \
      else                                                                                                           \
        hipLaunchKernelGGL((conv_halo_kernel<T, TH_, BN_, false, false, 3, false, true, false>), grid, dim3(512), 0, s, \
                           *p, slabs, cnt);                                                                          \
      FD_LAUNCH_CHECK();                                                                                             \
      return FD_OK;                                                                                                  \
    }
    FD_HALO_PH(16, 160)
    FD_HALO_PH(16, 128)
    FD_HALO_PH(8, 160)
    FD_HALO_PH(8, 128)
#undef FD_HALO_PH
    return FD_ERR_ARG;
  }
  if (pl.pt) {
    if (pl.th != 16 || pl.bn != 128 || pl.sk || pl.ns != 3) return FD_ERR_ARG;
    if (gi)
      hipLaunchKernelGGL((conv_halo_kernel<T, 16, 128, true, false, 3, true, false, false>), grid, dim3(512), 0, s, *p, slabs, cnt);
    else
      hipLaunchKernelGGL((conv_halo_kernel<T, 16, 128, false, false, 3, true, false, false>), grid, dim3(512), 0, s, *p, slabs, cnt);
    FD_LAUNCH_CHECK();
    return FD_OK;
  }
#define FD_HALO_L(TH_, BN_, GI_, SK_, NS_, PP_)                                                                      \
  hipLaunchKernelGGL((conv_halo_kernel<T, TH_, BN_, GI_, SK_, NS_, false, false, PP_>), grid, dim3(512), 0, s, *p, slabs, \
                     cnt)
#define FD_HALO(TH_, BN_, SK_, NS_)                                                                                  \
  if (pl.th == TH_ && pl.bn == BN_ && pl.sk == SK_ && pl.ns == NS_) {                                                \
    if (gi && pp) FD_HALO_L(TH_, BN_, true, SK_, NS_, true);                                                                   \
    else if (gi) FD_HALO_L(TH_, BN_, true, SK_, NS_, false);                                                                   \
    else if (pp) FD_HALO_L(TH_, BN_, false, SK_, NS_, true);                                                                   \
    else FD_HALO_L(TH_, BN_, false, SK_, NS_, false);                                                                          \
    FD_LAUNCH_CHECK();                                                                                               \
    return FD_OK;                                                                                                    \
  }
  FD_HALO(16, 160, 0, 3)
  FD_HALO(16, 128, 0, 3)
  FD_HALO(16, 128, 0, 4)
  FD_HALO(8, 160, 0, 3)
  FD_HALO(8, 128, 0, 3)
  FD_HALO(8, 160, 1, 3)
  FD_HALO(8, 128, 1, 3)
  FD_HALO(16, 160, 1, 3)
  FD_HALO(16, 128, 1, 3)
#undef FD_HALO
#undef FD_HALO_L
  return FD_ERR_ARG;
}

}  // namespace

// Rows per GroupNorm-statistics block this conv would write (256 / 128), 0 = the halo kernel does not take it.
extern "C" int fd_conv_halo_plan(const fd_gemm_params* p) {
  HaloPlan pl;
  if (!halo_plan(p, &pl)) return 0;
  return pl.th * 16;
}

// Workgroups of the PT form for this conv, 0 = one workgroup per tile (or not the halo kernel).
extern "C" int fd_conv_halo_pt(const fd_gemm_params* p) {
  HaloPlan pl;
  if (!p || !halo_plan(p, &pl)) return 0;
  return pl.pt;
}

// Split-K workspace of the halo kernel for this conv: -1 = the halo kernel does not take it, else bytes (0 = none).
extern "C" long long fd_conv_halo_ws_bytes(const fd_gemm_params* p) {
  HaloPlan pl;
  if (!p || !halo_plan(p, &pl)) return -1;
  if (!pl.sk) return 0;
  return 65536LL * sizeof(unsigned) + (long long)pl.tiles * slab_bytes(pl.th, pl.bn);
}

// Called by fd_gemm for every conv: 1 = launched here, 0 = not eligible (the implicit GEMM takes it), < 0 = error.
// gn_part is honoured when the tiles are whole (H % TH == 0, W % 16 == 0, N a multiple of the group width and of
// the tile's groups); p->gn_done reports it.  gi_affine (the consumer GroupNorm) requires this kernel: an ineligible
// conv with gi_affine set is FD_ERR_SHAPE (callers ask fd_conv_halo_plan first).
extern "C" int fd_conv_halo_try(fd_gemm_params* p, void* stream) {
  HaloPlan pl;
  if (!halo_plan(p, &pl)) return (p->gi_affine || p->up_phase) ? FD_ERR_SHAPE : 0;
  if (pl.sk && (!p->ws || p->ws_bytes < 65536LL * (long long)sizeof(unsigned) +
                                          (long long)pl.tiles * slab_bytes(pl.th, pl.bn)))
    return FD_ERR_ARG;
  fd_gemm_params q = *p;
  p->gn_done = 0;
  if (q.gn_part) {
    const int cpg = q.gn_groups > 0 ? q.N / q.gn_groups : 0;
    const bool ok = q.gn_groups > 0 && q.N % q.gn_groups == 0 && cpg >= 4 && pl.bn % cpg == 0 &&
                    512 % (pl.bn / cpg) == 0 && (pl.ph ? q.Hin : q.Hout) % pl.th == 0 &&
                    (pl.ph ? q.Win : q.Wout) % 16 == 0 &&
                    q.gn_hw == q.Hout * q.Wout && q.M == q.nimg * q.gn_hw;
    if (!ok) q.gn_part = nullptr;
  }
  int rc;
  if (q.dtype == FD_BF16) rc = launch_halo<bf16>(&q, pl, (hipStream_t)stream);
  else rc = launch_halo<f16>(&q, pl, (hipStream_t)stream);
  if (rc == FD_OK && q.gn_part) p->gn_done = pl.th * 16;
  return rc == FD_OK ? 1 : rc;
}

// Split-K hand-off health of this translation unit (see g8_splitk_health).
int halo_splitk_health(unsigned* timeouts, int reset, int drop) {
  unsigned v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_halo_sk_timeouts), sizeof(v)) != hipSuccess) return FD_ERR_HIP;
  if (timeouts) *timeouts += v;
  const unsigned z = 0u, d = (unsigned)drop;
  if (reset && hipMemcpyToSymbol(HIP_SYMBOL(g_halo_sk_timeouts), &z, sizeof(z)) != hipSuccess) return FD_ERR_HIP;
  if (drop >= 0 && hipMemcpyToSymbol(HIP_SYMBOL(g_halo_sk_drop), &d, sizeof(d)) != hipSuccess) return FD_ERR_HIP;
  return FD_OK;
}
