// Attention kernels for gfx950.
//
// flash_attn_d64: head_dim 64 flash attention (SDPA replacement for the 140 attn1/attn2 calls of a
// UNet forward).  One workgroup = NWV waves (4 by default; 2-wave workgroups measured no faster at Lq = 1024
// and 10 % slower at 4096) of one (batch, head); each wave owns 16 * NQB queries (16 or 32, by launch size).  K/V tiles of 64 keys are staged by global_load_lds into a double buffer.  The score
// tile is computed transposed, S^T = K Q^T (A = K rows from LDS, B = Q fragments held in VGPRs),
// so each lane owns one query column: the row max needs only two cross-lane shuffles, and the
// accumulator, packed to bf16/f16 in registers, is directly the B operand of O^T = V^T P^T (guide
// section 3, "an accumulator tile as the next MFMA's operand").  V^T fragments come from
// ds_read_b64_tr_b16 on a row-major V tile (T10).  Softmax is online, exp2-based, fp32.
//
// mha_seq_axis: the information transformer's MultiheadAttention over the batch axis (L = CFG pair).
// softmax_rows: fp32 row softmax for the single-head d=512 VAE mid attention (GEMM + softmax + GEMM).
#include <type_traits>
#include <utility>

#include "fd_common.h"

// amdgpu_waves_per_eu(1, 2): let the compiler use the full 256-VGPR budget of two waves per SIMD instead of
// capping arch VGPRs at 128 and spilling the O / S accumulators through AGPR moves (192 v_accvgpr per tile).
// max over lanes l, l^16, l^32, l^48 (the 4 row groups of a 16 x 16 MFMA block): gfx950 permlane swaps
// (VALU) instead of two ds_bpermute round trips in the softmax's dependent chain
// (plain v_max_f32 in asm: fmaxf on a permlane result makes hipcc canonicalise both inputs first)
__device__ __forceinline__ float vmax_raw(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// one v_fma_f32: hipcc SLP-packs adjacent f32 fmas into v_pk_fma_f32, which beside MFMAs costs ~22 cycles more
// than two single fmas (MI355X_MICROARCH.md, per-instruction cycle constants); same fused result bit for bit
__device__ __forceinline__ float fma_raw(float a, float b, float c) {
  float r;
  asm("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float xor_max_16_32(float x) {
  const unsigned u = __float_as_uint(x);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  x = vmax_raw(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const unsigned v = __float_as_uint(x);
  const auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return vmax_raw(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

#ifndef FLASH_NBUF
#define FLASH_NBUF 3
#endif
#ifndef FD_FLASH_SFMA
#define FD_FLASH_SFMA 1
#endif
// QPRE: Q pre-multiplied by scale * log2(e) (rounded to the 16-bit type once per query) and every score
// accumulator started at -m (the running max, log2 domain): the MFMA leaves exp2's argument ready, so a tile whose
// maxima did not grow needs one v_exp_f32 per score and nothing else (experimental; costs the rounding of Q * c)
#ifndef FD_FLASH_QPRE
#define FD_FLASH_QPRE 0
#endif
// KPRE: the next tile's K fragments are read right after a mid-tile barrier, under this tile's P.V MFMAs, and
// held in 32 VGPRs across the loop edge (the ring refill moves to that barrier as well)
#ifndef FD_FLASH_KPRE
#define FD_FLASH_KPRE 0
#endif
// DIAG (timing builds only, wrong results): 1 = no K/V loads after the prologue (the ring is reused as it stands)
#ifndef FD_FLASH_DIAG
#define FD_FLASH_DIAG 0
#endif
#ifndef FD_FLASH_TR_EARLY
#define FD_FLASH_TR_EARLY 1
#endif
// NQB: 16-query blocks per wave (2 = 32 queries, the register-heavy default; 1 = 16 queries in about half the
// VGPRs, so four waves share a SIMD and one wave's softmax VALU runs under another's MFMAs)
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// s_waitcnt vmcnt(PER * n) for a run-time n in [0, NMAX]
template <int PER, int NMAX>
__device__ __forceinline__ void wait_vm_tiles(int n) {
  if constexpr (NMAX > 0) {
    if (n >= NMAX) {
      wait_vm<PER * NMAX>();
      return;
    }
    wait_vm_tiles<PER, NMAX - 1>(n);
  } else {
    wait_vm<0>();
  }
}

// MXO: O is written as MX e4m3 (the use_fp8 model's out-projection operand): the fp32 normalised output of each
// (query, head) is two 32-column blocks, each spread over the 4 lanes of the query (xor 16 / 32 shuffles for its
// amax); bytes at O + b * obs + q * ldo + h * 64, E8M0 scales at osb[b * osbs + q * ldos + 2 h + {0, 1}].
template <typename T, int NWV, int NQB, int NBUF, bool MXO = false>
__global__ void __launch_bounds__(64 * NWV) __attribute__((amdgpu_waves_per_eu(NQB == 1 ? 4 : 1, NQB == 1 ? 4 : 2)))
flash_attn_d64_kernel(
    const T* __restrict__ Q, long long ldq, long long qbs, const T* __restrict__ K, long long ldk, long long kbs,
    const T* __restrict__ V, long long ldv, long long vbs, T* __restrict__ O, long long ldo, long long obs,
    int Lq, int Lk, int kv_mod, int causal, float scale_log2, int heads, int swz, uint8_t* __restrict__ osb = nullptr,
    long long ldos = 0, long long osbs = 0) {
  typedef typename VecT<T>::v8 V8;
  constexpr bool TR_EARLY = FD_FLASH_TR_EARLY;
  // NBUF-deep K/V ring: tile t+NBUF-1 is issued while tile t is consumed (counted vmcnt, raw s_barrier), so
  // each tile's load has NBUF-1 tiles of compute to land in.  (A software-pipelined variant -- scores of tile
  // t+1 under tile t's softmax, 4-deep ring -- measured 1.3x slower: 256 VGPRs and 4x the code.)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NBUF * 2 * 64 * 128];  // [buf][K|V][64 rows][128 B]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // 1-D grid; the q-blocks of one (batch, head) are contiguous after the XCD remap, so the head's K/V
  // stream is fetched into one L2 instead of all eight.
  constexpr int QB = 16 * NQB * NWV;  // queries per workgroup
  const int nq = (Lq + QB - 1) / QB;
  const int pid = swz ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int qblk = pid % nq, bh = pid / nq;
  const int h = bh % heads, b = bh / heads;
  const int kvb = kv_mod > 0 ? (b % kv_mod) : b;
  const T* Qb = Q + (long long)b * qbs + h * 64;
  const T* Kb = K + (long long)kvb * kbs + h * 64;
  const T* Vb = V + (long long)kvb * vbs + h * 64;
  const int q0 = qblk * QB + wave * 16 * NQB;
  const int fr = lane & 15, fg = lane >> 4;

  // Q fragments (B operand): lane holds Q[q0 + qb*16 + fr][ds*32 + 8*fg .. +7]
  V8 qf[NQB][2];
#pragma unroll
  for (int qb = 0; qb < NQB; ++qb) {
    int q = q0 + qb * 16 + fr;
    q = q < Lq ? q : Lq - 1;
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) qf[qb][ds] = *(const V8*)(Qb + (long long)q * ldq + ds * 32 + fg * 8);
  }
  constexpr bool QPRE = FD_FLASH_QPRE;
  if constexpr (QPRE) {
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb)
#pragma unroll
      for (int ds = 0; ds < 2; ++ds)
#pragma unroll
        for (int i = 0; i < 8; ++i) qf[qb][ds][i] = (T)((float)qf[qb][ds][i] * scale_log2);
  }

  const int lrow = lane >> 3, slot = lane & 7;
  constexpr int LPW = 8 / NWV;       // 8-row pieces of K (and of V) per wave per tile
  constexpr int PER = 2 * LPW;       // glds per wave per tile
  // per-lane byte offsets of this lane's K / V source rows inside a 64-key tile (XOR-swizzled 16-B chunk),
  // against a wave-uniform tile base that advances by 64 rows per tile: global_load_lds in saddr + voffset
  // form, no per-tile 64-bit address math
  unsigned koff[LPW], voff[LPW];
#pragma unroll
  for (int i = 0; i < LPW; ++i) {
    const int row = (i * NWV + wave) * 8 + lrow;
    koff[i] = (unsigned)(row * ldk + ((slot ^ ((row >> 1) & 7)) * 8)) * sizeof(T);
    voff[i] = (unsigned)(row * ldv + ((slot ^ (((row >> 1) & 3) << 1)) * 8)) * sizeof(T);
  }
  const int nt = (Lk + 63) / 64;
  auto stage = [&](int t, int bufi) {
    unsigned char* sk = smem + bufi * 16384;
    unsigned char* sv = sk + 8192;
    if (t * 64 + 64 <= Lk) {
      const char* kt = (const char*)(Kb + (long long)t * 64 * ldk);
      const char* vt = (const char*)(Vb + (long long)t * 64 * ldv);
#pragma unroll
      for (int i = 0; i < LPW; ++i) {
        __builtin_amdgcn_global_load_lds((const void*)(kt + koff[i]), LDS_PTR(sk + (i * NWV + wave) * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)(vt + voff[i]), LDS_PTR(sv + (i * NWV + wave) * 1024), 16, 0, 0);
      }
    } else {  // ragged last tile: rows past Lk re-read key Lk-1 (masked out of the softmax)
#pragma unroll
      for (int i = 0; i < LPW; ++i) {
        const int row = (i * NWV + wave) * 8 + lrow;
        const int key = min(t * 64 + row, Lk - 1);
        const int ck = slot ^ ((row >> 1) & 7);
        const int cv = slot ^ (((row >> 1) & 3) << 1);
        __builtin_amdgcn_global_load_lds((const void*)(Kb + (long long)key * ldk + ck * 8),
                                         LDS_PTR(sk + (i * NWV + wave) * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)(Vb + (long long)key * ldv + cv * 8),
                                         LDS_PTR(sv + (i * NWV + wave) * 1024), 16, 0, 0);
      }
    }
  };

  // lane-constant LDS read offsets (the buffer, key-block and half offsets are immediates):
  //   K fragment of (kb, ds): row kb*16 + fr, chunk (ds*4 + fg) ^ ((fr >> 1) & 7)
  //   V^T transposed read of (db, s, lo/hi): row 32s + 4fg + (fr>>2) (+16), chunk (2db + (pp>>1)) ^ sw
  int kro[2], vro[4];
#pragma unroll
  for (int ds = 0; ds < 2; ++ds) kro[ds] = fr * 128 + (((ds * 4 + fg) ^ ((fr >> 1) & 7)) << 4);
  {
    const int q = fr >> 2, pp = lane & 3;
    const int r0 = 4 * fg + q;
    const int sw = ((r0 >> 1) & 3) << 1;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const int col = db * 16 + 4 * pp;
      vro[db] = r0 * 128 + (((col >> 3) ^ sw) << 4) + (col & 7) * 2;
    }
  }

  f32x4 o[4][NQB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NQB; ++j) o[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float mrow[NQB];
#pragma unroll
  for (int j = 0; j < NQB; ++j) mrow[j] = QPRE ? 0.f : -INFINITY;
  f32x4 minit[NQB];  // QPRE: {-m} x 4, the score accumulators' starting value
#pragma unroll
  for (int j = 0; j < NQB; ++j) minit[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // softmax denominators on the MFMA pipe: lsum[qb] += ones(16 x 32) . P^T -- every row of the 16 x 16
  // block is the running sum for query column fr, of the same bf16 P the numerator uses (32 VALU adds
  // per tile traded for 4 MFMAs)
  f32x4 lsum[NQB];
#pragma unroll
  for (int j = 0; j < NQB; ++j) lsum[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  V8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (T)1.0f;

  typedef f32x4 Sc[4][NQB];
  // S^T(tile in buffer BUF) = K Q^T  (16 MFMAs)
  auto qk = [&](auto bufc, Sc& sd) {
    constexpr int BUF = decltype(bufc)::value;
    const unsigned char* sk = smem + BUF * 16384;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
      for (int qb = 0; qb < NQB; ++qb) sd[kb][qb] = QPRE ? minit[qb] : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < 2; ++ds) {
        const V8 kf = *(const V8*)(sk + kro[ds] + kb * 2048);
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) sd[kb][qb] = mfma16x16x32(kf, qf[qb][ds], sd[kb][qb]);
      }
    }
  };

  // V^T fragments of the tile in buffer BUF: inline asm, because hipcc treats the ds_read_tr builtin as
  // aliasing every in-flight LDS-DMA and drains vmcnt(0) in front of it (waiting out the K/V prefetch);
  // the asm reads are retired by an explicit lgkmcnt(0) + sched_barrier before the P.V MFMAs
  auto read_vtr = [&](auto bufc, s16x4 (&vtr)[4][2][2]) {
    constexpr int BUF = decltype(bufc)::value;
    // ds_read offsets are 16-bit: buffers from 32 KiB on move their base into the address register
    constexpr int HI = BUF * 16384 >= 32768 ? BUF * 16384 : 0, LO = BUF * 16384 - HI;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const unsigned va = (unsigned)(unsigned long)(LDS_PTR(smem + vro[db])) + HI;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vtr[db][s2][0]) : "v"(va),
                     "i"(LO + 8192 + s2 * 4096));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vtr[db][s2][1]) : "v"(va),
                     "i"(LO + 8192 + s2 * 4096 + 2048));
      }
    }
  };
  constexpr bool KPRE = FD_FLASH_KPRE;
  V8 kfr[KPRE ? 4 : 1][2];  // KPRE: K fragments of the next tile
  auto read_k = [&](auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    const unsigned char* sk = smem + BUF * 16384;
#pragma unroll
    for (int kb = 0; kb < (KPRE ? 4 : 1); ++kb)
#pragma unroll
      for (int ds = 0; ds < 2; ++ds) kfr[kb][ds] = *(const V8*)(sk + kro[ds] + kb * 2048);
  };
  auto qk_regs = [&](Sc& sd) {
#pragma unroll
    for (int kb = 0; kb < (KPRE ? 4 : 1); ++kb) {
#pragma unroll
      for (int qb = 0; qb < NQB; ++qb) sd[kb][qb] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < 2; ++ds)
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) sd[kb][qb] = mfma16x16x32(kfr[kb][ds], qf[qb][ds], sd[kb][qb]);
    }
  };
  const int nfull = Lk / 64;  // tiles with no key past Lk
#pragma unroll
  for (int i = 0; i < (KPRE ? NBUF : NBUF - 1); ++i)
    if (i < nt) stage(i, i);
  if constexpr (KPRE) {
    wait_vm_tiles<PER, NBUF - 1>(min(NBUF, nt) - 1);  // tile 0 landed
    __builtin_amdgcn_s_barrier();
    read_k(std::integral_constant<int, 0>());
  } else {
    wait_vm_tiles<PER, NBUF - 2>(min(NBUF - 1, nt) - 1);  // tile 0 landed
    __builtin_amdgcn_s_barrier();
  }

  // one 64-key tile in ring buffer BUF (compile-time, so every LDS address is base + immediate);
  // MASK: the ragged last tile (keys >= Lk scored -inf)
  auto iter = [&](auto bufc, auto maskc, int t) {
    constexpr int BUF = decltype(bufc)::value;
    constexpr bool MASK = decltype(maskc)::value;
    // buffer (BUF+NBUF-1)%NBUF was last read in the previous tile, which every wave finished before the barrier
    if (!KPRE && !FD_FLASH_DIAG && t + NBUF - 1 < nt) stage(t + NBUF - 1, (BUF + NBUF - 1) % NBUF);
    Sc sc;
    if constexpr (KPRE) qk_regs(sc);
    else qk(bufc, sc);
    s16x4 vtr[4][2][2];
    if (TR_EARLY) read_vtr(bufc, vtr);  // V^T reads in flight under the softmax VALU
    if (MASK) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = t * 64 + kb * 16 + fg * 4 + i;
          // ragged tail; causal (CLIP text encoders): query q0 + qb*16 + fr sees keys <= itself
#pragma unroll
          for (int qb = 0; qb < NQB; ++qb)
            if (key >= Lk || (causal && key > q0 + qb * 16 + fr)) sc[kb][qb][i] = -INFINITY;
        }
    }
    // ---- online softmax (one query per lane column; keys over fg groups, kb, i)
    V8 pf[NQB][2];
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb) {
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i) mx = fmaxf(mx, sc[kb][qb][i]);
      mx = xor_max_16_32(mx);
      if constexpr (QPRE) {
        // scores are already s * c - m: a query whose tile max is above its running max (or the first tile)
        // shifts by d; the others (d = 0) keep exp2(s') -- the same bits whether or not the branch runs
        float pv[4][4];
        const bool up = (t == 0) || (mx > 0.f);
        if (__any(up)) {
          const float d = (t == 0) ? mx : fmaxf(mx, 0.f);
#pragma unroll
          for (int kb = 0; kb < 4; ++kb)
#pragma unroll
            for (int i = 0; i < 4; ++i) pv[kb][i] = __builtin_amdgcn_exp2f(sc[kb][qb][i] - d);
          const float alpha = __builtin_amdgcn_exp2f(-d);
          lsum[qb] *= alpha;
#pragma unroll
          for (int db = 0; db < 4; ++db) o[db][qb] *= alpha;
          mrow[qb] += d;
          minit[qb] = (f32x4){-mrow[qb], -mrow[qb], -mrow[qb], -mrow[qb]};
        } else {
#pragma unroll
          for (int kb = 0; kb < 4; ++kb)
#pragma unroll
            for (int i = 0; i < 4; ++i) pv[kb][i] = __builtin_amdgcn_exp2f(sc[kb][qb][i]);
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          V8 v;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[i] = (T)pv[2 * s2][i];
            v[4 + i] = (T)pv[2 * s2 + 1][i];
          }
          pf[qb][s2] = v;
        }
        continue;
      }
      const float mnew = fmaxf(mrow[qb], mx * scale_log2);
      float pv[4][4];
      // raw v_exp_f32 (no denormal range fix-up: results below 2^-126 flush to 0, irrelevant to a softmax
      // numerator already divided by a sum >= 1)
      if constexpr (FD_FLASH_SFMA) {
        const float nm = -mnew;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int i = 0; i < 4; ++i) pv[kb][i] = __builtin_amdgcn_exp2f(fma_raw(sc[kb][qb][i], scale_log2, nm));
      } else {
        typedef __attribute__((ext_vector_type(2))) float f2;
        const f2 sc2 = {scale_log2, scale_log2}, mn2 = {-mnew, -mnew};
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int i = 0; i < 4; i += 2) {
            const f2 x = {sc[kb][qb][i], sc[kb][qb][i + 1]};
            const f2 y = __builtin_elementwise_fma(x, sc2, mn2);
            pv[kb][i] = __builtin_amdgcn_exp2f(y[0]);
            pv[kb][i + 1] = __builtin_amdgcn_exp2f(y[1]);
          }
      }
      // exact skip of the O / l rescale when no query of this wave raised its running max (most tiles
      // after the first few): alpha would be exactly 1
      if (__any(mnew != mrow[qb])) {
        const float alpha = __builtin_amdgcn_exp2f(mrow[qb] - mnew);
        lsum[qb] *= alpha;
#pragma unroll
        for (int db = 0; db < 4; ++db) o[db][qb] *= alpha;
      }
      mrow[qb] = mnew;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        V8 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = (T)pv[2 * s2][i];
          v[4 + i] = (T)pv[2 * s2 + 1][i];
        }
        pf[qb][s2] = v;
      }
    }
    // ---- O^T += V^T P^T   (A = V^T via transposed LDS reads)
    if (!TR_EARLY) read_vtr(bufc, vtr);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (KPRE) {
      // every wave is done with this tile's K (read one tile ago) and V^T (just waited): refill its buffer, and
      // read the next tile's K under the P.V MFMAs
      if (t + 1 < nt) {
        if (t + NBUF - 1 < nt) wait_vm<PER * (NBUF - 2)>();
        else wait_vm_tiles<PER, NBUF - 2>(nt - 2 - t);
        __builtin_amdgcn_s_barrier();
        if (t + NBUF < nt) stage(t + NBUF, BUF);
        read_k(std::integral_constant<int, (BUF + 1) % NBUF>());
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int db = 0; db < 4; ++db) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const s16x4 lo = vtr[db][s2][0], hi = vtr[db][s2][1];
        typedef __attribute__((ext_vector_type(8))) short s16x8;
        const s16x8 w = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const V8 vf = __builtin_bit_cast(V8, w);
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) o[db][qb] = mfma16x16x32(vf, pf[qb][s2], o[db][qb]);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
      for (int qb = 0; qb < NQB; ++qb) lsum[qb] = mfma16x16x32(ones, pf[qb][s2], lsum[qb]);
    }
    if (!KPRE && t + 1 < nt) {
      // tile t+1 landed (tiles t+2 .. t+NBUF-1, where issued, may still fly); every wave done reading tile t
      if (t + NBUF - 1 < nt) wait_vm<PER * (NBUF - 2)>();
      else wait_vm_tiles<PER, NBUF - 2>(nt - 2 - t);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_s_barrier();
    }
  };
  typedef std::integral_constant<bool, false> NM;
  typedef std::integral_constant<bool, true> YM;
  int t = 0;
  for (; !causal && t + NBUF <= nfull; t += NBUF) {
    [&]<int... I>(std::integer_sequence<int, I...>) {
      (iter(std::integral_constant<int, I>(), NM(), t + I), ...);
    }(std::make_integer_sequence<int, NBUF>());
  }
  // the remaining full tiles and the ragged tail (buffer index t % NBUF continues the ring)
  for (; t < nt; ++t) {
    const bool m = causal || t >= nfull;
    [&]<int... I>(std::integer_sequence<int, I...>) {
      ((t % NBUF == I ? (m ? iter(std::integral_constant<int, I>(), YM(), t)
                           : iter(std::integral_constant<int, I>(), NM(), t)), 0 : 0), ...);
    }(std::make_integer_sequence<int, NBUF>());
  }

  // ---- finalise: lane holds O^T[d = db*16 + 4*fg + j][q = qb*16 + fr]
#pragma unroll
  for (int qb = 0; qb < NQB; ++qb) {
    const float inv = 1.0f / lsum[qb][0];
    const int q = q0 + qb * 16 + fr;
    if constexpr (MXO) {
      float am[2] = {0.f, 0.f};
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int j = 0; j < 4; ++j) am[db >> 1] = fmaxf(am[db >> 1], fabsf(o[db][qb][j] * inv));
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        am[c] = fmaxf(am[c], __shfl_xor(am[c], 16, 64));
        am[c] = fmaxf(am[c], __shfl_xor(am[c], 32, 64));
      }
      if (q >= Lq) continue;
      const int E0 = mx_exp(am[0]), E1 = mx_exp(am[1]);
      uint8_t* o8 = (uint8_t*)O + (long long)b * obs + (long long)q * ldo + h * 64;
#pragma unroll
      for (int db = 0; db < 4; ++db)
        *(unsigned*)(o8 + db * 16 + fg * 4) = mx_pack4(o[db][qb][0] * inv, o[db][qb][1] * inv, o[db][qb][2] * inv,
                                                       o[db][qb][3] * inv, db < 2 ? E0 : E1);
      if (fg == 0) {
        uint8_t* sr = osb + (long long)b * osbs + (long long)q * ldos + h * 2;
        sr[0] = (uint8_t)(E0 + 127);
        sr[1] = (uint8_t)(E1 + 127);
      }
      continue;
    }
    if (q >= Lq) continue;
    T* orow = O + (long long)b * obs + (long long)q * ldo + h * 64;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      typedef __attribute__((ext_vector_type(4))) T T4;
      T4 w;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = (T)(o[db][qb][j] * inv);
      st_out8((T4*)(orow + db * 16 + fg * 4), w);
    }
  }
}

static int flash_d64(const void* q, long long ldq, long long qbs, const void* k, long long ldk, long long kbs,
                     const void* v, long long ldv, long long vbs, void* o, long long ldo, long long obs, int batch,
                     int heads, int Lq, int Lk, int kv_mod, int causal, float scale, int dtype, uint8_t* osb,
                     long long ldos, long long osbs, void* stream) {
  if (!q || !k || !v || !o) return FD_ERR_ARG;
  if (batch <= 0 || heads <= 0 || Lq <= 0 || Lk <= 0 || kv_mod < 0) return FD_ERR_SHAPE;
  if ((ldq | ldk | ldv | ldo) & 7) return FD_ERR_SHAPE;
  const int swz = fd_knob(FDK_FLASH_SWZ);
  int nwv = fd_knob(FDK_FLASH_WAVES);  // waves per workgroup: 4 (default), 2 or 8
  const int qpw = fd_knob(FDK_FLASH_QPW);  // queries per wave: 32 or 16 (0: by launch size, below)
  const int nqb = qpw == 0 ? 0 : (qpw == 16 ? 1 : 2);
  if (nwv != 2 && nwv != 8) nwv = 4;
  // 16 queries per wave (half the VGPRs: three waves per SIMD, one wave's softmax under another's MFMAs) while
  // the 32-query grid would give at most 4 workgroups per CU (scripts/attn_var.sh: C2's L = 1024 28.3 -> 24.4 us,
  // L = 4096 134 -> 127 us, cross-attention 8.6 -> 7.6 us); past that the 32-query kernel's fewer K/V fragment
  // reads per flop win (26 CFG-batched tiles: 200 vs 215 us).  Every query sees the same operations in either
  // form, so the choice changes no bit.
  int nq = nqb;
  if (nq == 0) nq = (long long)((Lq + 127) / 128) * heads * batch <= 1024 ? 1 : 2;
  const int nw = (nwv == 8 && nq == 2) ? 4 : nwv;
  const int QB = 16 * nq * nw;
  const long long nblk = (long long)((Lq + QB - 1) / QB) * heads * batch;
  if (nblk > 0x7fffffff) return FD_ERR_SHAPE;
  dim3 grid((unsigned)nblk), block(64 * nw);
  const float sl2 = scale * 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
#define FD_FLASH(NW_, NQ_)                                                                                      \
  if (osb) {                                                                                                     \
    if (dtype != FD_BF16) return FD_ERR_DTYPE;                                                                  \
    hipLaunchKernelGGL((flash_attn_d64_kernel<bf16, NW_, NQ_, FLASH_NBUF, true>), grid, block, 0, s, (const bf16*)q, \
                       ldq, qbs, (const bf16*)k, ldk, kbs, (const bf16*)v, ldv, vbs, (bf16*)o, ldo, obs, Lq, Lk,   \
                       kv_mod, causal, sl2, heads, swz, osb, ldos, osbs);                                        \
  } else                                                                                                         \
  FD_DISPATCH_T(dtype, hipLaunchKernelGGL((flash_attn_d64_kernel<T, NW_, NQ_, FLASH_NBUF>), grid, block, 0, s, (const T*)q, ldq, \
                                          qbs, (const T*)k, ldk, kbs, (const T*)v, ldv, vbs, (T*)o, ldo, obs, Lq, Lk, \
                                          kv_mod, causal, sl2, heads, swz))
  if (nq == 2 && nw == 4) {
    FD_FLASH(4, 2);
  } else if (nq == 2) {
    FD_FLASH(2, 2);
  } else if (nw == 4) {
    FD_FLASH(4, 1);
  } else if (nw == 8) {
    FD_FLASH(8, 1);
  } else {
    FD_FLASH(2, 1);
  }
#undef FD_FLASH
  FD_LAUNCH_CHECK();
  return FD_OK;
}

extern "C" int fd_flash_attn(const void* q, long long ldq, long long qbs, const void* k, long long ldk,
                             long long kbs, const void* v, long long ldv, long long vbs, void* o, long long ldo,
                             long long obs, int batch, int heads, int Lq, int Lk, int kv_mod, int causal,
                             float scale, int dtype, void* stream) {
  return flash_d64(q, ldq, qbs, k, ldk, kbs, v, ldv, vbs, o, ldo, obs, batch, heads, Lq, Lk, kv_mod, causal, scale,
                   dtype, nullptr, 0, 0, stream);
}

extern "C" int fd_flash_attn_mx(const void* q, long long ldq, long long qbs, const void* k, long long ldk,
                                long long kbs, const void* v, long long ldv, long long vbs, void* o8, long long ldo,
                                long long obs, void* osb, long long ldos, long long osbs, int batch, int heads, int Lq,
                                int Lk, int kv_mod, int causal, float scale, int dtype, void* stream) {
  if (!osb) return FD_ERR_ARG;
  if ((((unsigned long long)o8) & 3) || (ldo & 3) || (obs & 3) || ldos < 2 * heads) return FD_ERR_SHAPE;
  return flash_d64(q, ldq, qbs, k, ldk, kbs, v, ldv, vbs, o8, ldo, obs, batch, heads, Lq, Lk, kv_mod, causal, scale,
                   dtype, (uint8_t*)osb, ldos, osbs, stream);
}

// ------------------------------------------------------------------------------------------------
// flash_attn_d512: single-head d = 512 attention of the VAE mid block (diffusers Attention with one head of 512
// channels and upcast softmax; pipeline_FaithDiff_tlc.py:1436-1442 decodes through it, T = 16384 at 1024^2) --
// the [T, T] score and probability matrices (1.5 GB at T = 16384) are never formed.  One workgroup = NW waves x
// 16 queries; K / V tiles of 32 keys x 512 (32 KB each) double-buffered in LDS by global_load_lds (128 KB: one
// workgroup per CU).  Per tile and wave: S^T = K Q^T (32 MFMAs, Q fragments held in 64 VGPRs), online softmax in
// fp32 (one query per lane column, as flash_attn_d64), O^T += V^T P^T (32 MFMAs, O^T in 128 VGPRs, V^T fragments by
// ds_read_b64_tr_b16), denominators on the MFMA pipe (ones . P^T).
// LDS rows are 1024 B, so both tiles are XOR-swizzled at the source (K: 16-B chunk ^ (row & 15) for the 16-row
// ds_read_b128 fragments; V: chunk ^ 2 (row & 7) for the 8-row transposed reads) -- conflict-free reads.
// What bounds it: every workgroup streams the image's whole K and V (32 MB at T = 16384) through its CU, one 64-KB
// tile in flight -- ~30 GB/s per CU from the Infinity Cache, not the MFMAs.  NW = 8 (two waves per SIMD, 128
// queries per tile fetch) halves the bytes per flop; the keys are then split over `ks` workgroups per query block
// (so the grid still covers the CUs), each writing its O / l in fp32 and its log2-sum-exp to `part`, and
// flash_d512_combine_kernel merges the splits in split order (r05).
template <typename T, int NW, int QPW>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW / 4, NW / 4)))
flash_attn_d512_kernel(const T* __restrict__ Q, const T* __restrict__ K, const T* __restrict__ V, long long ld,
                       long long bs, T* __restrict__ O, long long ldo, long long obs, int L, float scale_log2,
                       float* __restrict__ part, int ks, int nbatch) {
  typedef typename VecT<T>::v8 V8;
  constexpr int KT = 32;            // keys per tile
  constexpr int TB = KT * 1024;     // bytes of one K (or V) tile in LDS
  constexpr int QB = 16 * NW * QPW; // queries per workgroup (QPW groups of 16 per wave)
  constexpr int RPW = KT / NW;      // K / V rows each wave stages per tile
  constexpr int JG = NW == 8 ? 4 : 8;  // V^T d-blocks read per LDS wait (VGPR budget at two waves per SIMD)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[4 * TB];  // [buf][K | V]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nq = (L + QB - 1) / QB;
  const int h = blockIdx.x % ks, qb = blockIdx.x / ks;
  const int qblk = qb % nq, b = qb / nq;
  const T* Qb = Q + (long long)b * bs;
  const T* Kb = K + (long long)b * bs;
  const T* Vb = V + (long long)b * bs;
  const int q0 = qblk * QB + wave * 16 * QPW;
  const int fr = lane & 15, fg = lane >> 4;
  const int nt = (L + KT - 1) / KT;
  const int nts = (nt + ks - 1) / ks;
  const int t0 = h * nts, t1 = min(nt, t0 + nts);

  V8 qf[QPW][16];  // B operand: Q[q0 + 16 u + fr][32 ds + 8 fg .. +7]
#pragma unroll
  for (int u = 0; u < QPW; ++u) {
    const int q = min(q0 + 16 * u + fr, L - 1);
#pragma unroll
    for (int ds = 0; ds < 16; ++ds) qf[u][ds] = *(const V8*)(Qb + (long long)q * ld + ds * 32 + fg * 8);
  }
  // DMA: wave w stages K / V rows r = w + NW i (i < RPW); lane l fills LDS chunk l of the row with source chunk
  // l ^ swz(r) (the swizzle is an involution on 0..63)
  auto stage = [&](int t, int bi) {
    unsigned char* sk = smem + bi * 2 * TB;
    unsigned char* sv = sk + TB;
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int r = wave + NW * i;
      const long long key = min(t * KT + r, L - 1);  // ragged last tile: rows past L re-read key L-1 (scored -inf)
      __builtin_amdgcn_global_load_lds((const void*)(Kb + key * ld + (lane ^ (r & 15)) * 8), LDS_PTR(sk + r * 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(Vb + key * ld + (lane ^ (2 * (r & 7))) * 8),
                                       LDS_PTR(sv + r * 1024), 16, 0, 0);
    }
  };
  // lane-constant LDS read offsets.  K fragment (kb, ds): row kb*16 + fr, chunk (4 ds + fg) ^ fr =
  //   16 (ds >> 2) + 4 ((ds & 3) ^ (fr >> 2)) + (fg ^ (fr & 3))  ->  base kro[ds & 3] + 256 (ds >> 2) + 16384 kb.
  // V^T (db = 8 dg + j, lo / hi): row r0 = 4 fg + (fr >> 2) (+16), element column 16 db + 4 (fr & 3):
  //   chunk 2 (db ^ (r0 & 7)) + ((fr & 3) >> 1), +8 B for odd (fr & 3)  ->  base vro[j] + 256 dg (+16384 hi).
  int kro[4], vro[8];
#pragma unroll
  for (int d4 = 0; d4 < 4; ++d4) kro[d4] = fr * 1024 + 16 * (4 * (d4 ^ (fr >> 2)) + (fg ^ (fr & 3)));
  {
    const int r0 = 4 * fg + (fr >> 2), pp = fr & 3;
#pragma unroll
    for (int j = 0; j < 8; ++j) vro[j] = r0 * 1024 + 32 * (j ^ (r0 & 7)) + 16 * (pp >> 1) + 8 * (pp & 1);
  }

  f32x4 o[QPW][32], lsum[QPW];
  float mrow[QPW];
#pragma unroll
  for (int u = 0; u < QPW; ++u) {
#pragma unroll
    for (int i = 0; i < 32; ++i) o[u][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    lsum[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
    mrow[u] = -INFINITY;
  }
  V8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (T)1.0f;

  if (t0 < t1) {
    stage(t0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  for (int t = t0; t < t1; ++t) {
    const int bi = (t - t0) & 1;
    if (t + 1 < t1) stage(t + 1, bi ^ 1);  // buffer bi^1 held tile t-1: every wave passed the barrier after it
    const unsigned char* sk = smem + bi * 2 * TB;
    f32x4 sc[QPW][2];
#pragma unroll
    for (int u = 0; u < QPW; ++u) sc[u][0] = sc[u][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ds = 0; ds < 16; ++ds) {
        const V8 kf = *(const V8*)(sk + kro[ds & 3] + 256 * (ds >> 2) + 16384 * kb);  // one read, QPW MFMAs
#pragma unroll
        for (int u = 0; u < QPW; ++u) sc[u][kb] = mfma16x16x32(kf, qf[u][ds], sc[u][kb]);
      }
    V8 pf[QPW];
#pragma unroll
    for (int u = 0; u < QPW; ++u) {
      if (t * KT + KT > L) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (t * KT + kb * 16 + fg * 4 + i >= L) sc[u][kb][i] = -INFINITY;
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i) mx = fmaxf(mx, sc[u][kb][i]);
      mx = xor_max_16_32(mx);
      const float mnew = fmaxf(mrow[u], mx * scale_log2);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          pf[u][kb * 4 + i] = (T)__builtin_amdgcn_exp2f(fmaf(sc[u][kb][i], scale_log2, -mnew));
      if (__any(mnew != mrow[u])) {  // exact skip when no query of this group raised its running max
        const float alpha = __builtin_amdgcn_exp2f(mrow[u] - mnew);
        lsum[u] *= alpha;
#pragma unroll
        for (int i = 0; i < 32; ++i) o[u][i] *= alpha;
      }
      mrow[u] = mnew;
    }
    // O^T += V^T P^T in groups of JG d-blocks (transposed V reads by inline asm: the builtin makes hipcc drain
    // vmcnt(0) -- the next tile's DMA -- in front of it); each V^T fragment feeds QPW MFMAs
    const unsigned vb = (unsigned)(unsigned long)LDS_PTR(smem + bi * 2 * TB + TB);
#pragma unroll
    for (int dg = 0; dg < 4; ++dg)
#pragma unroll
      for (int jh = 0; jh < 8 / JG; ++jh) {
        s16x4 vtr[JG][2];
#pragma unroll
        for (int jj = 0; jj < JG; ++jj) {
          const int j = jh * JG + jj;
          asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vtr[jj][0]) : "v"(vb + vro[j]), "i"(256 * dg));
          asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vtr[jj][1]) : "v"(vb + vro[j]),
                       "i"(256 * dg + 16384));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int jj = 0; jj < JG; ++jj) {
          typedef __attribute__((ext_vector_type(8))) short s16x8;
          const s16x4 lo = vtr[jj][0], hi = vtr[jj][1];
          const s16x8 w = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
          for (int u = 0; u < QPW; ++u)
            o[u][dg * 8 + jh * JG + jj] = mfma16x16x32(__builtin_bit_cast(V8, w), pf[u], o[u][dg * 8 + jh * JG + jj]);
        }
      }
#pragma unroll
    for (int u = 0; u < QPW; ++u) lsum[u] = mfma16x16x32(ones, pf[u], lsum[u]);
    if (t + 1 < t1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t+1 landed
      __builtin_amdgcn_s_waitcnt(0xc07f);                // this wave's reads of tile t retired
      __builtin_amdgcn_s_barrier();
    }
  }
  // lane holds O^T[d = 16 db + 4 fg + j][q = q0 + 16 u + fr]
#pragma unroll
  for (int u = 0; u < QPW; ++u) {
    const int q = q0 + 16 * u + fr;
    if (q >= L) continue;
    const float inv = lsum[u][0] > 0.f ? 1.0f / lsum[u][0] : 0.f;
    if (!part) {
      T* orow = O + (long long)b * obs + (long long)q * ldo;
      typedef __attribute__((ext_vector_type(4))) T T4;
#pragma unroll
      for (int db = 0; db < 32; ++db) {
        T4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = (T)(o[u][db][j] * inv);
        st_out8((T4*)(orow + db * 16 + fg * 4), w);
      }
      continue;
    }
    // split partial: O / l (fp32) and log2(sum_j 2^(s_j scale_log2)) = m + log2(l) (-inf for an empty key range)
    const long long row = ((long long)b * ks + h) * L + q;
    float* prow = part + row * 512;
#pragma unroll
    for (int db = 0; db < 32; ++db) *(f32x4*)(prow + db * 16 + fg * 4) = o[u][db] * inv;
    if (fg == 0)
      part[(long long)nbatch * ks * L * 512 + row] = lsum[u][0] > 0.f ? mrow[u] + __log2f(lsum[u][0]) : -INFINITY;
  }
}

// Merge of the key splits: O = sum_h w_h (O_h / l_h) / sum_h w_h with w_h = 2^(lse_h - max_h lse_h), in split
// order.  64 threads per output row, 8 channels each.
template <typename T>
__global__ void __launch_bounds__(256) flash_d512_combine_kernel(const float* __restrict__ part, int ks, int nbatch,
                                                                 int L, T* __restrict__ O, long long ldo,
                                                                 long long obs) {
  const long long rr = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (rr >= (long long)nbatch * L) return;
  const int b = (int)(rr / L), q = (int)(rr - (long long)b * L);
  const int c = (threadIdx.x & 63) * 8;
  const float* lse = part + (long long)nbatch * ks * L * 512;
  float mx = -INFINITY;
  for (int h = 0; h < ks; ++h) mx = fmaxf(mx, lse[((long long)b * ks + h) * L + q]);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, den = 0.f;
  for (int h = 0; h < ks; ++h) {
    const long long row = ((long long)b * ks + h) * L + q;
    const float w = __builtin_amdgcn_exp2f(lse[row] - mx);  // 0 for an empty split (lse -inf)
    const f32x4 v0 = *(const f32x4*)(part + row * 512 + c), v1 = *(const f32x4*)(part + row * 512 + c + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[j] = fmaf(w, v0[j], acc[j]);
      acc[4 + j] = fmaf(w, v1[j], acc[4 + j]);
    }
    den += w;
  }
  const float inv = 1.0f / den;
  typedef typename VecT<T>::v8 V8;
  V8 out;
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = (T)(acc[j] * inv);
  st_out16((V8*)(O + (long long)b * obs + (long long)q * ldo + c), out);
}

static int d512_check(const void* q, const void* k, const void* v, long long ld, long long bs, const void* o,
                      long long ldo, long long obs, int batch, int L) {
  if (!q || !k || !v || !o) return FD_ERR_ARG;
  if (batch <= 0 || L <= 0 || (long long)batch * ((L + 63) / 64) * 8 > 0x7fffffff) return FD_ERR_SHAPE;
  if ((ld & 7) || (ldo & 3) || ld < 512 || ldo < 512 || (bs & 7) || (obs & 3)) return FD_ERR_SHAPE;
  if ((((unsigned long long)q) | ((unsigned long long)k) | ((unsigned long long)v)) & 15) return FD_ERR_ARG;
  if (((unsigned long long)o) & 7) return FD_ERR_ARG;
  return FD_OK;
}

extern "C" int fd_flash_attn_d512(const void* q, const void* k, const void* v, long long ld, long long bs, void* o,
                                  long long ldo, long long obs, int batch, int L, float scale, int dtype,
                                  void* stream) {
  const int rc = d512_check(q, k, v, ld, bs, o, ldo, obs, batch, L);
  if (rc != FD_OK) return rc;
  dim3 grid((unsigned)(batch * ((L + 63) / 64))), block(256);
  const float sl2 = scale * 1.4426950408889634f;
  FD_DISPATCH_T(dtype, hipLaunchKernelGGL((flash_attn_d512_kernel<T, 4, 1>), grid, block, 0, (hipStream_t)stream,
                                          (const T*)q, (const T*)k, (const T*)v, ld, bs, (T*)o, ldo, obs, L, sl2,
                                          (float*)nullptr, 1, batch));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

extern "C" int fd_flash_attn_d512_ksplit(int batch, int L) {
  if (batch <= 0 || L <= 0) return 1;
  const long long wgs = (long long)batch * ((L + 127) / 128);
  const int nt = (L + 31) / 32;
  int ks = 1;
  while (ks < 8 && wgs * ks * 2 <= 320 && nt / (ks * 2) >= 4) ks *= 2;
  return ks;
}

extern "C" int fd_flash_attn_d512_split(const void* q, const void* k, const void* v, long long ld, long long bs,
                                        void* o, long long ldo, long long obs, int batch, int L, float scale,
                                        int dtype, float* part, long long part_floats, int ks, void* stream) {
  const int rc = d512_check(q, k, v, ld, bs, o, ldo, obs, batch, L);
  if (rc != FD_OK) return rc;
  if (ks < 1 || ks > 64) return FD_ERR_SHAPE;
  if (ks > 1 && (!part || (((unsigned long long)part) & 15))) return FD_ERR_ARG;
  if (ks > 1 && part_floats < (long long)batch * ks * L * 513) return FD_ERR_SHAPE;
  if (ks > 1 && ((ldo & 7) || (obs & 7) || (((unsigned long long)o) & 15))) return FD_ERR_SHAPE;  // combine: 16-B rows
  dim3 grid((unsigned)(batch * ((L + 127) / 128) * ks));
  const float sl2 = scale * 1.4426950408889634f;
  float* pp = ks > 1 ? part : (float*)nullptr;
  // 8 waves x 16 queries (two waves per SIMD).  4 waves x 32 queries (QPW = 2: each K / V^T fragment read feeding
  // two MFMAs) needs 256 O accumulators + 128 Q registers per wave and spills 78-388 VGPRs in either register form.
  FD_DISPATCH_T(dtype, hipLaunchKernelGGL((flash_attn_d512_kernel<T, 8, 1>), grid, dim3(512), 0, (hipStream_t)stream,
                                          (const T*)q, (const T*)k, (const T*)v, ld, bs, (T*)o, ldo, obs, L, sl2, pp,
                                          ks, batch));
  FD_LAUNCH_CHECK();
  if (ks > 1) {
    dim3 g2((unsigned)(((long long)batch * L + 3) / 4)), b2(256);
    FD_DISPATCH_T(dtype, hipLaunchKernelGGL((flash_d512_combine_kernel<T>), g2, b2, 0, (hipStream_t)stream,
                                            (const float*)part, ks, batch, L, (T*)o, ldo, obs));
    FD_LAUNCH_CHECK();
  }
  return FD_OK;
}

// ------------------------------------------------------------------------------------------------
// MultiheadAttention over the sequence axis L (the CFG pair) for every pixel n, grouped: rows
// [g*L, (g+1)*L) of the batch form one attention problem.  qkv [Btot][N][3E] -> o [Btot][N][E].
// One thread per (group, pixel, head) computes all L query rows; the heads of a pixel are adjacent
// threads, so a wave reads whole contiguous q/k/v rows with 16-B loads.  HBM-bound (reads qkv once).
template <typename T, int HD, int LMAX>
__global__ void __launch_bounds__(256) mha_seq_axis_kernel(const T* __restrict__ qkv, T* __restrict__ o, int L,
                                                           int groups, int N, int E, int heads) {
  typedef typename VecT<T>::v8 V8;
  constexpr int NV = HD / 8;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)groups * N * heads;
  if (idx >= total) return;
  const int h = idx % heads;
  const long long r = idx / heads;
  const int n = r % N;
  const int g = r / N;
  const float scale = rsqrtf((float)HD);
  const long long E3 = 3LL * E;
  float q[LMAX][HD];
  float s[LMAX][LMAX];
#pragma unroll
  for (int l = 0; l < LMAX; ++l) {
    if (l >= L) break;
    const T* row = qkv + ((long long)(g * L + l) * N + n) * E3 + h * HD;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const V8 x = *(const V8*)(row + v * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) q[l][v * 8 + i] = (float)x[i];
    }
  }
#pragma unroll
  for (int l2 = 0; l2 < LMAX; ++l2) {
    if (l2 >= L) break;
    const T* krow = qkv + ((long long)(g * L + l2) * N + n) * E3 + E + h * HD;
    float acc[LMAX];
#pragma unroll
    for (int l1 = 0; l1 < LMAX; ++l1) acc[l1] = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const V8 x = *(const V8*)(krow + v * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int l1 = 0; l1 < LMAX; ++l1) acc[l1] += q[l1][v * 8 + i] * (float)x[i];
    }
#pragma unroll
    for (int l1 = 0; l1 < LMAX; ++l1) s[l1][l2] = acc[l1] * scale;
  }
#pragma unroll
  for (int l1 = 0; l1 < LMAX; ++l1) {
    if (l1 >= L) break;
    float mx = -INFINITY;
    for (int l2 = 0; l2 < L; ++l2) mx = fmaxf(mx, s[l1][l2]);
    float den = 0.f;
    for (int l2 = 0; l2 < L; ++l2) {
      s[l1][l2] = __expf(s[l1][l2] - mx);
      den += s[l1][l2];
    }
    const float inv = 1.f / den;
    for (int l2 = 0; l2 < L; ++l2) s[l1][l2] *= inv;
  }
  // o[l1] = sum_l2 p[l1][l2] v[l2]   (q registers reused as the accumulator)
#pragma unroll
  for (int l1 = 0; l1 < LMAX; ++l1)
#pragma unroll
    for (int d = 0; d < HD; ++d) q[l1][d] = 0.f;
#pragma unroll
  for (int l2 = 0; l2 < LMAX; ++l2) {
    if (l2 >= L) break;
    const T* vrow = qkv + ((long long)(g * L + l2) * N + n) * E3 + 2 * E + h * HD;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const V8 x = *(const V8*)(vrow + v * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int l1 = 0; l1 < LMAX; ++l1) q[l1][v * 8 + i] += s[l1][l2] * (float)x[i];
    }
  }
#pragma unroll
  for (int l1 = 0; l1 < LMAX; ++l1) {
    if (l1 >= L) break;
    T* orow = o + ((long long)(g * L + l1) * N + n) * E + h * HD;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      V8 y;
#pragma unroll
      for (int i = 0; i < 8; ++i) y[i] = (T)q[l1][v * 8 + i];
      *(V8*)(orow + v * 8) = y;
    }
  }
}

extern "C" int fd_mha_seq_axis(const void* qkv, void* o, int L, int groups, int N, int E, int heads, int dtype,
                               void* stream) {
  if (!qkv || !o) return FD_ERR_ARG;
  if (L <= 0 || L > 2 || groups <= 0 || N <= 0 || heads <= 0 || E % heads || E / heads != 80) return FD_ERR_SHAPE;
  const long long total = (long long)groups * N * heads;
  dim3 grid((unsigned)((total + 255) / 256)), block(256);
  hipStream_t s = (hipStream_t)stream;
  FD_DISPATCH_T(dtype, hipLaunchKernelGGL((mha_seq_axis_kernel<T, 80, 2>), grid, block, 0, s, (const T*)qkv, (T*)o, L,
                                          groups, N, E, heads));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// ------------------------------------------------------------------------------------------------
// fp32 row softmax: p[r][c] = exp(scale*s - max) / sum  (one 256-thread block per row)
template <typename TO>
__global__ void __launch_bounds__(256) softmax_rows_kernel(const float* __restrict__ s, TO* __restrict__ p, int C,
                                                           long long ldp, float scale) {
  __shared__ float red[8];
  const long long r = blockIdx.x;
  const float* row = s + r * C;
  TO* out = p + r * ldp;
  float mx = -INFINITY;
  for (int c = threadIdx.x; c < C; c += 256) mx = fmaxf(mx, row[c] * scale);
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int c = threadIdx.x; c < C; c += 256) sum += __expf(row[c] * scale - mx);
  sum = wave_sum(sum);
  if ((threadIdx.x & 63) == 0) red[4 + (threadIdx.x >> 6)] = sum;
  __syncthreads();
  const float inv = 1.f / (red[4] + red[5] + red[6] + red[7]);
  for (int c = threadIdx.x; c < C; c += 256) out[c] = (TO)(__expf(row[c] * scale - mx) * inv);
}

extern "C" int fd_softmax_rows(const float* s, void* p, int R, int C, long long ldp, float scale, int dtype,
                               void* stream) {
  if (!s || !p) return FD_ERR_ARG;
  if (R <= 0 || C <= 0 || ldp < C) return FD_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  FD_DISPATCH_O(dtype, hipLaunchKernelGGL(softmax_rows_kernel<TO>, dim3(R), dim3(256), 0, st, s, (TO*)p, C, ldp, scale));
  FD_LAUNCH_CHECK();
  return FD_OK;
}

// ------------------------------------------------------------------------------------------------
// Cross-attention as two GEMMs (fdhip/unet.py, HipUNet.set_context): per prompt row r the score matrix
// B1[r] = scale * blockdiag_h(K_r,h) . W_q' (rows h * slot + j, one per (head, key), W_q' = W_q diag(gamma) of the
// folded norm2) is written by a batched GEMM; this kernel adds the LayerNorm-fold constants of those rows:
//   c[n] = sum_k B1[n][k]                                   (of the stored 16-bit values, fixed order)
//   d[n] = scale * sum_e K_r[j][h * 64 + e] * dq[h * 64 + e]  (dq = W_q . beta, fp32; 0 for pad keys j >= Lk)
// so the score GEMM's epilogue computes rstd (x . B1^T - mean c) + d = scale * LN(x) W_q^T K^T.  One wave per row.
template <typename T>
__global__ void __launch_bounds__(256) xattn_consts_kernel(const T* __restrict__ B1, long long ldb, int rows, int K,
                                                            const T* __restrict__ kv, long long ldkv,
                                                            long long kv_rstride, const float* __restrict__ dq,
                                                            int heads, int slot, int Lk, float scale,
                                                            float* __restrict__ c, float* __restrict__ d) {
  typedef typename VecT<T>::v8 V8;
  const int lane = threadIdx.x & 63;
  const long long n = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= rows) return;
  const T* row = B1 + n * ldb;
  float s = 0.f;
  for (int v = lane; v < K / 8; v += 64) {
    const V8 x = *(const V8*)(row + v * 8);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += (float)x[i];
  }
  s = wave_sum(s);
  const int j = (int)(n % slot), h = (int)((n / slot) % heads);
  const long long r = n / ((long long)slot * heads);
  float t = 0.f;
  if (j < Lk) t = (float)kv[r * kv_rstride + (long long)j * ldkv + h * 64 + lane] * dq[h * 64 + lane];
  t = wave_sum(t);
  if (lane == 0) {
    c[n] = s;
    d[n] = j < Lk ? scale * t : 0.f;
  }
}

extern "C" int fd_xattn_consts(const void* B1, long long ldb, int rows, int K, const void* kv, long long ldkv,
                               long long kv_rstride, const float* dq, int heads, int slot, int Lk, float scale,
                               float* c, float* d, int dtype, void* stream) {
  if (!B1 || !kv || !dq || !c || !d) return FD_ERR_ARG;
  if (rows <= 0 || K <= 0 || K % 8 || ldb % 8 || heads <= 0 || slot <= 0 || Lk <= 0 || Lk > slot ||
      rows % (slot * heads))
    return FD_ERR_SHAPE;
  if ((((unsigned long long)B1) & 15)) return FD_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  FD_DISPATCH_T(dtype, hipLaunchKernelGGL(xattn_consts_kernel<T>, dim3((rows + 3) / 4), dim3(256), 0, st,
                                          (const T*)B1, ldb, rows, K, (const T*)kv, ldkv, kv_rstride, dq, heads,
                                          slot, Lk, scale, c, d));
  FD_LAUNCH_CHECK();
  return FD_OK;
}
