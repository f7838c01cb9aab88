// Ping-pong MFMA GEMM core for gfx950 -- prototype + A/B against libfaithdiff_hip's fd_gemm in one process.
//
// C[M][N] (bf16) = A[M][K] . B[N][K]^T, fp32 accumulation on v_mfma_f32_16x16x32_bf16.
// 512 threads = two wave groups of 4 (waves 0-3 = group 0, 4-7 = group 1; wave w and w+4 share a SIMD).  Group g
// owns output rows [g*BM/2, (g+1)*BM/2) of the BM x BN tile, its 4 waves GW_M x GW_N.  A "phase" is one 32-deep K
// slice; every wave runs, per phase, a LOAD segment (its fragment ds_reads for the phase, its share of a later K tile's
// LDS-DMA, the counted vmcnt) and a COMPUTE segment (lgkmcnt(0) + the phase's MFMAs), each closed by s_barrier.
// Group 1 starts one barrier late, so on every SIMD one wave's compute segment runs beside its partner's load
// segment: MFMA ping-pong (cdna_hip_programming.md section 5, the 256^2 8-phase template's stagger).
// LDS: NBUF K tiles of BK (64 or 32) as [rows][BK] with a source-side XOR swizzle (rule 21); tile t + NBUF - 1 is
// issued in tile t's first load segment into the buffer tile t - 1 used (last read by group 1 before the barrier
// that opens group 0's load segment of tile t), and tile t + 1 must have landed (vmcnt) by the end of tile t's last
// load segment.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <cmath>
#include <vector>

#include "../include/faithdiff_hip.h"

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// clock stamps (DIAG & 8): per workgroup {memtime, memrealtime} at loop start and end (diagnostic only; nothing
// else reads this buffer)
__device__ unsigned long long g_stamps[65536 * 4];

template <int N>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ROWB bytes per LDS row: 128 (BK 64, 8 chunks of 16 B, chunk ^= (row >> 1) & 7) or 64 (BK 32, chunk ^= (row >> 2) & 3)
template <int ROWB>
__device__ __forceinline__ int swz(int row, int chunk) {
  return ROWB == 128 ? (chunk ^ ((row >> 1) & 7)) : (chunk ^ ((row >> 2) & 3));
}

// GL: where a wave issues its LDS-DMA share of tile t + NBUF - 1: 0 = all in tile t's first load segment, 1 = split
// evenly over the tile's KH load segments, 2 = inside the compute segments, between the MFMAs.  EPI 0: no stores.
template <int BM, int BN, int BK, int NBUF, int GW_M, int PRIO, int GL = 0, int EPI = 1, int DIAG = 0>
__global__ void __launch_bounds__(512) gemm_pp(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                               bf16* __restrict__ C, int M, int N, int K, int group_m) {
  constexpr int ROWB = BK * 2;
  constexpr int CPR = ROWB / 16;                 // 16-B chunks per row
  constexpr int STAGE = (BM + BN) * ROWB;
  static_assert(NBUF * STAGE <= 163840, "LDS");
  constexpr int GM = BM / 2, GW_N = 4 / GW_M;
  constexpr int WM = GM / GW_M, WN = BN / GW_N;
  constexpr int MT = WM / 16, NT = WN / 16;
  static_assert(MT * 16 == WM && NT * 16 == WN, "wave tile");
  constexpr int KH = BK / 32;                    // phases per K tile
  constexpr int RPI = 1024 / ROWB;               // rows per LDS-DMA wave-instruction
  constexpr int NI = (BM + BN) / RPI;            // LDS-DMA instructions per K tile
  constexpr int IHI = (NI + 7) / 8, ILO = NI / 8, NHI = NI % 8 == 0 ? 8 : NI % 8;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NBUF * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w >> 2, wi = w & 3;
  const int wm = wi / GW_N, wn = wi % GW_N;
  const bool hi = w < NHI;                       // this wave issues IHI (else ILO) DMA instructions per tile

  const int tiles_m = M / BM, tiles_n = N / BN;
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
  const int nk = K / BK;

  // this lane's source row pointers (one per DMA instruction it issues)
  const bf16* src[IHI];
#pragma unroll
  for (int i = 0; i < IHI; ++i) {
    const int ins = w + 8 * i;                   // instruction index within the K tile
    const int row = min(ins, NI - 1) * RPI + lane / CPR;
    const int ch = swz<ROWB>(row, lane % CPR);
    src[i] = row < BM ? A + (long long)(m0 + row) * K + ch * 8 : B + (long long)(n0 + row - BM) * K + ch * 8;
  }
  // part p of KP: this wave's instructions i with i % KP == p
  auto stage = [&](int t, int p, int KP) {
    if (DIAG & 1) return;
    unsigned char* s = smem + (t % NBUF) * STAGE;
#pragma unroll
    for (int i = 0; i < IHI; ++i)
      if ((i < ILO || hi) && i % KP == p)
        __builtin_amdgcn_global_load_lds((const void*)(src[i] + (long long)t * BK), LDS_PTR(s + (w + 8 * i) * 1024),
                                         16, 0, 0);
  };
  // all but this wave's youngest `ahead` tiles landed
  auto wait_ahead = [&](int ahead) {
    if (NBUF >= 5 && ahead >= 3) {
      if (hi) vmcnt<3 * IHI>(); else vmcnt<3 * ILO>();
    } else if (NBUF >= 4 && ahead == 2) {
      if (hi) vmcnt<2 * IHI>(); else vmcnt<2 * ILO>();
    } else if (NBUF >= 3 && ahead == 1) {
      if (hi) vmcnt<IHI>(); else vmcnt<ILO>();
    } else {
      vmcnt<0>();
    }
  };

  const int fr = lane & 15, fg = lane >> 4;
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 af[MT], bfr[NT];

  // prologue: tiles 0 .. NBUF-2 in flight, tile 0 landed and visible
#pragma unroll
  for (int t = 0; t < NBUF - 1; ++t)
    if (t < nk) stage(t, 0, 1);
  wait_ahead(min(NBUF - 2, nk - 1));
  __builtin_amdgcn_s_barrier();
  if ((DIAG & 8) && tid == 0 && blockIdx.x < 65536) {
    g_stamps[blockIdx.x * 4 + 0] = __builtin_amdgcn_s_memtime();
    g_stamps[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime();
  }
  if (g == 1) __builtin_amdgcn_s_barrier();      // the stagger: group 1 runs one barrier behind
  if (PRIO && g == 1) __builtin_amdgcn_s_setprio(1);

  for (int t = 0; t < nk; ++t) {
    const unsigned char* sa = smem + (t % NBUF) * STAGE;
    const unsigned char* sb = sa + BM * ROWB;
#pragma unroll
    for (int h = 0; h < KH; ++h) {
      // ---- load segment
      const int ch = h * 4 + fg;
      if (!(DIAG & 2)) {
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int r = g * GM + wm * WM + mi * 16 + fr;
        af[mi] = *(const bf16x8*)(sa + r * ROWB + (swz<ROWB>(r, ch) << 4));
      }
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) {
        const int r = wn * WN + ni * 16 + fr;
        bfr[ni] = *(const bf16x8*)(sb + r * ROWB + (swz<ROWB>(r, ch) << 4));
      }
      } else {
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) asm volatile("" : "+v"(af[mi]));
#pragma unroll
        for (int ni = 0; ni < NT; ++ni) asm volatile("" : "+v"(bfr[ni]));
      }
      const bool more = t + NBUF - 1 < nk;
      if (GL == 0 && h == 0 && more) stage(t + NBUF - 1, 0, 1);
      if (GL == 1 && more) stage(t + NBUF - 1, h, KH);
      if (h == KH - 1 && GL != 2) wait_ahead(min(NBUF - 2, nk - 2 - t));  // tile t+1 landed (this wave's part)
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      // ---- compute segment
      __builtin_amdgcn_s_waitcnt(0xc07f);
      if (DIAG & 4) {
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) asm volatile("" ::"v"(af[mi]));
#pragma unroll
        for (int ni = 0; ni < NT; ++ni) asm volatile("" ::"v"(bfr[ni]));
      } else {
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NT; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
      }
      if (GL == 2) {
        if (more) stage(t + NBUF - 1, h, KH);
        constexpr int NG = (IHI + KH - 1) / KH;
#pragma unroll
        for (int i = 0; i < NG; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, (MT * NT) / (NG + 1), 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read (the LDS-DMA)
        }
        __builtin_amdgcn_sched_group_barrier(0x008, MT * NT, 0);
        if (h == KH - 1) wait_ahead(min(NBUF - 2, nk - 2 - t));
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
    }
  }
  if (g == 0) __builtin_amdgcn_s_barrier();      // re-align the groups
  if (PRIO && g == 1) __builtin_amdgcn_s_setprio(0);
  if ((DIAG & 8) && tid == 0 && blockIdx.x < 65536) {
    g_stamps[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_memtime();
    g_stamps[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_memrealtime();
  }

  // epilogue (probe): straight from the accumulators
  if (EPI == 0) {
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) asm volatile("" ::"v"(acc[mi][ni]));
    return;
  }
#pragma unroll
  for (int mi = 0; mi < MT; ++mi)
#pragma unroll
    for (int ni = 0; ni < NT; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + g * GM + wm * WM + mi * 16 + fg * 4 + j, n = n0 + wn * WN + ni * 16 + fr;
        C[(long long)m * N + n] = (bf16)acc[mi][ni][j];
      }
}

// Loader-wave variant: the two compute groups run the same ping-pong but issue no LDS-DMA; NL extra waves (one per
// SIMD) do all of it, spread evenly over every barrier interval, so the DMA stream never sits on a compute wave's
// critical path.  Interval j (closed by barrier b_j, j = -1 .. 2P-1 for P = 2 nk phases) issues part (j + 1) % 4 of
// stage (j + 1) / 4 + 2 (tile t + 2 goes into the buffer tile t - 1 used, free after b_{4t-1}); at the end of
// interval 4t + 2 each loader waits for stage t + 1 (vmcnt = its share of stage t + 2, all issued by then).
template <int BM, int BN, int GW_M, int NL, int EPI = 0>
__global__ void __launch_bounds__(512 + 64 * NL) gemm_lw(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                        bf16* __restrict__ C, int M, int N, int K, int group_m) {
  constexpr int BK = 64, NBUF = 3, ROWB = 128, CPR = 8;
  constexpr int STAGE = (BM + BN) * ROWB;
  static_assert(NBUF * STAGE <= 163840, "LDS");
  constexpr int GM = BM / 2, GW_N = 4 / GW_M;
  constexpr int WM = GM / GW_M, WN = BN / GW_N;
  constexpr int MT = WM / 16, NT = WN / 16;
  constexpr int RPI = 8;                          // rows per LDS-DMA instruction (8 x 128 B)
  constexpr int NI = (BM + BN) / RPI;             // LDS-DMA instructions per K tile
  static_assert(NI % NL == 0, "even loader shares");
  constexpr int IPL = NI / NL;                    // per loader per tile
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NBUF * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_m = M / BM, tiles_n = N / BN;
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
  const int nk = K / BK, P = 2 * nk;

  if (w >= 8) {  // ---------------- loader wave
    const int l = w - 8;
    const bf16* src[IPL];
#pragma unroll
    for (int k = 0; k < IPL; ++k) {
      const int ins = l + NL * k;
      const int row = ins * RPI + lane / CPR;
      const int ch = swz<ROWB>(row, lane % CPR);
      src[k] = row < BM ? A + (long long)(m0 + row) * K + ch * 8 : B + (long long)(n0 + row - BM) * K + ch * 8;
    }
    auto issue = [&](int t, int part) {  // part of 4: instructions k with k % 4 == part
      unsigned char* s = smem + (t % NBUF) * STAGE;
#pragma unroll
      for (int k = 0; k < IPL; ++k)
        if (k % 4 == part)
          __builtin_amdgcn_global_load_lds((const void*)(src[k] + (long long)t * BK),
                                           LDS_PTR(s + (l + NL * k) * 1024), 16, 0, 0);
    };
    // prologue: stages 0 and 1, stage 0 landed
#pragma unroll
    for (int part = 0; part < 4; ++part) issue(0, part);
    if (nk > 1) {
#pragma unroll
      for (int part = 0; part < 4; ++part) issue(1, part);
      vmcnt<IPL>();
    } else {
      vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    for (int j = -1; j < 2 * P; ++j) {  // 2P + 1 barrier intervals
      const int u = j + 1, t2 = u / 4 + 2, part = u % 4;
      if (t2 < nk) {
        switch (part) {
          case 0: issue(t2, 0); break;
          case 1: issue(t2, 1); break;
          case 2: issue(t2, 2); break;
          default: issue(t2, 3); break;
        }
      }
      if (part == 3 && u / 4 + 1 < nk) {  // end of interval 4t + 2: stage t + 1 landed (t = u / 4)
        if (t2 < nk) vmcnt<IPL>(); else vmcnt<0>();
      }
      __builtin_amdgcn_s_barrier();
    }
    return;
  }

  // ---------------- compute waves: identical ping-pong, no DMA
  const int g = w >> 2, wi = w & 3;
  const int wm = wi / GW_N, wn = wi % GW_N;
  const int fr = lane & 15, fg = lane >> 4;
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 af[MT], bfr[NT];
  __builtin_amdgcn_s_barrier();
  if (g == 1) __builtin_amdgcn_s_barrier();
  for (int t = 0; t < nk; ++t) {
    const unsigned char* sa = smem + (t % NBUF) * STAGE;
    const unsigned char* sb = sa + BM * ROWB;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ch = h * 4 + fg;
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int r = g * GM + wm * WM + mi * 16 + fr;
        af[mi] = *(const bf16x8*)(sa + r * ROWB + (swz<ROWB>(r, ch) << 4));
      }
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) {
        const int r = wn * WN + ni * 16 + fr;
        bfr[ni] = *(const bf16x8*)(sb + r * ROWB + (swz<ROWB>(r, ch) << 4));
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_s_waitcnt(0xc07f);
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NT; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
    }
  }
  if (g == 0) __builtin_amdgcn_s_barrier();
  if (EPI == 0) {
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) asm volatile("" ::"v"(acc[mi][ni]));
    return;
  }
#pragma unroll
  for (int mi = 0; mi < MT; ++mi)
#pragma unroll
    for (int ni = 0; ni < NT; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + g * GM + wm * WM + mi * 16 + fg * 4 + j, n = n0 + wn * WN + ni * 16 + fr;
        C[(long long)m * N + n] = (bf16)acc[mi][ni][j];
      }
}

__global__ void ref_gemm(const bf16* A, const bf16* B, float* C, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += (float)A[(long long)m * K + k] * (float)B[(long long)n * K + k];
  C[(long long)m * N + n] = s;
}

__global__ void fill(bf16* p, long long n, unsigned seed) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = (bf16)(((int)(x & 0xffff) - 32768) / 32768.0f);  // uniform [-1, 1)
  }
}

static int pick_gm(int tiles_m, int tiles_n) {
  const long long per_xcd = ((long long)tiles_m * tiles_n + 7) / 8;
  int gm = 1;
  double bestc = 1e30;
  for (int g = 1; g <= tiles_m; g *= 2) {
    const long long cols = per_xcd < g ? 1 : (per_xcd + g - 1) / g;
    const long long rows = per_xcd < g ? per_xcd : g;
    const double c = rows + (double)std::min<long long>(cols, tiles_n);
    if (c < bestc - 1e-9) {
      bestc = c;
      gm = g;
    }
  }
  return gm;
}

struct Ctx {
  bf16 *A, *B, *C;
  float* ref;
  int (*fd_gemm)(fd_gemm_params*, void*);
  long long (*fd_ws)(const fd_gemm_params*);
  void* ws;
};

static float time_us(const std::function<void()>& f, int reps = 20) {
  for (int i = 0; i < 3; ++i) f();
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> t;
  for (int b = 0; b < 5; ++b) {
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) f();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms * 1e3f / reps);
  }
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  std::sort(t.begin(), t.end());
  return t[2];
}

static double check(Ctx& c, int M, int N, int K) {
  // fp32 GPU dot products into c.ref (2048 x 16384 floats at most)
  if ((size_t)M * N > 2048ull * 16384) return -2;
  std::vector<float> r((size_t)M * N), got_f;
  ref_gemm<<<dim3((N + 255) / 256, M), 256>>>(c.A, c.B, c.ref, M, N, K);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(r.data(), c.ref, (size_t)M * N * 4, hipMemcpyDeviceToHost));
  std::vector<bf16> got((size_t)M * N);
  CHECK(hipMemcpy(got.data(), c.C, (size_t)M * N * 2, hipMemcpyDeviceToHost));
  double num = 0, den = 0;
  for (size_t i = 0; i < r.size(); ++i) {
    const double d = (double)(float)got[i] - r[i];
    num += d * d;
    den += (double)r[i] * r[i];
  }
  return std::sqrt(num / den);
}

template <int BM, int BN, int BK, int NBUF, int GW_M, int PRIO, int GL = 0, int EPI = 1, int DIAG = 0>
static void run_pp(Ctx& c, int M, int N, int K, bool verify) {
  if (M % BM || N % BN || K % BK) return;
  const int tiles_m = M / BM, tiles_n = N / BN;
  const int gm = pick_gm(tiles_m, tiles_n);
  auto f = [&]() {
    hipLaunchKernelGGL((gemm_pp<BM, BN, BK, NBUF, GW_M, PRIO, GL, EPI, DIAG>), dim3(tiles_m * tiles_n), dim3(512), 0, 0, c.A, c.B, c.C,
                       M, N, K, gm);
  };
  CHECK(hipMemset(c.C, 0, (size_t)M * N * 2));
  f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipGetLastError());
  double err = verify && EPI && !DIAG ? check(c, M, N, K) : -1;
  const float us = time_us(f);
  double ghz = 0;
  if (DIAG & 8) {
    const int nt = std::min(tiles_m * tiles_n, 65536);
    std::vector<unsigned long long> st((size_t)nt * 4);
    CHECK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamps), st.size() * 8));
    std::vector<double> cl;
    for (int i = 0; i < nt; ++i) {
      const double dt = (double)(st[i * 4 + 2] - st[i * 4]), dr = (double)(st[i * 4 + 3] - st[i * 4 + 1]);
      if (dr > 0) cl.push_back(dt / dr * 0.1);  // memrealtime ticks at 100 MHz
    }
    std::sort(cl.begin(), cl.end());
    ghz = cl.empty() ? 0 : cl[cl.size() / 2];
  }
  printf("  pp %3dx%-3d BK=%d NBUF=%d GW_M=%d PRIO=%d GL=%d EPI=%d DIAG=%d tiles=%-5d %9.2f us %7.1f TF/s  rel=%.2e"
         "  clock %.2f GHz\n", BM, BN, BK, NBUF, GW_M, PRIO, GL, EPI, DIAG, tiles_m * tiles_n, us,
         2.0 * M * N * K / us / 1e6, err, ghz);
  fflush(stdout);
}

template <int BM, int BN, int GW_M, int NL, int EPI>
static void run_lw(Ctx& c, int M, int N, int K, bool verify) {
  if (M % BM || N % BN || K % 64) return;
  const int tiles_m = M / BM, tiles_n = N / BN;
  const int gm = pick_gm(tiles_m, tiles_n);
  auto f = [&]() {
    hipLaunchKernelGGL((gemm_lw<BM, BN, GW_M, NL, EPI>), dim3(tiles_m * tiles_n), dim3(512 + 64 * NL), 0, 0, c.A, c.B,
                       c.C, M, N, K, gm);
  };
  CHECK(hipMemset(c.C, 0, (size_t)M * N * 2));
  f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipGetLastError());
  double err = verify && EPI ? check(c, M, N, K) : -1;
  const float us = time_us(f);
  printf("  lw %3dx%-3d GW_M=%d NL=%d EPI=%d tiles=%-5d %9.2f us %7.1f TF/s  rel=%.2e\n", BM, BN, GW_M, NL, EPI,
         tiles_m * tiles_n, us, 2.0 * M * N * K / us / 1e6, err);
  fflush(stdout);
}

static void run_lib(Ctx& c, int M, int N, int K, bool verify) {
  fd_gemm_params p = {};
  p.A = c.A;
  p.B = c.B;
  p.C = c.C;
  p.lda = K;
  p.ldb = K;
  p.ldc = N;
  p.M = M;
  p.N = N;
  p.K = K;
  p.batch = 1;
  p.alpha = 1.f;
  p.act = FD_ACT_NONE;
  p.dtype = FD_BF16;
  p.out_dtype = FD_BF16;
  p.rows_per_group = 1;
  p.ws = c.ws;
  p.ws_bytes = 1ll << 28;
  if (c.fd_ws(&p) > p.ws_bytes) {
    printf("  lib: workspace too small\n");
    return;
  }
  auto f = [&]() { c.fd_gemm(&p, nullptr); };
  CHECK(hipMemset(c.C, 0, (size_t)M * N * 2));
  const int rc = c.fd_gemm(&p, nullptr);
  CHECK(hipDeviceSynchronize());
  double err = verify ? check(c, M, N, K) : -1;
  const float us = time_us(f);
  printf("  lib fd_gemm (rc %d)                         %9.2f us %7.1f TF/s  rel=%.2e\n", rc, us,
         2.0 * M * N * K / us / 1e6, err);
  fflush(stdout);
}

int main(int argc, char** argv) {
  Ctx c;
  const size_t maxA = 8192ull * 8192, maxB = 16384ull * 8192, maxC = 8192ull * 16384;
  CHECK(hipMalloc(&c.A, maxA * 2));
  CHECK(hipMalloc(&c.B, maxB * 2));
  CHECK(hipMalloc(&c.C, maxC * 2));
  CHECK(hipMalloc(&c.ref, 2048ull * 16384 * 4));
  CHECK(hipMalloc(&c.ws, 1ull << 28));
  CHECK(hipMemset(c.ws, 0, 1ull << 28));
  fill<<<1024, 256>>>(c.A, maxA, 1u);
  fill<<<1024, 256>>>(c.B, maxB, 2u);
  CHECK(hipDeviceSynchronize());
  void* h = dlopen(argc > 1 ? argv[1] : "faithdiff-dev_amd/fdhip/libfaithdiff_hip.so", RTLD_NOW);
  if (!h) {
    fprintf(stderr, "dlopen: %s\n", dlerror());
    return 1;
  }
  c.fd_gemm = (int (*)(fd_gemm_params*, void*))dlsym(h, "fd_gemm");
  c.fd_ws = (long long (*)(const fd_gemm_params*))dlsym(h, "fd_gemm_ws_bytes");

  struct S { int M, N, K; bool verify; };
  const char* sel = argc > 2 ? argv[2] : "ablate";
  if (!strcmp(sel, "pmc")) {  // one shape, the full kernel and its three single-path variants (rocprofv3 --pmc runs)
    const S s{2048, 10240, 1280, false};
    run_pp<256, 160, 64, 3, 2, 0, 0, 0, 0>(c, s.M, s.N, s.K, false);
    run_pp<256, 160, 64, 3, 2, 0, 0, 0, 3>(c, s.M, s.N, s.K, false);
    run_pp<256, 160, 64, 3, 2, 0, 0, 0, 6>(c, s.M, s.N, s.K, false);
    run_pp<256, 160, 64, 3, 2, 0, 0, 0, 5>(c, s.M, s.N, s.K, false);
    run_lw<256, 160, 2, 4, 0>(c, s.M, s.N, s.K, false);
    return 0;
  }
  const S shapes[] = {{2048, 10240, 1280, true}, {4096, 4096, 4096, false}};
  for (const S& s : shapes) {
    printf("M=%d N=%d K=%d\n", s.M, s.N, s.K);
    // full, no glds, no ds_read, no MFMA, MFMA only, glds only -- each with the clock stamps (DIAG & 8)
    run_pp<256, 160, 64, 3, 2, 0, 0, 0, 8>(c, s.M, s.N, s.K, false);
    run_pp<256, 160, 64, 3, 2, 0, 0, 0, 9>(c, s.M, s.N, s.K, false);
    run_pp<256, 160, 64, 3, 2, 0, 0, 0, 10>(c, s.M, s.N, s.K, false);
    run_pp<256, 160, 64, 3, 2, 0, 0, 0, 12>(c, s.M, s.N, s.K, false);
    run_pp<256, 160, 64, 3, 2, 0, 0, 0, 11>(c, s.M, s.N, s.K, false);
    run_pp<256, 160, 64, 3, 2, 0, 0, 0, 14>(c, s.M, s.N, s.K, false);
    run_pp<256, 256, 64, 2, 2, 0, 0, 0, 8>(c, s.M, s.N, s.K, false);
    run_pp<256, 256, 64, 2, 2, 0, 0, 0, 11>(c, s.M, s.N, s.K, false);
  }
  return 0;
}
