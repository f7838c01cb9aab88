// Operand-intake microbenchmark for gfx950 (MI355X): how many bytes per second can one CU pull from L2 into
// LDS (or into VGPRs) with the access pattern of this repo's GEMM tiles?  Standalone (not part of the
// product library); built by probes/Makefile, run on the GPU box:  ./probes/intake_probe > out.txt
//
// Each workgroup owns one output tile (tm, tn) of an M x N x K bf16 GEMM, with the tile walk of gemm.hip
// (bijective XCD remap + GROUP_M = 4), and streams exactly the operand bytes that tile needs -- BM rows of A
// and BN rows of W, K-contiguous, one PIECE-byte run per row per K step -- and nothing else: no LDS reads, no
// MFMA.  Variants:
//   MODE 0  global_load_lds_dwordx4 into an NSLOT ring (lane-linear 1 KiB per wave-instruction)
//   MODE 1  global_load_dwordx4 into VGPRs (DEPTH register stages), consumed by one XOR per load
//   NWG/NL  waves per workgroup / of which issue loads (the rest only join the barriers)
//   DEPTH   K steps in flight per wave (counted s_waitcnt vmcnt)
//   BAR     one raw s_barrier per K step (what a consumer needs before it may read the slot)
//   PIECE   contiguous bytes per row per K step: 128 = a 64-deep bf16 K step (every kernel in the repo),
//           256 = 128-deep
// Reported: us per launch (median of 7 timed batches of 20 launches), and the intake rate per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ void tile_of(int bid, int nwg, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int pid = xcd_remap(bid, nwg);
  constexpr int GROUP_M = 4;
  const int group = pid / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int in_group = pid - group * (GROUP_M * tiles_n);
  tm = first_m + in_group % gsz;
  tn = in_group / gsz;
}

template <int N>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN, int NWG, int NL, int DEPTH, int BAR, int PIECE>
__global__ void __launch_bounds__(NWG * 64) probe_glds(const unsigned char* A, const unsigned char* W, long long lda,
                                                      long long ldw, int ksteps, int tiles_m, int tiles_n) {
  constexpr int RPI = 1024 / PIECE;             // rows per wave-instruction
  constexpr int INSTR = (BM + BN) / RPI;        // wave-instructions per K step (whole workgroup)
  static_assert(INSTR % NL == 0 && NL <= NWG, "instructions split evenly over the loader waves");
  constexpr int IPW = INSTR / NL;
  constexpr int SLOT = (BM + BN) * PIECE;
  // the slot being read + DEPTH-1 in flight; nothing reads the ring here, so a ring with fewer slots than that
  // (256 x 256 tiles) only overwrites bytes no one looks at
  constexpr int NSLOT = DEPTH * SLOT <= 160 * 1024 ? DEPTH : (160 * 1024) / SLOT;
  static_assert(NSLOT >= 1, "LDS");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NSLOT * SLOT];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int tm, tn;
  tile_of(blockIdx.x, gridDim.x, tiles_m, tiles_n, tm, tn);
  const unsigned char* src[IPW];
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int row = (i * NL + wave) * RPI + lane / (PIECE / 16);
    const int part = lane % (PIECE / 16);
    const int rr = min(row, BM + BN - 1);
    src[i] = rr < BM ? A + (long long)(tm * BM + rr) * lda + part * 16
                     : W + (long long)(tn * BN + rr - BM) * ldw + part * 16;
  }
  const bool loader = wave < NL;
  auto stage = [&](int kt) {
    if (!loader) return;
    unsigned char* s = smem + (kt % NSLOT) * SLOT;
#pragma unroll
    for (int i = 0; i < IPW; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src[i] + (long long)kt * PIECE),
                                       LDS_PTR(s + (i * NL + wave) * 1024), 16, 0, 0);
  };
#pragma unroll
  for (int s = 0; s < DEPTH - 1; ++s)
    if (s < ksteps) stage(s);
  for (int kt = 0; kt < ksteps; ++kt) {
    if (kt + DEPTH - 1 < ksteps) {
      stage(kt + DEPTH - 1);
      vmcnt<(DEPTH - 1) * IPW>();
    } else {
      vmcnt<0>();
    }
    if (BAR) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  vmcnt<0>();
}

template <int BM, int BN, int NWG, int NL, int DEPTH, int BAR, int PIECE>
__global__ void __launch_bounds__(NWG * 64) probe_vgpr(const unsigned char* A, const unsigned char* W, long long lda,
                                                      long long ldw, int ksteps, int tiles_m, int tiles_n,
                                                      unsigned* sink) {
  constexpr int RPI = 1024 / PIECE;
  constexpr int INSTR = (BM + BN) / RPI;
  static_assert(INSTR % NL == 0 && NL <= NWG, "instructions split evenly over the loader waves");
  constexpr int IPW = INSTR / NL;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int tm, tn;
  tile_of(blockIdx.x, gridDim.x, tiles_m, tiles_n, tm, tn);
  const unsigned char* src[IPW];
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int row = (i * NL + wave) * RPI + lane / (PIECE / 16);
    const int part = lane % (PIECE / 16);
    const int rr = min(row, BM + BN - 1);
    src[i] = rr < BM ? A + (long long)(tm * BM + rr) * lda + part * 16
                     : W + (long long)(tn * BN + rr - BM) * ldw + part * 16;
  }
  u32x4 r[DEPTH][IPW];
  unsigned acc = 0;
  if (wave >= NL) {  // idle waves: only the barriers
    if (BAR)
      for (int kt = 0; kt < ksteps; ++kt) __builtin_amdgcn_s_barrier();
    return;
  }
#pragma unroll
  for (int s = 0; s < DEPTH - 1; ++s)
#pragma unroll
    for (int i = 0; i < IPW; ++i) r[s][i] = *(const u32x4*)(src[i] + (long long)s * PIECE);
  for (int k0 = 0; k0 < ksteps; k0 += DEPTH) {
#pragma unroll
    for (int s = 0; s < DEPTH; ++s) {
      const int kt = k0 + s;
      if (kt < ksteps) {
        const int kn = kt + DEPTH - 1;
#pragma unroll
        for (int i = 0; i < IPW; ++i)
          r[(s + DEPTH - 1) % DEPTH][i] = *(const u32x4*)(src[i] + (long long)min(kn, ksteps - 1) * PIECE);
#pragma unroll
        for (int i = 0; i < IPW; ++i) acc ^= r[s][i][0] ^ r[s][i][3];
        if (BAR) __builtin_amdgcn_s_barrier();
      }
    }
  }
  if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;  // keeps every load live; practically never stored
}

struct Case {
  const char* name;
  int M, N, K;
};

static unsigned char *gA, *gW;
static unsigned* gSink;

template <int MODE, int BM, int BN, int NWG, int NL, int DEPTH, int BAR, int PIECE>
static void run(const Case& c) {
  const int tiles_m = c.M / BM, tiles_n = c.N / BN, tiles = tiles_m * tiles_n;
  const long long lda = (long long)c.K * 2, ldw = (long long)c.K * 2;
  const int ksteps = (int)(lda / PIECE);
  auto launch = [&]() {
    if (MODE == 0)
      hipLaunchKernelGGL((probe_glds<BM, BN, NWG, NL, DEPTH, BAR, PIECE>), dim3(tiles), dim3(NWG * 64), 0, 0, gA, gW, lda,
                         ldw, ksteps, tiles_m, tiles_n);
    else
      hipLaunchKernelGGL((probe_vgpr<BM, BN, NWG, NL, DEPTH, BAR, PIECE>), dim3(tiles), dim3(NWG * 64), 0, 0, gA, gW, lda,
                         ldw, ksteps, tiles_m, tiles_n, gSink);
  };
  for (int i = 0; i < 5; ++i) launch();
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> t;
  for (int b = 0; b < 7; ++b) {
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < 20; ++i) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms * 1e3f / 20);
  }
  CHECK(hipGetLastError());
  std::sort(t.begin(), t.end());
  const double us = t[3];
  const double bytes_wg = (double)(BM + BN) * c.K * 2;
  const double cus = std::min(tiles, 256);
  printf("%-22s %-5s %3dx%-3d NWG=%-2d NL=%-2d DEPTH=%d BAR=%d PIECE=%-4d tiles=%-4d  %8.2f us  %6.1f GB/s per CU  %6.2f TB/s chip\n",
         c.name, MODE == 0 ? "glds" : "vgpr", BM, BN, NWG, NL, DEPTH, BAR, PIECE, tiles, us,
         bytes_wg * tiles / cus / (us * 1e-6) / 1e9, bytes_wg * tiles / (us * 1e-6) / 1e12);
  fflush(stdout);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

// 64 x 160 (28 wave-instructions of 1 KiB per 64-deep K step): the gemm.hip tile of the M = 2048 projections
static void sweep_64x160(const Case& c) {
  run<0, 64, 160, 4, 4, 2, 1, 128>(c);
  run<0, 64, 160, 4, 4, 3, 1, 128>(c);
  run<0, 64, 160, 4, 4, 4, 1, 128>(c);
  run<0, 64, 160, 8, 4, 4, 1, 128>(c);  // the product kernel's shape: 8 waves, waves 0-3 load, 4-deep ring
  run<0, 64, 160, 8, 7, 3, 1, 128>(c);
  run<0, 64, 160, 8, 7, 4, 1, 128>(c);
  run<0, 64, 160, 8, 7, 4, 0, 128>(c);
  run<0, 64, 160, 16, 14, 4, 1, 128>(c);
  run<0, 64, 160, 8, 4, 2, 1, 256>(c);
  run<0, 64, 160, 8, 8, 3, 1, 256>(c);
  run<0, 64, 160, 16, 14, 3, 1, 256>(c);
  run<1, 64, 160, 4, 4, 2, 1, 128>(c);
  run<1, 64, 160, 8, 7, 2, 1, 128>(c);
  run<1, 64, 160, 8, 7, 3, 0, 128>(c);
  run<1, 64, 160, 16, 14, 2, 0, 128>(c);
  run<1, 64, 160, 16, 14, 3, 0, 128>(c);
}

int main() {
  // operand buffers big enough for every case (A: up to 32768 x 1280, W: up to 10240 x 5120), random bytes
  const size_t nA = 96ull << 20, nW = 112ull << 20;
  CHECK(hipMalloc(&gA, nA));
  CHECK(hipMalloc(&gW, nW));
  CHECK(hipMalloc(&gSink, 4096));
  {
    std::vector<unsigned> h(nW / 4);
    unsigned s = 12345;
    for (auto& v : h) v = (s = s * 1664525u + 1013904223u) & 0x3f7f3f7fu;
    CHECK(hipMemcpy(gA, h.data(), nA, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(gW, h.data(), nW, hipMemcpyHostToDevice));
  }
  const Case c1{"M2048 N1280 K1280", 2048, 1280, 1280};  // the 32^2 level projections (136 launches / step)
  const Case c2{"M2048 N1280 K5120", 2048, 1280, 5120};  // the 32^2 ff out
  const Case c3{"M2048 N1280 K16384", 2048, 1280, 16384};  // steady state (long K)
  printf("# per-CU operand intake, GEMM tile access pattern (no LDS reads, no MFMA)\n");
  sweep_64x160(c1);
  sweep_64x160(c2);
  sweep_64x160(c3);
  run<0, 128, 128, 8, 8, 3, 1, 128>(c1);
  run<0, 128, 128, 8, 8, 4, 1, 128>(c1);
  run<0, 128, 128, 16, 16, 4, 1, 128>(c1);
  run<0, 128, 128, 8, 8, 3, 1, 128>(c3);
  run<0, 256, 128, 8, 8, 3, 1, 128>(c3);
  run<0, 256, 256, 8, 8, 3, 1, 128>(c3);
  run<0, 256, 256, 8, 8, 4, 1, 128>(c3);
  run<0, 256, 256, 16, 16, 4, 1, 128>(c3);
  // a launch with no K steps: the fixed cost of a 256-workgroup launch
  run<0, 64, 160, 8, 4, 2, 1, 128>(Case{"K=0 (launch floor)", 2048, 1280, 0});
  return 0;
}
