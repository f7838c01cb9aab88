// Shader-clock sampler (is a kernel slower in context because the chip clocks down?).  One wave
// on one CU, launched on a side stream beside the measured work: every `interval` ticks of the 100 MHz constant
// counter (s_memrealtime) lane 0 stores (realtime, shader cycles from s_memtime) as one 16-B vector store.  It stops
// after n samples or once *stop != 0 (set by a kernel queued behind the measured work), whichever comes first, so
// every launch drains.  Not part of libfaithdiff_hip.
#include <hip/hip_runtime.h>

typedef unsigned long long u64;
typedef __attribute__((ext_vector_type(2))) u64 u64x2;

__global__ void __launch_bounds__(64) clk_kernel(u64x2* __restrict__ out, int* __restrict__ count, int n, u64 interval,
                                                 const int* __restrict__ stop) {
  if (threadIdx.x != 0) return;
  const u64 r0 = __builtin_readsteadycounter();
  int i = 0;
  for (; i < n; ++i) {
    const u64 target = r0 + (u64)i * interval;
    u64 r;
    do {
      r = __builtin_readsteadycounter();
    } while (r < target);
    const u64 c = __builtin_readcyclecounter();
    out[i] = u64x2{r, c};
    if (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
      ++i;
      break;
    }
  }
  *count = i;
}

extern "C" int clk_launch(void* out, void* count, int n, unsigned long long interval, const void* stop, void* stream) {
  if (!out || !count || !stop || n <= 0 || interval == 0) return -1;
  hipLaunchKernelGGL(clk_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (u64x2*)out, (int*)count, n,
                     (u64)interval, (const int*)stop);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
