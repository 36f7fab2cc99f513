// scripts/mall_probe.hip — does a weight read that the previous kernel already
// streamed hit MI355X's 256 MB MALL (Infinity Cache)?  Standalone probe for the
// decode-step prefetch idea (read the next projection's weights while the
// bandwidth-idle attention kernel runs).  Built by scripts/mall_probe.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void read_kernel(const u32x4* __restrict__ p, size_t n, unsigned* sink) {
  unsigned acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u32x4 v = NT ? __builtin_nontemporal_load(p + i) : p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;  // practically never; keeps the loads alive
}

extern "C" int mall_read(const void* p, size_t bytes, void* sink, int nt, int blocks, hipStream_t s) {
  const size_t n = bytes / 16;
  if (nt)
    read_kernel<true><<<blocks, 256, 0, s>>>((const u32x4*)p, n, (unsigned*)sink);
  else
    read_kernel<false><<<blocks, 256, 0, s>>>((const u32x4*)p, n, (unsigned*)sink);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
