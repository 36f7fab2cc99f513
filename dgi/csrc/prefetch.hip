// dgi/csrc/prefetch.hip — warm the memory-side cache (MALL / Infinity Cache, 256 MB)
// with the rows a later kernel will stream.
//
// A batch-1 decode layer is a chain of HBM-bound weight streams with one latency-bound
// kernel in it: paged decode attention reads ~2 MB of KV on a handful of CUs for ~10 us
// while HBM sits idle (profiles/r5_decode/decode8b_b1_step_breakdown_r5.md).  Forked onto a
// side stream beside it, this kernel reads the next projection's weight rows so that the
// projection finds them in the MALL instead of HBM.  It is a plain read: every 16-byte
// chunk of the listed rows is loaded once (normal cached loads, so the lines allocate),
// folded into a per-lane xor and dropped; the store behind an impossible compare keeps
// the loads alive.  No other memory is written.
#include "common.h"

using namespace dgi;

namespace {

constexpr int kThreads = 256;
constexpr int kUnroll = 8;

// rows == nullptr: rows 0..nrows-1.  Chunk c of the (virtual) row list is 16 bytes at
// row rows[c / row_chunks], offset c % row_chunks; each thread issues kUnroll loads
// before it consumes any, so a wave keeps 8 x 1 KB in flight.
__global__ __launch_bounds__(kThreads) void mall_prefetch_kernel(const u32x4* __restrict__ base,
                                                                 const int* __restrict__ rows, int nrows,
                                                                 int row_chunks, unsigned magic,
                                                                 unsigned* __restrict__ sink) {
  const long total = (long)nrows * row_chunks;
  const long stride = (long)gridDim.x * kThreads;
  unsigned acc = 0u;
  for (long c0 = (long)blockIdx.x * kThreads + threadIdx.x; c0 < total; c0 += stride * kUnroll) {
    u32x4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const long c = c0 + u * stride;
      v[u] = u32x4{0u, 0u, 0u, 0u};
      if (c < total) {
        const int r = (int)(c / row_chunks);
        const long row = rows ? (long)rows[r] : (long)r;
        v[u] = base[row * row_chunks + (c - (long)r * row_chunks)];
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (acc == magic) sink[threadIdx.x] = acc;  // practically never; keeps the loads
}

}  // namespace

// Warm `nrows` rows of `row_bytes` each (row ids from `rows`, or 0..nrows-1) of the
// matrix at `base` with `blocks` workgroups.  sink: >= 256 u32 of scratch.
extern "C" int dgi_mall_prefetch(const void* base, const int* rows, int nrows, int row_bytes, int blocks,
                                 void* sink, hipStream_t s) {
  if (nrows <= 0) return 0;
  if (row_bytes <= 0 || (row_bytes & 15) || blocks <= 0) return 1;
  if (((uintptr_t)base & 15) != 0) return 1;
  mall_prefetch_kernel<<<dim3(blocks), kThreads, 0, s>>>(reinterpret_cast<const u32x4*>(base), rows, nrows,
                                                         row_bytes >> 4, 0x7fc3a5e1u,
                                                         reinterpret_cast<unsigned*>(sink));
  return (int)hipGetLastError();
}
