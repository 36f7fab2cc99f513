// dgi/csrc/kv_ops.hip — block-level KV movement.
//
// The block pool is one tensor per engine: [L, 2, num_blocks, n_kv, bs, hd]
// bf16, so one block id names the page of every local layer.  These kernels
// move whole pages:
//   * gather  : pages of `ids` -> contiguous [L, 2, n, page] buffer (KV
//               migration send buffer / CPU-tier spill staging),
//   * scatter : contiguous buffer -> pages of `ids` (migration receive /
//               CPU-tier restore),
//   * copy    : page src[i] -> page dst[i] (radix-cache copy-on-write and
//               speculative-decoding KV compaction).
// The reference does these moves with per-block torch copies / pickles
// (worker/distributed/kv_cache.py:447-475, 522-542; grpc_server.py:196-219).
#include "common.h"

using namespace dgi;

namespace {

// page = n_kv * bs * hd elements; moved as 16-byte chunks.
// BM (block-major): buf is [n, LK, page] — every page of one block id (all layers, K and V)
// contiguous, the host KV tier's slot layout, so a run of consecutive host slots is ONE DMA
// and no permute pass is needed; otherwise buf is [LK, n, page] (the migration layout).
template <bool BM>
__global__ __launch_bounds__(256) void kv_gather_kernel(const u32x4* __restrict__ cache,
                                                        const int* __restrict__ ids, int n,
                                                        int num_blocks, int page_chunks, int LK,
                                                        u32x4* __restrict__ buf) {
  const long total = (long)LK * n * page_chunks;
  for (long c = (long)blockIdx.x * 256 + threadIdx.x; c < total; c += (long)gridDim.x * 256) {
    const int within = (int)(c % page_chunks);
    const long pg = c / page_chunks;
    const int i = BM ? (int)(pg / LK) : (int)(pg % n);
    const int lk = BM ? (int)(pg % LK) : (int)(pg / n);
    buf[c] = cache[((long)lk * num_blocks + ids[i]) * page_chunks + within];
  }
}

template <bool BM>
__global__ __launch_bounds__(256) void kv_scatter_kernel(u32x4* __restrict__ cache,
                                                         const int* __restrict__ ids, int n,
                                                         int num_blocks, int page_chunks, int LK,
                                                         const u32x4* __restrict__ buf) {
  const long total = (long)LK * n * page_chunks;
  for (long c = (long)blockIdx.x * 256 + threadIdx.x; c < total; c += (long)gridDim.x * 256) {
    const int within = (int)(c % page_chunks);
    const long pg = c / page_chunks;
    const int i = BM ? (int)(pg / LK) : (int)(pg % n);
    const int lk = BM ? (int)(pg % LK) : (int)(pg / n);
    cache[((long)lk * num_blocks + ids[i]) * page_chunks + within] = buf[c];
  }
}

__global__ __launch_bounds__(256) void kv_copy_kernel(u32x4* __restrict__ cache,
                                                      const int* __restrict__ src,
                                                      const int* __restrict__ dst, int n,
                                                      int num_blocks, int page_chunks, int LK) {
  const long total = (long)LK * n * page_chunks;
  for (long c = (long)blockIdx.x * 256 + threadIdx.x; c < total; c += (long)gridDim.x * 256) {
    const int within = (int)(c % page_chunks);
    const long pg = c / page_chunks;
    const int i = (int)(pg % n);
    const int lk = (int)(pg / n);
    cache[((long)lk * num_blocks + dst[i]) * page_chunks + within] =
        cache[((long)lk * num_blocks + src[i]) * page_chunks + within];
  }
}

// Token-slot moves (EAGLE KV compaction: accepted tree nodes -> consecutive positions):
// slot s = block * bs + offset; a slot of one (layer, k/v) is n_kv rows of hd elements at
// stride bs * hd.  Gather every source slot into buf [n, LK, n_kv, hd] first, then scatter:
// the moves of one sequence chain (a node's source slot can be another move's destination),
// so all reads must land before any write (what the torch advanced-index version did, in 36
// launches per verify step).
__global__ __launch_bounds__(256) void kv_slot_gather_kernel(const u32x4* __restrict__ cache,
                                                             const int* __restrict__ src, int n, int LK,
                                                             int num_blocks, int nkv, int bs, int hdc,
                                                             u32x4* __restrict__ buf) {
  const long total = (long)n * LK * nkv * hdc;
  for (long c = (long)blockIdx.x * 256 + threadIdx.x; c < total; c += (long)gridDim.x * 256) {
    const int d = (int)(c % hdc);
    long r = c / hdc;
    const int h = (int)(r % nkv);
    r /= nkv;
    const int lk = (int)(r % LK);
    const int i = (int)(r / LK);
    const int s = src[i];
    buf[c] = cache[(((long)lk * num_blocks + s / bs) * nkv + h) * bs * hdc + (long)(s % bs) * hdc + d];
  }
}

__global__ __launch_bounds__(256) void kv_slot_scatter_kernel(u32x4* __restrict__ cache,
                                                              const int* __restrict__ dst, int n, int LK,
                                                              int num_blocks, int nkv, int bs, int hdc,
                                                              const u32x4* __restrict__ buf) {
  const long total = (long)n * LK * nkv * hdc;
  for (long c = (long)blockIdx.x * 256 + threadIdx.x; c < total; c += (long)gridDim.x * 256) {
    const int d = (int)(c % hdc);
    long r = c / hdc;
    const int h = (int)(r % nkv);
    r /= nkv;
    const int lk = (int)(r % LK);
    const int i = (int)(r / LK);
    const int s = dst[i];
    cache[(((long)lk * num_blocks + s / bs) * nkv + h) * bs * hdc + (long)(s % bs) * hdc + d] = buf[c];
  }
}

int grid_for(long total) {
  long b = (total + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

}  // namespace

// LK = L*2 (layer x {k,v}); page_elems = n_kv*bs*hd; block_major: buf [n, LK, page] instead of [LK, n, page]
extern "C" int dgi_kv_gather(const void* cache, const int* ids, int n, int LK, int num_blocks,
                             int page_elems, void* buf, int block_major, hipStream_t s) {
  if (n == 0) return 0;
  if (page_elems % 8) return -2;
  const int pc = page_elems / 8;
  const int g = grid_for((long)LK * n * pc);
  if (block_major)
    kv_gather_kernel<true><<<g, 256, 0, s>>>((const u32x4*)cache, ids, n, num_blocks, pc, LK, (u32x4*)buf);
  else
    kv_gather_kernel<false><<<g, 256, 0, s>>>((const u32x4*)cache, ids, n, num_blocks, pc, LK, (u32x4*)buf);
  DGI_CHECK_LAUNCH();
  return 0;
}

extern "C" int dgi_kv_scatter(void* cache, const int* ids, int n, int LK, int num_blocks,
                              int page_elems, const void* buf, int block_major, hipStream_t s) {
  if (n == 0) return 0;
  if (page_elems % 8) return -2;
  const int pc = page_elems / 8;
  const int g = grid_for((long)LK * n * pc);
  if (block_major)
    kv_scatter_kernel<true><<<g, 256, 0, s>>>((u32x4*)cache, ids, n, num_blocks, pc, LK, (const u32x4*)buf);
  else
    kv_scatter_kernel<false><<<g, 256, 0, s>>>((u32x4*)cache, ids, n, num_blocks, pc, LK, (const u32x4*)buf);
  DGI_CHECK_LAUNCH();
  return 0;
}

extern "C" int dgi_kv_copy(void* cache, const int* src, const int* dst, int n, int LK,
                           int num_blocks, int page_elems, hipStream_t s) {
  if (n == 0) return 0;
  if (page_elems % 8) return -2;
  const int pc = page_elems / 8;
  kv_copy_kernel<<<grid_for((long)LK * n * pc), 256, 0, s>>>((u32x4*)cache, src, dst, n,
                                                             num_blocks, pc, LK);
  DGI_CHECK_LAUNCH();
  return 0;
}

// cache [L, 2, NB, nkv, bs, hd] bf16; src / dst: token slots; buf: n * LK * nkv * hd elements
extern "C" int dgi_kv_slot_copy(void* cache, const int* src, const int* dst, int n, int LK, int num_blocks,
                                int nkv, int bs, int hd, void* buf, hipStream_t s) {
  if (n == 0) return 0;
  if (hd % 8) return -2;
  const int hdc = hd / 8;
  const long total = (long)n * LK * nkv * hdc;
  kv_slot_gather_kernel<<<grid_for(total), 256, 0, s>>>((const u32x4*)cache, src, n, LK, num_blocks, nkv, bs, hdc,
                                                        (u32x4*)buf);
  DGI_CHECK_LAUNCH();
  kv_slot_scatter_kernel<<<grid_for(total), 256, 0, s>>>((u32x4*)cache, dst, n, LK, num_blocks, nkv, bs, hdc,
                                                         (const u32x4*)buf);
  DGI_CHECK_LAUNCH();
  return 0;
}
