// dgi/csrc/rope_cache.hip — fused RoPE(q,k) + paged KV-cache write.
//
// The reference relies on HF rotary embeddings and copies whole KV pages
// in Python (worker/distributed/kv_cache.py:133-136, 460-461).  Here one
// kernel reads the fused QKV GEMM output once:
//   * rotates q in place (NeoX/Llama "rotate_half" pairing, dims i, i+hd/2),
//   * rotates k and scatters k and v into the paged cache at slot_mapping[t].
// Cache layout per layer: [num_blocks, n_kv, block_size, head_dim] so one
// (block, kv-head) page is a contiguous block_size*head_dim run that the
// attention kernels stream with 16-byte loads.
// Positions are arbitrary per token (chunked prefill, prefix reuse and
// EAGLE tree verification all pass non-contiguous positions).
#include "common.h"

using namespace dgi;

__global__ __launch_bounds__(256) void rope_cache_kernel(
    uint16_t* __restrict__ qkv, int qkv_stride, const int* __restrict__ positions,
    const float* __restrict__ cos_sin, int nh, int nkv, int hd,
    const int* __restrict__ slot_mapping, uint16_t* __restrict__ k_cache,
    uint16_t* __restrict__ v_cache, int block_size, int rotate_v_only_k) {
  const int t = blockIdx.x;
  const int pos = positions[t];
  const int half = hd >> 1;
  const int rchunks = half >> 3;  // 8-pair chunks per head
  const int vchunks = hd >> 3;
  uint16_t* row = qkv + (size_t)t * qkv_stride;
  const float* cs = cos_sin + (size_t)pos * hd;
  const int slot = slot_mapping ? slot_mapping[t] : -1;
  const int blk = slot >= 0 ? slot / block_size : 0;
  const int off = slot >= 0 ? slot - blk * block_size : 0;

  const int n_rot = (nh + nkv) * rchunks;
  const int n_v = nkv * vchunks;
  for (int it = threadIdx.x; it < n_rot + n_v; it += blockDim.x) {
    if (it < n_rot) {
      const int head = it / rchunks;
      const int c = it - head * rchunks;
      uint16_t* hp = row + head * hd;  // q heads then k heads are contiguous
      u32x4* p0 = reinterpret_cast<u32x4*>(hp + c * 8);
      u32x4* p1 = reinterpret_cast<u32x4*>(hp + half + c * 8);
      float a[8], b[8], oa[8], ob[8];
      unpack8(*p0, a);
      unpack8(*p1, b);
      const float4* cp = reinterpret_cast<const float4*>(cs + c * 8);
      const float4* sp = reinterpret_cast<const float4*>(cs + half + c * 8);
      float cv[8], sv[8];
      *reinterpret_cast<float4*>(cv) = cp[0];
      *reinterpret_cast<float4*>(cv + 4) = cp[1];
      *reinterpret_cast<float4*>(sv) = sp[0];
      *reinterpret_cast<float4*>(sv + 4) = sp[1];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        oa[j] = a[j] * cv[j] - b[j] * sv[j];
        ob[j] = b[j] * cv[j] + a[j] * sv[j];
      }
      const u32x4 ra = pack8(oa), rb = pack8(ob);
      if (head < nh) {
        *p0 = ra;
        *p1 = rb;
      } else {
        const int kh = head - nh;
        if (!rotate_v_only_k) { *p0 = ra; *p1 = rb; }
        if (slot >= 0) {
          uint16_t* dst = k_cache + (((size_t)blk * nkv + kh) * block_size + off) * hd;
          *reinterpret_cast<u32x4*>(dst + c * 8) = ra;
          *reinterpret_cast<u32x4*>(dst + half + c * 8) = rb;
        }
      }
    } else if (slot >= 0) {
      const int j = it - n_rot;
      const int vh = j / vchunks;
      const int c = j - vh * vchunks;
      const u32x4 v = *reinterpret_cast<const u32x4*>(row + (nh + nkv + vh) * hd + c * 8);
      uint16_t* dst = v_cache + (((size_t)blk * nkv + vh) * block_size + off) * hd;
      *reinterpret_cast<u32x4*>(dst + c * 8) = v;
    }
  }
}

extern "C" int dgi_rope_cache(void* qkv, int T, int qkv_stride, const int* positions,
                              const float* cos_sin, int nh, int nkv, int hd, const int* slot_mapping,
                              void* k_cache, void* v_cache, int block_size, hipStream_t s) {
  if (hd % 16 || qkv_stride % 8) return -2;
  if (T == 0) return 0;
  rope_cache_kernel<<<T, 256, 0, s>>>((uint16_t*)qkv, qkv_stride, positions, cos_sin, nh, nkv, hd,
                                      slot_mapping, (uint16_t*)k_cache, (uint16_t*)v_cache,
                                      block_size, 1);
  DGI_CHECK_LAUNCH();
  return 0;
}
