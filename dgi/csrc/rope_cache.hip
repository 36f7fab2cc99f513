// dgi/csrc/rope_cache.hip — fused RoPE(q,k) + paged KV-cache write.
//
// The reference relies on HF rotary embeddings and copies whole KV pages
// in Python (worker/distributed/kv_cache.py:133-136, 460-461).  Here one
// kernel reads the fused QKV GEMM output once:
//   * rotates q in place (NeoX/Llama "rotate_half" pairing, dims i, i+rd/2, or
//     GPT-J/GLM interleaved pairs 2i, 2i+1; partial rotary over the first rd dims),
//   * rotates k and scatters k and v into the paged cache at slot_mapping[t].
// Cache layout per layer: [num_blocks, n_kv, block_size, head_dim] so one
// (block, kv-head) page is a contiguous block_size*head_dim run that the
// attention kernels stream with 16-byte loads.
// Positions are arbitrary per token (chunked prefill, prefix reuse and
// EAGLE tree verification all pass non-contiguous positions).
#include "common.h"

using namespace dgi;

// mode 0: NeoX / Llama pairing (d, d + rd/2); mode 1: GPT-J / GLM interleaved
// pairing (2i, 2i+1).  Only the first rd dims rotate (partial rotary, GLM-4:
// rd = hd/2); dims [rd, hd) pass through (k still goes to the cache).
// cos_sin row layout: [rd/2 cos | rd/2 sin] for the rd/2 frequencies.
__global__ __launch_bounds__(256) void rope_cache_kernel(
    uint16_t* __restrict__ qkv, int qkv_stride, const int* __restrict__ positions,
    const float* __restrict__ cos_sin, int nh, int nkv, int hd, int rd, int mode,
    const int* __restrict__ slot_mapping, uint16_t* __restrict__ k_cache,
    uint16_t* __restrict__ v_cache, int block_size) {
  const int t = blockIdx.x;
  const int pos = positions[t];
  const int rhalf = rd >> 1;
  // work items per head: NeoX = pairs of 8-dim chunks (d, d+rd/2); interleaved = 8-dim chunks
  const int rchunks = mode == 0 ? (rhalf >> 3) : (rd >> 3);
  const int pchunks = (hd - rd) >> 3;   // pass-through chunks (k -> cache only)
  const int vchunks = hd >> 3;
  uint16_t* row = qkv + (size_t)t * qkv_stride;
  const float* cs = cos_sin + (size_t)pos * rd;
  const int slot = slot_mapping ? slot_mapping[t] : -1;
  const int blk = slot >= 0 ? slot / block_size : 0;
  const int off = slot >= 0 ? slot - blk * block_size : 0;

  const int n_rot = (nh + nkv) * rchunks;
  const int n_pass = nkv * pchunks;
  const int n_v = nkv * vchunks;
  for (int it = threadIdx.x; it < n_rot + n_pass + n_v; it += blockDim.x) {
    if (it < n_rot) {
      const int head = it / rchunks;
      const int c = it - head * rchunks;
      uint16_t* hp = row + head * hd;  // q heads then k heads are contiguous
      const int kh = head - nh;
      uint16_t* dst = (head >= nh && slot >= 0)
                          ? k_cache + (((size_t)blk * nkv + kh) * block_size + off) * hd : nullptr;
      if (mode == 0) {
        u32x4* p0 = reinterpret_cast<u32x4*>(hp + c * 8);
        u32x4* p1 = reinterpret_cast<u32x4*>(hp + rhalf + c * 8);
        float a[8], b[8], oa[8], ob[8], cv[8], sv[8];
        unpack8(*p0, a);
        unpack8(*p1, b);
        const float4* cp = reinterpret_cast<const float4*>(cs + c * 8);
        const float4* sp = reinterpret_cast<const float4*>(cs + rhalf + c * 8);
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
        } else if (dst) {
          *reinterpret_cast<u32x4*>(dst + c * 8) = ra;
          *reinterpret_cast<u32x4*>(dst + rhalf + c * 8) = rb;
        }
      } else {
        u32x4* p0 = reinterpret_cast<u32x4*>(hp + c * 8);
        float a[8], o[8];
        unpack8(*p0, a);
        const float4 cv = *reinterpret_cast<const float4*>(cs + c * 4);
        const float4 sv = *reinterpret_cast<const float4*>(cs + rhalf + c * 4);
        const float cc[4] = {cv.x, cv.y, cv.z, cv.w}, ss[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[2 * j] = a[2 * j] * cc[j] - a[2 * j + 1] * ss[j];
          o[2 * j + 1] = a[2 * j + 1] * cc[j] + a[2 * j] * ss[j];
        }
        const u32x4 r = pack8(o);
        if (head < nh) *p0 = r;
        else if (dst) *reinterpret_cast<u32x4*>(dst + c * 8) = r;
      }
    } else if (it < n_rot + n_pass) {
      if (slot < 0) continue;
      const int j = it - n_rot;
      const int kh = j / pchunks;
      const int c = j - kh * pchunks;
      const u32x4 k = *reinterpret_cast<const u32x4*>(row + (nh + kh) * hd + rd + c * 8);
      uint16_t* dst = k_cache + (((size_t)blk * nkv + kh) * block_size + off) * hd;
      *reinterpret_cast<u32x4*>(dst + rd + c * 8) = k;
    } else if (slot >= 0) {
      const int j = it - n_rot - n_pass;
      const int vh = j / vchunks;
      const int c = j - vh * vchunks;
      const u32x4 v = *reinterpret_cast<const u32x4*>(row + (nh + nkv + vh) * hd + c * 8);
      uint16_t* dst = v_cache + (((size_t)blk * nkv + vh) * block_size + off) * hd;
      *reinterpret_cast<u32x4*>(dst + c * 8) = v;
    }
  }
}

extern "C" int dgi_rope_cache(void* qkv, int T, int qkv_stride, const int* positions,
                              const float* cos_sin, int nh, int nkv, int hd, int rd, int mode,
                              const int* slot_mapping, void* k_cache, void* v_cache, int block_size,
                              hipStream_t s) {
  if (hd % 8 || qkv_stride % 8 || rd > hd || rd <= 0) return -2;
  if ((mode == 0 && rd % 16) || (mode == 1 && rd % 8) || (mode != 0 && mode != 1)) return -3;
  if (T == 0) return 0;
  rope_cache_kernel<<<T, 256, 0, s>>>((uint16_t*)qkv, qkv_stride, positions, cos_sin, nh, nkv, hd, rd, mode,
                                      slot_mapping, (uint16_t*)k_cache, (uint16_t*)v_cache, block_size);
  DGI_CHECK_LAUNCH();
  return 0;
}
