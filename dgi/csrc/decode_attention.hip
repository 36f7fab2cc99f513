// dgi/csrc/decode_attention.hip — paged GQA decode attention, split-KV.
//
// The reference decodes through HF `model.generate` with a dense per-request
// cache (worker/engines/llm.py:61-69) and its shard path drops the KV
// entirely (worker/distributed/grpc_server.py:365-374).  This kernel reads
// the paged pool written by rope_cache.hip.
//
// Work decomposition (CDNA4, wave64):
//   grid = (max_splits, n_kv_heads, batch), 4 waves (8 when a short-context,
//   small-batch step runs one split per sequence: no partials, no reduce kernel).
//   A workgroup owns one (sequence, kv-head, KV split) and all G = nh/nkv
//   query heads of that kv head, so each K/V byte is read from HBM once per
//   decode step regardless of the GQA ratio.
//   Each wave walks 32-token tiles.  Scores are computed "swapped":
//     S^T[token][query] = K[token][:] . Q[query][:]   (mfma_f32_16x16x32_bf16,
//   K fragments straight from HBM into VGPRs, Q fragments resident), so a lane
//   owns one query column and the online softmax needs only two xor-shuffles.
//   The probabilities then feed  O^T[dim][query] += V^T[dim][token] . P^T
//   directly from the accumulator registers; V^T comes from a per-wave LDS
//   tile through ds_read_b64_tr_b16 (hardware transpose) with an XOR swizzle
//   that makes the transposed reads bank-conflict free.
//   The 4 waves merge (m, l, O) through LDS; with more than one split the
//   partial results (normalised O and log2-sum-exp) go to a workspace and
//   either the last-arriving split of each (sequence, kv head) combines them
//   in the same launch (ticket counters in the workspace: write-through
//   partials, one relaxed ticket, one acquire on the last arriver) or a small
//   reduce kernel does.
#include "common.h"

using namespace dgi;

namespace {

// buffer resource word 3 of a raw (stride 0, byte-addressed) buffer on gfx9, and the cache
// policy bit of a write-through (sc1) access
constexpr int kRsrcWord3 = 0x00020000;
constexpr int kSc1 = 16;

template <int HD>
__device__ __forceinline__ int v_lds_off(int row, int col) {
  constexpr int NCH = HD / 8;  // 16-byte chunks per row
  const int ch = (col >> 3) ^ (((row & 7) << 1) & (NCH - 1));
  return row * HD + (ch << 3) + (col & 7);
}

// per-wave LDS: the V tile (32 x HD bf16), reused after the loop for the wave's
// partial O (16 queries x HD fp32, rows padded by 4 floats so the 16 query rows
// of one store land in different banks) plus m / l
__device__ __forceinline__ int o_swz(int q) { return ((q & 3) << 3) | (q >> 2); }

template <int HD>
constexpr int decode_wave_lds() {
  return (32 * HD * 2 > 16 * (HD + 4) * 4 ? 32 * HD * 2 : 16 * (HD + 4) * 4) + 128;
}

template <int HD, int NW>
__global__ __launch_bounds__(64 * NW) void paged_decode_kernel(
    const uint16_t* __restrict__ q, int q_stride, const uint16_t* __restrict__ k_cache,
    const uint16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ context_lens, uint16_t* __restrict__ out, int out_stride,
    float* __restrict__ part_o, float* __restrict__ part_lse, int* __restrict__ counters, int max_splits, int nh,
    int nkv, int bs_log2, int part_size, float scale_log2, bool page16) {
  constexpr int KS = HD / 32;   // k-steps of the QK^T product
  constexpr int NC = HD / 16;   // 16-wide dim blocks of the PV product
  constexpr int VCH = HD / 8;   // 16-byte chunks per V row
  constexpr int WREG = decode_wave_lds<HD>();  // per-wave LDS bytes (V tile, then O/m/l)
  // fp32 row of the merged partial O: unpadded, columns XOR-swizzled per query row
  // (bits 0-1 ^= q >> 2, bits 3-4 ^= q & 3) so each 32-lane half of a ds_write_b32
  // (16 queries x 2 dim groups; banks (a/4) mod 32) hits 32 different banks; a padded
  // row (HD + 4) put 4 lanes on one bank
  constexpr int OROW = HD;
  constexpr int NT = 64 * NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int split = blockIdx.x;
  const int h = blockIdx.y;
  const int b = blockIdx.z;
  const int ctx = context_lens[b];
  // write-through views of the split workspace (fused reduce); byte ranges cover the launch
  const __amdgpu_buffer_rsrc_t po_rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)part_o, 0, (int)min((size_t)gridDim.z * nh * max_splits * HD * 4, (size_t)0x7fffffff), kRsrcWord3);
  const __amdgpu_buffer_rsrc_t pl_rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)part_lse, 0, (int)min((size_t)gridDim.z * nh * max_splits * 4, (size_t)0x7fffffff), kRsrcWord3);
  // part_size <= 0: device-side split plan from this sequence's own context —
  // up to max_splits parts of at least -part_size tokens (32-token multiples),
  // so a graph captured for the longest context does not leave short ones
  // with idle workgroups or a needless reduce
  int nsplit, part;
  if (part_size > 0) {
    part = part_size;
    nsplit = (ctx + part - 1) / part;
  } else {
    nsplit = max(1, min(max_splits, (ctx + (-part_size) - 1) / (-part_size)));
    part = (((ctx + nsplit - 1) / nsplit) + 31) & ~31;
    nsplit = (ctx + part - 1) / part;
  }
  const int start = split * part;
  if (start >= ctx) return;
  const int end = min(start + part, ctx);
  const int G = nh / nkv;
  const int bs = 1 << bs_log2;

  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: tile bases in SGPRs
  const int lane = tid & 63;
  const int qi = lane & 15;
  const int g = lane >> 4;
  uint16_t* vt = reinterpret_cast<uint16_t*>(smem + w * WREG);

  // Q fragments (B operand): B[k = 8g + j][col = query qi] = Q[qi][32 s + 8 g + j].  The 8-wave
  // one-split variant (small batch, short context: one or two tiles per wave) issues them after
  // its first tile's K/V loads, so the two round trips overlap instead of running back to back.
  u32x4 qf[KS];
  auto load_q = [&]() {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (qi < G) {
        qf[s] = *reinterpret_cast<const u32x4*>(q + (size_t)b * q_stride + (h * G + qi) * HD + 32 * s + 8 * g);
      } else {
        qf[s] = u32x4{0, 0, 0, 0};
      }
    }
  };
  constexpr bool LATE_Q = NW == 8;
  if (!LATE_Q) load_q();

  const int* bt = block_tables + (size_t)b * bt_stride;
  const size_t head_stride = (size_t)bs * HD;

  float m_run = -1e30f, l_run = 0.f;
  f32x4 o[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) o[c] = f32x4{0, 0, 0, 0};

  const int ntiles = (end - start + 31) >> 5;
  for (int t = w; t < ntiles; t += NW) {
    const int tb = start + (t << 5);
    u32x4 kf[2][KS];
    u32x4 vr[VCH / 2];
    if (page16 && tb + 32 <= end) {
      // full tile of 16-token pages (the engine's page size): its two pages come from two
      // scalar block-table reads, every lane's offset inside a page is a constant, so each
      // load is an SGPR base + a fixed VGPR offset (no per-load 64-bit address arithmetic:
      // at small batch the tile loop is VALU-issue-bound)
      const int fb = tb >> 4;
      const uint16_t* kp[2];
      const uint16_t* vp[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const size_t page = ((size_t)bt[fb + j] * nkv + h) * head_stride;
        kp[j] = k_cache + page;
        vp[j] = v_cache + page;
      }
      // ---- K fragments straight to VGPRs (A operand: row = token, k = dims)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int s = 0; s < KS; ++s)
          kf[u][s] = *reinterpret_cast<const u32x4*>(kp[u] + qi * HD + 32 * s + 8 * g);
      // ---- V tile -> registers (row 4k + lane / VCH of the tile; rows 16-31 on the second page)
#pragma unroll
      for (int k = 0; k < VCH / 2; ++k) {
        const int idx = k * 64 + lane;
        const int row = idx / VCH;
        vr[k] = *reinterpret_cast<const u32x4*>(vp[row >> 4] + (row & 15) * HD + (idx % VCH) * 8);
      }
    } else {
      // ---- K fragments straight to VGPRs (A operand: row = token, k = dims)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        int tok = tb + 16 * u + qi;
        tok = min(tok, end - 1);
        const int blk = bt[tok >> bs_log2];
        const uint16_t* kpl = k_cache + ((size_t)blk * nkv + h) * head_stride + (size_t)(tok & (bs - 1)) * HD;
#pragma unroll
        for (int s = 0; s < KS; ++s) kf[u][s] = *reinterpret_cast<const u32x4*>(kpl + 32 * s + 8 * g);
      }
      // ---- V tile -> registers -> swizzled LDS
#pragma unroll
      for (int k = 0; k < VCH / 2; ++k) {
        // 32 rows x VCH chunks; each pass covers 64/VCH rows
        const int idx = k * 64 + lane;
        const int row = idx / VCH;
        const int ch = idx % VCH;
        int tok = min(tb + row, end - 1);
        const int blk = bt[tok >> bs_log2];
        const uint16_t* vpl = v_cache + ((size_t)blk * nkv + h) * head_stride + (size_t)(tok & (bs - 1)) * HD;
        vr[k] = *reinterpret_cast<const u32x4*>(vpl + ch * 8);
      }
    }
    if (LATE_Q && t == w) load_q();
    // ---- S^T = K Q^T
    f32x4 sacc[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      sacc[u] = f32x4{0, 0, 0, 0};
#pragma unroll
      for (int s = 0; s < KS; ++s)
        sacc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(kf[u][s]), as_bf16x8(qf[s]), sacc[u], 0, 0, 0);
    }
    // write V (the previous tile's transposed reads are complete: in-order LDS per wave)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < VCH / 2; ++k) {
      const int idx = k * 64 + lane;
      const int row = idx / VCH;
      const int ch = idx % VCH;
      *reinterpret_cast<u32x4*>(vt + v_lds_off<HD>(row, ch * 8)) = vr[k];
    }
    // ---- online softmax (lane owns query qi; tokens 16u + 4g + i); only the sequence's last
    // tile has tokens past its end to mask
    const bool full = tb + 32 <= end;
    float x[2][4];
    float mx = -1e30f;
    if (full) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          x[u][i] = sacc[u][i] * scale_log2;
          mx = fmaxf(mx, x[u][i]);
        }
    } else {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int tok = tb + 16 * u + 4 * g + i;
          const float v = (tok < end) ? sacc[u][i] * scale_log2 : -1e30f;
          x[u][i] = v;
          mx = fmaxf(mx, v);
        }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    float psum = 0.f;
    float p[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // masked tokens hold -1e30: exp2 of (-1e30 - m_new) is exactly 0
        p[u][i] = __builtin_amdgcn_exp2f(x[u][i] - m_new);
        psum += p[u][i];
      }
    psum += __shfl_xor(psum, 16, 64);
    psum += __shfl_xor(psum, 32, 64);
    l_run = l_run * alpha + psum;
    m_run = m_new;
#pragma unroll
    for (int c = 0; c < NC; ++c) o[c] *= alpha;
    u32x4 pf;
    pf[0] = pack_bf16x2(p[0][0], p[0][1]);
    pf[1] = pack_bf16x2(p[0][2], p[0][3]);
    pf[2] = pack_bf16x2(p[1][0], p[1][1]);
    pf[3] = pack_bf16x2(p[1][2], p[1][3]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // ---- O^T += V^T P^T ; V^T fragments via transposed LDS reads
    const int tq = qi >> 2, tp = qi & 3;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_short4*)(vt + v_lds_off<HD>(4 * g + tq, 16 * c + 4 * tp)));
      short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_short4*)(vt + v_lds_off<HD>(16 + 4 * g + tq, 16 * c + 4 * tp)));
      u32x4 vf;
      vf[0] = (uint32_t)(uint16_t)lo[0] | ((uint32_t)(uint16_t)lo[1] << 16);
      vf[1] = (uint32_t)(uint16_t)lo[2] | ((uint32_t)(uint16_t)lo[3] << 16);
      vf[2] = (uint32_t)(uint16_t)hi[0] | ((uint32_t)(uint16_t)hi[1] << 16);
      vf[3] = (uint32_t)(uint16_t)hi[2] | ((uint32_t)(uint16_t)hi[3] << 16);
      o[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(vf), as_bf16x8(pf), o[c], 0, 0, 0);
    }
  }

  // ---- merge the NW waves through LDS
  __syncthreads();
  constexpr int MLOFF = WREG - 128;
  float* ow = reinterpret_cast<float*>(smem + w * WREG);            // [16 q][OROW] fp32
  float* ml = reinterpret_cast<float*>(smem + w * WREG + MLOFF);    // m[16], l[16]
  if (qi < G) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) ow[qi * OROW + ((16 * c + 4 * g + i) ^ o_swz(qi))] = o[c][i];
    if (g == 0) {
      ml[qi] = m_run;
      ml[16 + qi] = l_run;
    }
  }
  __syncthreads();
  for (int idx = tid; idx < G * HD; idx += NT) {
    const int qq = idx / HD;
    const int d = idx - qq * HD;
    float M = -1e30f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) M = fmaxf(M, reinterpret_cast<float*>(smem + ww * WREG + MLOFF)[qq]);
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) {
      const float* mlw = reinterpret_cast<float*>(smem + ww * WREG + MLOFF);
      const float sc = exp2f(mlw[qq] - M);
      L += mlw[16 + qq] * sc;
      acc += reinterpret_cast<float*>(smem + ww * WREG)[qq * OROW + (d ^ o_swz(qq))] * sc;
    }
    const int head = h * G + qq;
    const float r = acc / L;
    if (nsplit == 1) {
      out[(size_t)b * out_stride + head * HD + d] = f32_to_bf16(r);
    } else if (counters != nullptr) {
      // fused reduce: partials leave with write-through (sc1) stores, so no release fence
      // (an agent release writes back the whole L2) is needed before the ticket below
      const size_t pi = ((size_t)b * nh + head) * max_splits + split;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, r), po_rs,
                                            (int)((pi * HD + d) * 4), 0, kSc1);
      if (d == 0)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, M + log2f(L)), pl_rs, (int)(pi * 4), 0,
                                              kSc1);
    } else {
      const size_t pi = ((size_t)b * nh + head) * max_splits + split;
      part_o[pi * HD + d] = r;
      if (d == 0) part_lse[pi] = M + log2f(L);
    }
  }
  if (nsplit == 1 || counters == nullptr) return;
  // ---- fused split reduce (MI355X_MICROARCH "Valid forms"): every wave drains its sc1 stores,
  // the workgroup meets at a barrier, one lane takes a relaxed agent-scope ticket; the workgroup
  // that draws nsplit - 1 acquires once (invalidates its CU's L1) and combines every split in
  // split order (deterministic).  No workgroup waits for another: placement-independent.
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int ticket = __hip_atomic_fetch_add(&counters[b * nkv + h], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = ticket == nsplit - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // ready for the next launch (stream-ordered after this one)
      __hip_atomic_store(&counters[b * nkv + h], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  for (int idx = tid; idx < G * HD; idx += NT) {
    const int qq = idx / HD;
    const int d = idx - qq * HD;
    const int head = h * G + qq;
    const size_t base = ((size_t)b * nh + head) * max_splits;
    float M = -1e30f;
    for (int sp = 0; sp < nsplit; ++sp) M = fmaxf(M, part_lse[base + sp]);
    float W = 0.f, acc = 0.f;
    for (int sp = 0; sp < nsplit; ++sp) {
      const float wgt = exp2f(part_lse[base + sp] - M);
      W += wgt;
      acc += wgt * part_o[(base + sp) * HD + d];
    }
    out[(size_t)b * out_stride + head * HD + d] = f32_to_bf16(acc / W);
  }
}

template <int HD>
__global__ __launch_bounds__(HD) void decode_reduce_kernel(
    const float* __restrict__ part_o, const float* __restrict__ part_lse,
    const int* __restrict__ context_lens, uint16_t* __restrict__ out, int out_stride, int max_splits,
    int nh, int part_size) {
  const int b = blockIdx.x;
  const int head = blockIdx.y;
  const int ctx = context_lens[b];
  int nsplit;
  if (part_size > 0) {
    nsplit = (ctx + part_size - 1) / part_size;
  } else {  // same device-side plan as the attention kernel
    nsplit = max(1, min(max_splits, (ctx + (-part_size) - 1) / (-part_size)));
    const int part = (((ctx + nsplit - 1) / nsplit) + 31) & ~31;
    nsplit = (ctx + part - 1) / part;
  }
  if (nsplit <= 1) return;
  const size_t base = ((size_t)b * nh + head) * max_splits;
  float M = -1e30f;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, part_lse[base + s]);
  float W = 0.f, acc = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const float wgt = exp2f(part_lse[base + s] - M);
    W += wgt;
    acc += wgt * part_o[(base + s) * HD + threadIdx.x];
  }
  out[(size_t)b * out_stride + head * HD + threadIdx.x] = f32_to_bf16(acc / W);
}

}  // namespace

extern "C" int dgi_paged_decode(const void* q, int q_stride, const void* k_cache,
                                const void* v_cache, const int* block_tables, int bt_stride,
                                const int* context_lens, void* out, int out_stride, float* part_o,
                                float* part_lse, int* counters, int B, int nh, int nkv, int hd, int block_size,
                                int max_splits, int part_size, float scale, hipStream_t s) {
  if (B == 0) return 0;
  if (nh % nkv || nh / nkv > 16) return -2;
  // fixed parts: multiples of 128 tokens; dynamic (part_size <= 0): minimum part a multiple of 32
  if ((part_size > 0 && part_size % 128) || (part_size <= 0 && (part_size == 0 || (-part_size) % 32))) return -3;
  if (max_splits <= 1) counters = nullptr;
  // the fused reduce addresses the partials through 32-bit buffer offsets
  if ((size_t)B * nh * max_splits * hd * 4 >= ((size_t)1 << 31)) counters = nullptr;
  int bs_log2 = 0;
  while ((1 << bs_log2) < block_size) ++bs_log2;
  if ((1 << bs_log2) != block_size) return -4;
  const float scale_log2 = scale * 1.4426950408889634f;
  // full tiles of 16-token pages take the scalar-page-base load path (DGI_DECODE_PAGE16=0: off)
  static const bool page16_on = [] {
    const char* e = getenv("DGI_DECODE_PAGE16");
    return !(e && e[0] == '0');
  }();
  const bool page16 = page16_on && bs_log2 == 4;
  dim3 grid(max_splits, nkv, B);
  // few workgroups (small batch, one split: every (sequence, kv head) walks its whole
  // context): 8 waves per workgroup halve the serial tile chain of each wave
  const bool wide = max_splits == 1 && B * nkv <= 128;
  if (hd == 128) {
    if (wide) {
      paged_decode_kernel<128, 8><<<grid, 512, 8 * decode_wave_lds<128>(), s>>>(
          (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache,
          block_tables, bt_stride, context_lens, (uint16_t*)out, out_stride, part_o, part_lse,
          counters, max_splits, nh, nkv, bs_log2, part_size, scale_log2, page16);
    } else {
      paged_decode_kernel<128, 4><<<grid, 256, 4 * decode_wave_lds<128>(), s>>>(
          (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache,
          block_tables, bt_stride, context_lens, (uint16_t*)out, out_stride, part_o, part_lse,
          counters, max_splits, nh, nkv, bs_log2, part_size, scale_log2, page16);
    }
    DGI_CHECK_LAUNCH();
    if (max_splits > 1 && counters == nullptr) {
      decode_reduce_kernel<128><<<dim3(B, nh), 128, 0, s>>>(part_o, part_lse, context_lens,
                                                            (uint16_t*)out, out_stride, max_splits,
                                                            nh, part_size);
      DGI_CHECK_LAUNCH();
    }
  } else if (hd == 64) {
    if (wide) {
      paged_decode_kernel<64, 8><<<grid, 512, 8 * decode_wave_lds<64>(), s>>>(
          (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache,
          block_tables, bt_stride, context_lens, (uint16_t*)out, out_stride, part_o, part_lse,
          counters, max_splits, nh, nkv, bs_log2, part_size, scale_log2, page16);
    } else {
      paged_decode_kernel<64, 4><<<grid, 256, 4 * decode_wave_lds<64>(), s>>>(
          (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache,
          block_tables, bt_stride, context_lens, (uint16_t*)out, out_stride, part_o, part_lse,
          counters, max_splits, nh, nkv, bs_log2, part_size, scale_log2, page16);
    }
    DGI_CHECK_LAUNCH();
    if (max_splits > 1 && counters == nullptr) {
      decode_reduce_kernel<64><<<dim3(B, nh), 64, 0, s>>>(part_o, part_lse, context_lens,
                                                          (uint16_t*)out, out_stride, max_splits,
                                                          nh, part_size);
      DGI_CHECK_LAUNCH();
    }
  } else {
    return -5;
  }
  return 0;
}
