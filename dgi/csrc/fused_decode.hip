// dgi/csrc/fused_decode.hip — decode-step weight-streaming GEMMs with their
// neighbours fused in (SURVEY K2/K4/K9 folded into K3).
//
// At decode batch sizes (M <= 16) every layer is a chain of weight reads plus
// small per-row kernels.  On MI355X each of those small kernels costs 4-10 us
// of dispatch + ramp for a few KB of work (profiles/r1_decode8b_b1_kernel_stats.md:
// RMSNorm x2, RoPE+KV write, SiLU·mul = ~20 us per layer of a 4.1 ms 8B step).
// This kernel is the skinny GEMM of skinny_gemm.hip (16-column tiles, NW waves
// splitting K, weight fragments streamed straight to VGPRs as MFMA B operands)
// with two column tiles per workgroup — a *pair* (c0, c1 = c0 + pair_off) — and:
//
//  prologue PRO (the GEMM input is the normalised residual stream):
//    1: x = rmsnorm(h) * gamma                   (first layer: residual = h)
//    2: x = rmsnorm(h + res) * gamma, res_out = bf16(h + res)   (fused add)
//    Every workgroup stages the M <= 16 normalised rows in LDS itself (8-16 KB
//    per row from L2, overlapped with its first weight loads) and feeds the
//    MFMA A fragments from there, so no normalised copy of X goes to HBM and
//    the norm costs M*K work per workgroup, not 16 MFMA rows per lane.
//    Workgroup 0 writes res_out; res_out must not alias h or res (the other
//    workgroups are still reading them).
//  epilogue EPI on the pair:
//    0: store both tiles (plain 32-column GEMM);
//    1: SwiGLU — c0 is a gate column, c1 = c0 + I its up column:
//       y[:, c0] = silu(bf16(gate)) * bf16(up), the [M, 2I] intermediate never
//       exists;
//    2: RoPE + paged KV write — the pair is (d, d + 64) of one 128-dim head
//       (NeoX rotate-half pairing): q heads are rotated into y, k heads are
//       rotated into the paged cache (y keeps the raw k/v like rope_cache.hip
//       does), v heads are copied to the cache.
// Rounding follows the unfused kernels step by step (bf16 residual, bf16 GEMM
// outputs before SiLU / RoPE), so fused and unfused decode agree to the last
// bf16 ulp except for fp32 summation order inside the norm.
#include "common.h"

using namespace dgi;

namespace {

constexpr size_t kMaxStagedBytes = 136 * 1024;

struct FusedArgs {
  const uint16_t* x;  // h [M, ldx]
  int ldx;
  const uint16_t* res;  // residual [M, ldr] (PRO 2)
  int ldr;
  uint16_t* res_out;  // [M, ldr] (PRO 2)
  const uint16_t* gamma;  // [K]
  float eps;
  const uint16_t* w;  // [N_rows, K]
  const uint16_t* bias;  // [N_rows] or null
  uint16_t* y;
  int ldy;
  int M, K;
  int tpg, gstride, pair_off;  // column pair of workgroup b: c0 = (b / tpg) * gstride + (b % tpg) * 16
  // EPI 2
  const int* positions;
  const float* cos_sin;  // [max_pos, 128] = [64 cos | 64 sin]
  const int* slots;
  uint16_t* k_cache;  // [blocks, nkv, bs, 128]
  uint16_t* v_cache;
  int nh, nkv, bs_log2;
  // KS > 1: per-tile fp32 partials [tile][KS][64 lanes] and arrival counters (zero between launches)
  float* ws;
  int* cnt;
};

// buffer resource word 3 of a raw byte-addressed buffer, and the write-through (sc1) policy bit
constexpr int kRsrcWord3 = 0x00020000;
constexpr int kSc1 = 16;
constexpr int kKsMaxTiles = 4096;
constexpr int kKsMax = 2;

template <int U, int TW>
struct Frag {
  u32x4 w[U][TW][2];
};

// Stage the M normalised X rows into LDS (residual add + RMSNorm per PRO): only the
// M useful rows, spread over all threads (not 16 MFMA rows per lane).  Workgroup 0
// writes res_out.
template <int NW, int PRO>
__device__ __forceinline__ void stage_x(const FusedArgs& a, uint16_t* xs, float (*s_part)[16], float* s_inv,
                                        int bid) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int K = a.K;
  const int M = a.M;
  const int ldx = K + 8;
  const int nchunk = K >> 3;
  for (int m = 0; m < M; ++m) {
    float ss = 0.f;
    for (int c = tid; c < nchunk; c += NW * 64) {
      u32x4 p = reinterpret_cast<const u32x4*>(a.x + (size_t)m * a.ldx)[c];
      if (PRO == 2) {
        float v[8], rr[8];
        unpack8(p, v);
        unpack8(reinterpret_cast<const u32x4*>(a.res + (size_t)m * a.ldr)[c], rr);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += rr[j];
        p = pack8(v);  // the residual stream is bf16
        if (bid == 0) reinterpret_cast<u32x4*>(a.res_out + (size_t)m * a.ldr)[c] = p;
      }
      if (PRO) {
        float v[8];
        unpack8(p, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
      }
      *reinterpret_cast<u32x4*>(xs + m * ldx + c * 8) = p;
    }
    if (PRO) {
      ss = wave_sum(ss);
      if (lane == 0) s_part[w][m] = ss;
    }
  }
  if (PRO) {
    __syncthreads();
    if (tid < M) {
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < NW; ++j) t += s_part[j][tid];
      s_inv[tid] = rsqrtf(t / (float)K + a.eps);
    }
    __syncthreads();
    // each thread rescales the chunks it staged itself (same (m, c) mapping)
    for (int m = 0; m < M; ++m) {
      const float inv = s_inv[m];
      for (int c = tid; c < nchunk; c += NW * 64) {
        float v[8], gm[8], o[8];
        unpack8(*reinterpret_cast<const u32x4*>(xs + m * ldx + c * 8), v);
        unpack8(reinterpret_cast<const u32x4*>(a.gamma)[c], gm);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = v[j] * inv * gm[j];
        *reinterpret_cast<u32x4*>(xs + m * ldx + c * 8) = pack8(o);
      }
    }
  }
  __syncthreads();
}

// Epilogue rows on wave 0: (v0, v1) = output rows (row0, row1) for the M rows of lane
// group g; st0 / st1: this lane stores row0 / row1.  EPI 0 store, 1 SwiGLU (row0 a gate
// row, row1 its up row), 2 RoPE + paged KV write (row0 = d, row1 = d + 64 of one head).
template <int EPI>
__device__ __forceinline__ void store_rows(const FusedArgs& a, int row0, int row1, int g, bool st0, bool st1,
                                           float b0, float b1, const f32x4& v0, const f32x4& v1) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = g * 4 + i;
    if (m >= a.M) break;
    uint16_t* yrow = a.y + (size_t)m * a.ldy;
    if (EPI == 0) {
      if (st0) yrow[row0] = f32_to_bf16(v0[i] + b0);
      if (st1) yrow[row1] = f32_to_bf16(v1[i] + b1);
    } else if (EPI == 1) {
      const float gt = bf16_to_f32(f32_to_bf16(v0[i] + b0));
      const float up = bf16_to_f32(f32_to_bf16(v1[i] + b1));
      if (st0) yrow[row0] = f32_to_bf16(gt * __builtin_amdgcn_rcpf(1.f + __expf(-gt)) * up);
    } else {
      const int head = row0 >> 7;
      const int d = row0 & 127;  // 0..63
      const uint16_t x1 = f32_to_bf16(v0[i] + b0), x2 = f32_to_bf16(v1[i] + b1);
      if (head < a.nh + a.nkv) {
        const float* cs = a.cos_sin + (size_t)a.positions[m] * 128;
        const float cv = cs[d], sv = cs[64 + d];
        const float f1 = bf16_to_f32(x1), f2 = bf16_to_f32(x2);
        const uint16_t o1 = f32_to_bf16(f1 * cv - f2 * sv);
        const uint16_t o2 = f32_to_bf16(f2 * cv + f1 * sv);
        if (head < a.nh) {
          if (st0) yrow[row0] = o1;
          if (st1) yrow[row1] = o2;
        } else {
          if (st0) yrow[row0] = x1;
          if (st1) yrow[row1] = x2;
          const int slot = a.slots[m];
          if (slot >= 0) {
            const int bs = 1 << a.bs_log2;
            const size_t base = (((size_t)(slot >> a.bs_log2) * a.nkv + (head - a.nh)) * bs + (slot & (bs - 1))) * 128;
            if (st0) a.k_cache[base + d] = o1;
            if (st1) a.k_cache[base + d + 64] = o2;
          }
        }
      } else {
        if (st0) yrow[row0] = x1;
        if (st1) yrow[row1] = x2;
        const int slot = a.slots[m];
        if (slot >= 0) {
          const int bs = 1 << a.bs_log2;
          const size_t base =
              (((size_t)(slot >> a.bs_log2) * a.nkv + (head - a.nh - a.nkv)) * bs + (slot & (bs - 1))) * 128;
          if (st0) a.v_cache[base + d] = x1;
          if (st1) a.v_cache[base + d + 64] = x2;
        }
      }
    }
  }
}

// Epilogue of one column pair on wave 0: (v0, v1) = rows (c0 + rr, c1 + rr).
template <int TW, int EPI>
__device__ __forceinline__ void store_pair(const FusedArgs& a, int c0, int c1, int r, int g, bool lo,
                                           const f32x4& v0, const f32x4& v1) {
  const int rr = TW == 2 ? r : (r & 7);
  const float b0 = (TW == 2 && a.bias) ? bf16_to_f32(a.bias[c0 + r]) : 0.f;
  const float b1 = (TW == 2 && a.bias) ? bf16_to_f32(a.bias[c1 + r]) : 0.f;
  // TW 1: lanes r < 8 store the pair's first half, r >= 8 the second
  store_rows<EPI>(a, c0 + rr, c1 + rr, g, TW == 2 || lo, TW == 2 || !lo, b0, b1, v0, v1);
}

// TW: 16-row weight tiles per workgroup.  TW = 2 is the pair (c0 + r, c1 + r);
// TW = 1 packs both halves of a pair into one tile — lanes r < 8 read rows c0 + r,
// lanes r >= 8 rows c1 + r - 8 — and swaps the halves with a lane shuffle in the
// epilogue: half the rows per workgroup, twice the workgroups (qkv on 8B: 384
// instead of 192 on 256 CUs).  D: load groups in flight (register ring); the
// first D are issued before the X staging.
// KS > 1 (TW = 1 only) splits K over KS workgroups per pair tile: 8B qkv has 384 pair
// tiles, 1.5 per CU, so half the CUs stream twice the bytes of the other half; 768
// half-K workgroups are 3 per CU.  Each part publishes its cross-wave sum (1 KB) with
// write-through stores and bumps the tile's counter; the last part to arrive sums every
// part in part order (deterministic) and runs the epilogue.
template <int NW, int U, int TW, int D, int PRO, int EPI, int KS = 1>
__global__ __launch_bounds__(NW * 64) void fused_skinny_kernel(FusedArgs a) {
  static_assert(KS == 1 || TW == 1, "split-K pairs are one-tile workgroups");
  // normalised X rows live in LDS for the whole kernel: [M][K + 8] bf16 (16-byte
  // row pad keeps the 16-row fragment reads off one bank)
  extern __shared__ __attribute__((aligned(16))) uint16_t xs[];
  __shared__ f32x4 red[NW][TW][64];
  __shared__ float s_part[NW][16];
  __shared__ float s_inv[16];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int K = a.K;
  const int M = a.M;
  const int ldx = K + 8;
  const int bid = blockIdx.x;
  // KS > 1: the parts of one tile are workgroups 8 apart (one XCD under round-robin
  // dispatch, so the partials meet in that XCD's L2) when the grid is a multiple of 8 KS
  int tile = bid, part = 0;
  if (KS > 1) {
    if ((gridDim.x % (8 * KS)) == 0) {
      tile = (bid / (8 * KS)) * 8 + (bid & 7);
      part = (bid >> 3) % KS;
    } else {
      tile = bid / KS;
      part = bid % KS;
    }
  }
  const int c0 = (tile / a.tpg) * a.gstride + (tile % a.tpg) * (TW == 2 ? 16 : 8);
  const int c1 = c0 + a.pair_off;
  const int ngroups = ((K / KS) >> 6) / (NW * U);
  const size_t lane_k = (size_t)g * 16 + (size_t)w * 64 + (size_t)part * (K / KS);
  const bool lo = r < 8;
  const uint16_t* w0 = a.w + (size_t)(TW == 2 ? c0 + r : (lo ? c0 + r : c1 + r - 8)) * K + lane_k;
  const uint16_t* w1 = a.w + (size_t)(c1 + r) * K + lane_k;
  const bool xval = r < M;

  auto load = [&](Frag<U, TW>& f, int grp) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t off = ((size_t)grp * NW * U + (size_t)u * NW) * 64;
      const u32x4* p0 = reinterpret_cast<const u32x4*>(w0 + off);
      f.w[u][0][0] = __builtin_nontemporal_load(p0);
      f.w[u][0][1] = __builtin_nontemporal_load(p0 + 1);
      if (TW == 2) {
        const u32x4* p1 = reinterpret_cast<const u32x4*>(w1 + off);
        f.w[u][TW - 1][0] = __builtin_nontemporal_load(p1);
        f.w[u][TW - 1][1] = __builtin_nontemporal_load(p1 + 1);
      }
    }
  };

  // the first D groups stream while X is staged
  Frag<U, TW> ring[D];
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (d < ngroups) load(ring[d], d);

  stage_x<NW, PRO>(a, xs, s_part, s_inv, bid);

  const uint16_t* xl = xs + (xval ? r : 0) * ldx + lane_k;
  f32x4 acc[TW];
#pragma unroll
  for (int nt = 0; nt < TW; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const Frag<U, TW>& f, int grp) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int off = (grp * NW * U + u * NW) * 64;
      u32x4 xa = u32x4{0u, 0u, 0u, 0u}, xb = u32x4{0u, 0u, 0u, 0u};
      if (xval) {
        xa = *reinterpret_cast<const u32x4*>(xl + off);
        xb = *reinterpret_cast<const u32x4*>(xl + off + 8);
      }
#pragma unroll
      for (int nt = 0; nt < TW; ++nt) {
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xa), as_bf16x8(f.w[u][nt][0]), acc[nt], 0, 0, 0);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xb), as_bf16x8(f.w[u][nt][1]), acc[nt], 0, 0, 0);
      }
    }
  };
  for (int base = 0; base < ngroups; base += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      if (base + d < ngroups) {  // uniform; only the last round of a ragged ring is partial
        compute(ring[d], base + d);
        if (base + D + d < ngroups) load(ring[d], base + D + d);
      }
    }
  }

#pragma unroll
  for (int nt = 0; nt < TW; ++nt) red[w][nt][lane] = acc[nt];
  __syncthreads();
  if (w != 0) return;
  f32x4 v0 = red[0][0][lane], v1 = red[0][TW - 1][lane];
#pragma unroll
  for (int j = 1; j < NW; ++j) {
    v0 += red[j][0][lane];
    if (TW == 2) v1 += red[j][1][lane];
  }
  if (KS > 1) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.ws + (size_t)tile * KS * 256), 0, KS * 256 * 4, kRsrcWord3);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v0), rs, (part * 64 + lane) * 16, 0, kSc1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __shfl(old, 0);
    if (old != KS - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (lane == 0) __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v0 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < KS; ++j)
      v0 += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (j * 64 + lane) * 16, 0, 0));
    v1 = v0;
  }
  if (TW == 1) {
    // this lane holds row c0 + r (r < 8) or c1 + r - 8; bring the other half of
    // the pair over from lane ^ 8 (same row group g) so the epilogue below sees
    // (v0, v1) = (row c0 + (r & 7), row c1 + (r & 7)) on every lane
    const float bo = a.bias ? bf16_to_f32(a.bias[lo ? c0 + r : c1 + r - 8]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float own = v0[i] + bo;
      const float oth = __shfl_xor(own, 8);
      v0[i] = lo ? own : oth;
      v1[i] = lo ? oth : own;
    }
  }
  store_pair<TW, EPI>(a, c0, c1, r, g, lo, v0, v1);
}

// Persistent variant (TW = 1): a workgroup owns `tpw` consecutive pair tiles and
// streams their weights as ONE register ring — the next tile's first groups are in
// flight while the current tile's last groups are consumed and its epilogue runs —
// and stages X once per workgroup instead of once per tile.  With one workgroup per
// CU (8B gate_up: 1792 tiles = 7 per CU) every CU reads one unbroken weight stream
// instead of a launch's worth of short per-tile ramps and drains.  The cross-wave sum
// uses two LDS buffers by tile parity, so one barrier per tile suffices.
template <int NW, int U, int D, int PRO, int EPI>
__global__ __launch_bounds__(NW * 64) void fused_skinny_persist_kernel(FusedArgs a, int tpw, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) uint16_t xs[];
  __shared__ f32x4 red[2][NW][64];
  __shared__ float s_part[NW][16];
  __shared__ float s_inv[16];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int K = a.K;
  const int M = a.M;
  const int ldx = K + 8;
  const int bid = blockIdx.x;
  const int t_first = bid * tpw;
  const int nt_local = min(tpw, ntiles - t_first);   // >= 1: the host sizes the grid
  const int ngroups = (K >> 6) / (NW * U);
  const int total = nt_local * ngroups;
  const size_t lane_k = (size_t)g * 16 + (size_t)w * 64;
  const bool lo = r < 8;
  const bool xval = r < M;
  // Walk the flattened groups s (tile t_first + s / ngroups, K group s % ngroups) with
  // incremental cursors: a runtime integer division is ~30 scalar instructions, and with
  // two per group (consumer and loader) the scalar unit, shared by the CU's 16 waves, was
  // issuing more than the vector units (PMC, profiles/r4_decode/pmc_decode8b_b1_step.md)
  struct Cursor { int grp, tq, tr; };       // K group, (tile / tpg, tile % tpg)
  auto c0_of = [&](const Cursor& c) { return c.tq * a.gstride + c.tr * 8; };
  auto advance = [&](Cursor& c) {
    if (++c.grp == ngroups) {
      c.grp = 0;
      if (++c.tr == a.tpg) { c.tr = 0; ++c.tq; }
    }
  };
  auto load = [&](Frag<U, 1>& f, const Cursor& c) {
    const int c0 = c0_of(c);
    const uint16_t* w0 = a.w + (size_t)(lo ? c0 + r : c0 + a.pair_off + r - 8) * K + lane_k;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t off = ((size_t)c.grp * NW * U + (size_t)u * NW) * 64;
      const u32x4* p0 = reinterpret_cast<const u32x4*>(w0 + off);
      f.w[u][0][0] = __builtin_nontemporal_load(p0);
      f.w[u][0][1] = __builtin_nontemporal_load(p0 + 1);
    }
  };
  Cursor cons{0, t_first / a.tpg, t_first % a.tpg};   // the group being consumed
  Cursor ld = cons;                                      // the next group to load
  Frag<U, 1> ring[D];
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (d < total) {
      load(ring[d], ld);
      advance(ld);
    }

  stage_x<NW, PRO>(a, xs, s_part, s_inv, bid);

  const uint16_t* xl = xs + (xval ? r : 0) * ldx + lane_k;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  int parity = 0;
  for (int base = 0; base < total; base += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int s = base + d;
      if (s < total) {          // uniform
        const int grp = cons.grp;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int off = (grp * NW * U + u * NW) * 64;
          u32x4 xa = u32x4{0u, 0u, 0u, 0u}, xb = u32x4{0u, 0u, 0u, 0u};
          if (xval) {
            xa = *reinterpret_cast<const u32x4*>(xl + off);
            xb = *reinterpret_cast<const u32x4*>(xl + off + 8);
          }
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xa), as_bf16x8(ring[d].w[u][0][0]), acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xb), as_bf16x8(ring[d].w[u][0][1]), acc, 0, 0, 0);
        }
        if (s + D < total) {
          load(ring[d], ld);
          advance(ld);
        }
        if (grp == ngroups - 1) {     // tile done: cross-wave sum, epilogue on wave 0
          red[parity][w][lane] = acc;
          __syncthreads();
          if (w == 0) {
            const int c0 = c0_of(cons);
            const int c1 = c0 + a.pair_off;
            f32x4 v = red[parity][0][lane];
#pragma unroll
            for (int j = 1; j < NW; ++j) v += red[parity][j][lane];
            const float bo = a.bias ? bf16_to_f32(a.bias[lo ? c0 + r : c1 + r - 8]) : 0.f;
            f32x4 v0, v1;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float own = v[i] + bo;
              const float oth = __shfl_xor(own, 8);
              v0[i] = lo ? own : oth;
              v1[i] = lo ? oth : own;
            }
            store_pair<1, EPI>(a, c0, c1, r, g, lo, v0, v1);
          }
          acc = f32x4{0.f, 0.f, 0.f, 0.f};
          parity ^= 1;
        }
        advance(cons);
      }
    }
  }
}

// Balanced persistent variant ("quarter pairs"): the rows are cut into quarter pairs of
// 4 + 4 rows (half of a TW = 1 pair tile) and every workgroup streams qpw consecutive
// quarters, two per MFMA step (lanes r & 7 < 4 hold the step's first quarter, >= 4 its
// second; a step with one quarter leaves the upper lanes idle: no loads, no stores).
// 8B qkv: 384 pair tiles are 1.5 per CU, so the one-tile workgroups put 262 KB on half of
// the CUs and 131 KB on the rest; 768 quarters = 3 per CU stream 196 KB on every CU.
template <int NW, int U, int D, int PRO, int EPI>
__global__ __launch_bounds__(NW * 64) void fused_skinny_quarter_kernel(FusedArgs a, int qpw, int nq) {
  extern __shared__ __attribute__((aligned(16))) uint16_t xs[];
  __shared__ f32x4 red[2][NW][64];
  __shared__ float s_part[NW][16];
  __shared__ float s_inv[16];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int K = a.K;
  const int M = a.M;
  const int ldx = K + 8;
  const int bid = blockIdx.x;
  const int q_first = bid * qpw;
  const int nq_local = min(qpw, nq - q_first);   // >= 1: the host sizes the grid
  const int nsteps = (nq_local + 1) >> 1;
  const int ngroups = (K >> 6) / (NW * U);
  const int total = nsteps * ngroups;
  const size_t lane_k = (size_t)g * 16 + (size_t)w * 64;
  const bool lo = r < 8;
  const int j = r & 7;
  const bool xval = r < M;
  // c0-side weight row of this lane in step st; -1 when the step has no second quarter
  auto lane_row = [&](int st) -> int {
    const int qq = 2 * st + (j >> 2);
    if (qq >= nq_local) return -1;
    const int qp = q_first + qq;
    const int ti = qp >> 1;
    return (ti / a.tpg) * a.gstride + (ti % a.tpg) * 8 + (qp & 1) * 4 + (j & 3);
  };
  // incremental cursor over the flattened groups (step s / ngroups, K group s % ngroups): no
  // integer division per group; the lane's row is recomputed once per step
  struct Cursor { int grp, st, row; };
  auto advance = [&](Cursor& c) {
    if (++c.grp == ngroups) {
      c.grp = 0;
      c.row = lane_row(++c.st);
    }
  };
  auto load = [&](Frag<U, 1>& f, const Cursor& c) {
    if (c.row < 0) return;   // idle lanes: their MFMA columns are never stored
    const uint16_t* w0 = a.w + (size_t)(lo ? c.row : c.row + a.pair_off) * K + lane_k;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t off = ((size_t)c.grp * NW * U + (size_t)u * NW) * 64;
      const u32x4* p0 = reinterpret_cast<const u32x4*>(w0 + off);
      f.w[u][0][0] = __builtin_nontemporal_load(p0);
      f.w[u][0][1] = __builtin_nontemporal_load(p0 + 1);
    }
  };
  Cursor cons{0, 0, lane_row(0)};
  Cursor ld = cons;
  Frag<U, 1> ring[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
#pragma unroll
    for (int u = 0; u < U; ++u) ring[d].w[u][0][0] = ring[d].w[u][0][1] = u32x4{0u, 0u, 0u, 0u};
    if (d < total) {
      load(ring[d], ld);
      advance(ld);
    }
  }

  stage_x<NW, PRO>(a, xs, s_part, s_inv, bid);

  const uint16_t* xl = xs + (xval ? r : 0) * ldx + lane_k;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  int parity = 0;
  for (int base = 0; base < total; base += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int s = base + d;
      if (s < total) {          // uniform
        const int grp = cons.grp;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int off = (grp * NW * U + u * NW) * 64;
          u32x4 xa = u32x4{0u, 0u, 0u, 0u}, xb = u32x4{0u, 0u, 0u, 0u};
          if (xval) {
            xa = *reinterpret_cast<const u32x4*>(xl + off);
            xb = *reinterpret_cast<const u32x4*>(xl + off + 8);
          }
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xa), as_bf16x8(ring[d].w[u][0][0]), acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xb), as_bf16x8(ring[d].w[u][0][1]), acc, 0, 0, 0);
        }
        if (s + D < total) {
          load(ring[d], ld);
          advance(ld);
        }
        if (grp == ngroups - 1) {     // step done: cross-wave sum, epilogue on wave 0
          red[parity][w][lane] = acc;
          __syncthreads();
          if (w == 0) {
            const int row = cons.row;
            f32x4 v = red[parity][0][lane];
#pragma unroll
            for (int jj = 1; jj < NW; ++jj) v += red[parity][jj][lane];
            const float bo = (a.bias && row >= 0) ? bf16_to_f32(a.bias[lo ? row : row + a.pair_off]) : 0.f;
            f32x4 v0, v1;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float own = v[i] + bo;
              const float oth = __shfl_xor(own, 8);
              v0[i] = lo ? own : oth;
              v1[i] = lo ? oth : own;
            }
            if (row >= 0) store_rows<EPI>(a, row, row + a.pair_off, g, lo, !lo, 0.f, 0.f, v0, v1);
          }
          acc = f32x4{0.f, 0.f, 0.f, 0.f};
          parity ^= 1;
        }
        advance(cons);
      }
    }
  }
}

template <int NW, int U, int D, int PRO, int EPI>
int launch_quarter(FusedArgs a, int ntiles, hipStream_t s) {
  if ((a.K / 64) % (NW * U)) return -7;
  const size_t lds = (size_t)a.M * (a.K + 8) * 2;
  const size_t lds_static = (size_t)2 * NW * 64 * 16 + (size_t)NW * 16 * 4 + 16 * 4;
  if (lds + lds_static > 160 * 1024) return -6;
  // TW = 1 pair geometry (as launch_cfg)
  if (EPI == 0) {
    a.gstride = 16;
    a.pair_off = 8;
  } else if (EPI == 1) {
    a.gstride = 8;
  } else {
    a.tpg = 8;
  }
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  const int nq = 2 * ntiles;
  const int qpw = (nq + cus - 1) / cus;
  const int nblocks = (nq + qpw - 1) / qpw;
  fused_skinny_quarter_kernel<NW, U, D, PRO, EPI><<<dim3(nblocks), NW * 64, lds, s>>>(a, qpw, nq);
  DGI_CHECK_LAUNCH();
  return 0;
}

// Per-device split-K workspace (KS partial slabs + one counter per pair tile), allocated on
// first use outside stream capture; the engine runs its decode projections on one stream.
struct KsWorkspace {
  float* ws = nullptr;
  int* cnt = nullptr;
};

KsWorkspace* ks_workspace(hipStream_t s) {
  static KsWorkspace per_dev[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  KsWorkspace& w = per_dev[dev];
  if (w.ws) return &w;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  float* ws = nullptr;
  int* cnt = nullptr;
  if (hipMalloc(&ws, (size_t)kKsMaxTiles * kKsMax * 256 * sizeof(float)) != hipSuccess) return nullptr;
  if (hipMalloc(&cnt, (size_t)kKsMaxTiles * sizeof(int)) != hipSuccess ||
      hipMemset(cnt, 0, (size_t)kKsMaxTiles * sizeof(int)) != hipSuccess) {
    hipFree(ws);
    return nullptr;
  }
  w.ws = ws;
  w.cnt = cnt;
  return &w;
}

template <int NW, int U, int TW, int D, int PRO, int EPI, int KS = 1>
int launch_cfg(FusedArgs a, int N, int ntiles, hipStream_t s) {
  static_assert(KS <= kKsMax, "workspace holds kKsMax parts");
  if constexpr (KS > 1) {
    KsWorkspace* ks = ntiles <= kKsMaxTiles ? ks_workspace(s) : nullptr;
    // no workspace (first call inside a capture, huge N): the same launch without the split
    if (!ks) return launch_cfg<NW, U, TW, D * KS <= 8 ? D * KS : D, PRO, EPI, 1>(a, N, ntiles, s);
    a.ws = ks->ws;
    a.cnt = ks->cnt;
  }
  if ((a.K / KS / 64) % (NW * U)) return -7;
  const size_t lds = (size_t)a.M * (a.K + 8) * 2;
  // static (reduce tiles + norm partials) + staged X must fit the 160 KB of LDS
  const size_t lds_static = (size_t)NW * TW * 64 * 16 + (size_t)NW * 16 * 4 + 16 * 4;
  if (lds + lds_static > 160 * 1024) return -6;
  if (TW == 1) {
    // pairs of 8 rows: epi 0 16 consecutive columns, epi 1 8 gate + 8 up, epi 2 8 (d, d + 64) pairs
    if (EPI == 0) {
      a.gstride = 16;
      a.pair_off = 8;
    } else if (EPI == 1) {
      a.gstride = 8;
    } else {
      a.tpg = 8;
    }
  }
  const int nblocks = (TW == 2 ? ntiles / 2 : ntiles) * KS;
  fused_skinny_kernel<NW, U, TW, D, PRO, EPI, KS><<<dim3(nblocks), NW * 64, lds, s>>>(a);
  DGI_CHECK_LAUNCH();
  (void)N;
  return 0;
}

template <int NW, int U, int D, int PRO, int EPI>
int launch_persist(FusedArgs a, int ntiles, hipStream_t s) {
  if ((a.K / 64) % (NW * U)) return -7;
  const size_t lds = (size_t)a.M * (a.K + 8) * 2;
  const size_t lds_static = (size_t)2 * NW * 64 * 16 + (size_t)NW * 16 * 4 + 16 * 4;
  if (lds + lds_static > 160 * 1024) return -6;
  // TW = 1 pair geometry (as launch_cfg)
  if (EPI == 0) {
    a.gstride = 16;
    a.pair_off = 8;
  } else if (EPI == 1) {
    a.gstride = 8;
  } else {
    a.tpg = 8;
  }
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  const int tpw = (ntiles + cus - 1) / cus;
  const int nblocks = (ntiles + tpw - 1) / tpw;
  fused_skinny_persist_kernel<NW, U, D, PRO, EPI><<<dim3(nblocks), NW * 64, lds, s>>>(a, tpw, ntiles);
  DGI_CHECK_LAUNCH();
  return 0;
}

// cfg: (waves per workgroup, K-steps per load group, tiles per workgroup, groups in flight);
// 12-16: persistent (waves, K-steps per group, groups in flight) with TW = 1
template <int PRO, int EPI>
int launch(const FusedArgs& a, int N, int ntiles, int cfg, hipStream_t s) {
  switch (cfg) {
    case 0: case 1: return launch_cfg<8, 2, 2, 2, PRO, EPI>(a, N, ntiles, s);
    case 2: return launch_cfg<4, 4, 2, 2, PRO, EPI>(a, N, ntiles, s);
    case 3: return launch_cfg<16, 1, 2, 2, PRO, EPI>(a, N, ntiles, s);
    case 4: return launch_cfg<8, 1, 2, 2, PRO, EPI>(a, N, ntiles, s);
    case 5: return launch_cfg<4, 2, 2, 2, PRO, EPI>(a, N, ntiles, s);
    case 6: return launch_cfg<8, 1, 1, 4, PRO, EPI>(a, N, ntiles, s);
    case 7: return launch_cfg<8, 1, 2, 4, PRO, EPI>(a, N, ntiles, s);
    case 8: return launch_cfg<4, 2, 1, 4, PRO, EPI>(a, N, ntiles, s);
    case 9: return launch_cfg<4, 2, 2, 4, PRO, EPI>(a, N, ntiles, s);
    case 10: return launch_cfg<8, 2, 1, 2, PRO, EPI>(a, N, ntiles, s);
    case 11: return launch_cfg<4, 1, 1, 8, PRO, EPI>(a, N, ntiles, s);
    // persistent one-ring workgroups (TW = 1 pair tiles, ntiles of them)
    case 12: return launch_persist<8, 1, 8, PRO, EPI>(a, ntiles, s);
    case 13: return launch_persist<8, 2, 4, PRO, EPI>(a, ntiles, s);
    case 14: return launch_persist<4, 2, 8, PRO, EPI>(a, ntiles, s);
    case 15: return launch_persist<8, 2, 6, PRO, EPI>(a, ntiles, s);
    case 16: return launch_persist<16, 1, 4, PRO, EPI>(a, ntiles, s);
    // K split over two workgroups per pair tile (one-tile workgroups, TW = 1)
    case 17: return launch_cfg<8, 1, 1, 4, PRO, EPI, 2>(a, N, ntiles, s);
    case 18: return launch_cfg<4, 1, 1, 4, PRO, EPI, 2>(a, N, ntiles, s);
    case 19: return launch_cfg<8, 2, 1, 2, PRO, EPI, 2>(a, N, ntiles, s);
    case 20: return launch_cfg<4, 2, 1, 4, PRO, EPI, 2>(a, N, ntiles, s);
    case 21: return launch_cfg<4, 1, 1, 8, PRO, EPI, 2>(a, N, ntiles, s);
    // balanced persistent quarter-pair workgroups (waves, K-steps per group, groups in flight)
    case 22: return launch_quarter<8, 1, 8, PRO, EPI>(a, ntiles, s);
    case 23: return launch_quarter<8, 2, 4, PRO, EPI>(a, ntiles, s);
    case 24: return launch_quarter<16, 1, 4, PRO, EPI>(a, ntiles, s);
    case 25: return launch_quarter<4, 2, 8, PRO, EPI>(a, ntiles, s);
    case 26: return launch_quarter<8, 1, 4, PRO, EPI>(a, ntiles, s);
    default: return -5;
  }
}

}  // namespace

// pro: 0 none, 1 rmsnorm(x), 2 add + rmsnorm; epi: 0 store, 1 SwiGLU, 2 RoPE + KV write.
// N = output columns of y covered by the pairs: epi 0 -> N columns (pairs of adjacent 16-col
// tiles), epi 1 -> N = I gate columns (up rows at I + c), epi 2 -> N = (nh + 2 nkv) * 128.
extern "C" int dgi_fused_skinny(const void* x, int ldx, const void* res, int ldr, void* res_out,
                                const void* gamma, float eps, const void* w, const void* bias, void* y,
                                int ldy, int M, int N, int K, int pro, int epi, const int* positions,
                                const float* cos_sin, const int* slots, void* k_cache, void* v_cache, int nh,
                                int nkv, int block_size, int cfg, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 16) return -2;
  if (K % 1024 || ldx % 8 || (pro == 2 && ldr % 8)) return -3;
  if ((size_t)M * (K + 8) * 2 > kMaxStagedBytes) return -6;  // X must fit in LDS next to the reduce buffer
  FusedArgs a{(const uint16_t*)x, ldx, (const uint16_t*)res, ldr, (uint16_t*)res_out, (const uint16_t*)gamma,
              eps, (const uint16_t*)w, (const uint16_t*)bias, (uint16_t*)y, ldy, M, K, 1, 32, 16,
              positions, cos_sin, slots, (uint16_t*)k_cache, (uint16_t*)v_cache, nh, nkv, 0};
  int ntiles;  // 16-row weight tiles of the launch (two per workgroup at TW = 2)
  if (epi == 0) {
    if (N % 32) return -4;
    ntiles = N / 16;
  } else if (epi == 1) {
    if (N % 16) return -4;
    a.gstride = 16;
    a.pair_off = N;
    ntiles = N / 8;
  } else if (epi == 2) {
    if (N != (nh + 2 * nkv) * 128) return -4;
    int bl = 0;
    while ((1 << bl) < block_size) ++bl;
    if ((1 << bl) != block_size) return -4;
    a.bs_log2 = bl;
    a.tpg = 4;
    a.gstride = 128;
    a.pair_off = 64;
    ntiles = N / 16;
  } else {
    return -5;
  }
  if (pro < 0 || pro > 2) return -5;
#define DGI_FS(P, E) if (pro == P && epi == E) return launch<P, E>(a, N, ntiles, cfg, s);
  DGI_FS(0, 0) DGI_FS(1, 0) DGI_FS(2, 0)
  DGI_FS(0, 1) DGI_FS(1, 1) DGI_FS(2, 1)
  DGI_FS(0, 2) DGI_FS(1, 2) DGI_FS(2, 2)
#undef DGI_FS
  return -5;
}
