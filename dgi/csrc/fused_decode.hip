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
//    Every workgroup reduces the M <= 16 row norms itself (8 KB per row from
//    L2, overlapped with its first weight loads) and normalises its own X
//    fragments in registers, so no normalised copy of X ever goes to memory.
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
};

template <int U, int PRO>
struct Frag {
  u32x4 w[U][2][2];
  u32x4 x[U][2];
  u32x4 r[U][PRO == 2 ? 2 : 1];
  u32x4 gm[U][PRO ? 2 : 1];
};

template <int PRO>
__device__ __forceinline__ u32x4 normalise(u32x4 x, u32x4 r, u32x4 gm, float inv) {
  float v[8], g[8], o[8];
  unpack8(x, v);
  if (PRO == 2) {
    float rr[8];
    unpack8(r, rr);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += rr[j];
    unpack8(pack8(v), v);  // the residual stream is bf16
  }
  unpack8(gm, g);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = v[j] * inv * g[j];
  return pack8(o);
}

template <int NW, int U, int PRO, int EPI>
__global__ __launch_bounds__(NW * 64) void fused_skinny_kernel(FusedArgs a) {
  __shared__ f32x4 red[NW][2][64];
  __shared__ float s_part[NW][16];
  __shared__ float s_inv[16];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int K = a.K;
  const int bid = blockIdx.x;
  const int c0 = (bid / a.tpg) * a.gstride + (bid % a.tpg) * 16;
  const int c1 = c0 + a.pair_off;
  const int ngroups = (K >> 6) / (NW * U);
  const size_t lane_k = (size_t)g * 16 + (size_t)w * 64;
  const uint16_t* w0 = a.w + (size_t)(c0 + r) * K + lane_k;
  const uint16_t* w1 = a.w + (size_t)(c1 + r) * K + lane_k;
  const bool xval = r < a.M;
  const uint16_t* xrow = a.x + (size_t)(xval ? r : 0) * a.ldx + lane_k;
  const uint16_t* rrow = PRO == 2 ? a.res + (size_t)(xval ? r : 0) * a.ldr + lane_k : nullptr;
  const uint16_t* grow = PRO ? a.gamma + lane_k : nullptr;

  auto load = [&](Frag<U, PRO>& f, int grp) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t off = ((size_t)grp * NW * U + (size_t)u * NW) * 64;
      const u32x4* p0 = reinterpret_cast<const u32x4*>(w0 + off);
      const u32x4* p1 = reinterpret_cast<const u32x4*>(w1 + off);
      f.w[u][0][0] = __builtin_nontemporal_load(p0);
      f.w[u][0][1] = __builtin_nontemporal_load(p0 + 1);
      f.w[u][1][0] = __builtin_nontemporal_load(p1);
      f.w[u][1][1] = __builtin_nontemporal_load(p1 + 1);
      if (xval) {
        const u32x4* px = reinterpret_cast<const u32x4*>(xrow + off);
        f.x[u][0] = px[0];
        f.x[u][1] = px[1];
        if (PRO == 2) {
          const u32x4* pr = reinterpret_cast<const u32x4*>(rrow + off);
          f.r[u][0] = pr[0];
          f.r[u][1] = pr[1];
        }
      } else {
        f.x[u][0] = f.x[u][1] = u32x4{0u, 0u, 0u, 0u};
        if (PRO == 2) f.r[u][0] = f.r[u][1] = u32x4{0u, 0u, 0u, 0u};
      }
      if (PRO) {
        const u32x4* pg = reinterpret_cast<const u32x4*>(grow + off);
        f.gm[u][0] = pg[0];
        f.gm[u][1] = pg[1];
      }
    }
  };

  Frag<U, PRO> cur, nxt;
  load(cur, 0);  // first weight group in flight during the norm reduction

  float inv = 0.f;
  if (PRO) {
    // ---- row norms: M rows x K, 8 elements per thread-chunk
    const int nchunk = K >> 3;
    for (int m = 0; m < a.M; ++m) {
      float ss = 0.f;
      for (int c = tid; c < nchunk; c += NW * 64) {
        float v[8];
        unpack8(reinterpret_cast<const u32x4*>(a.x + (size_t)m * a.ldx)[c], v);
        if (PRO == 2) {
          float rr[8];
          unpack8(reinterpret_cast<const u32x4*>(a.res + (size_t)m * a.ldr)[c], rr);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] += rr[j];
          const u32x4 p = pack8(v);
          if (bid == 0) reinterpret_cast<u32x4*>(a.res_out + (size_t)m * a.ldr)[c] = p;
          unpack8(p, v);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
      }
      ss = wave_sum(ss);
      if (lane == 0) s_part[w][m] = ss;
    }
    __syncthreads();
    if (tid < a.M) {
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < NW; ++j) t += s_part[j][tid];
      s_inv[tid] = rsqrtf(t / (float)K + a.eps);
    }
    __syncthreads();
    inv = xval ? s_inv[r] : 0.f;
  }

  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  auto compute = [&](const Frag<U, PRO>& f) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      u32x4 xa = f.x[u][0], xb = f.x[u][1];
      if (PRO) {
        xa = normalise<PRO>(xa, f.r[u][0], f.gm[u][0], inv);
        xb = normalise<PRO>(xb, f.r[u][PRO == 2 ? 1 : 0], f.gm[u][1], inv);
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xa), as_bf16x8(f.w[u][nt][0]), acc[nt], 0, 0, 0);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xb), as_bf16x8(f.w[u][nt][1]), acc[nt], 0, 0, 0);
      }
    }
  };
  for (int grp = 0; grp + 1 < ngroups; ++grp) {
    load(nxt, grp + 1);
    compute(cur);
    cur = nxt;
  }
  compute(cur);

  red[w][0][lane] = acc[0];
  red[w][1][lane] = acc[1];
  __syncthreads();
  if (w != 0) return;
  f32x4 v0 = red[0][0][lane], v1 = red[0][1][lane];
#pragma unroll
  for (int j = 1; j < NW; ++j) {
    v0 += red[j][0][lane];
    v1 += red[j][1][lane];
  }
  const float b0 = a.bias ? bf16_to_f32(a.bias[c0 + r]) : 0.f;
  const float b1 = a.bias ? bf16_to_f32(a.bias[c1 + r]) : 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = g * 4 + i;
    if (m >= a.M) break;
    uint16_t* yrow = a.y + (size_t)m * a.ldy;
    if (EPI == 0) {
      yrow[c0 + r] = f32_to_bf16(v0[i] + b0);
      yrow[c1 + r] = f32_to_bf16(v1[i] + b1);
    } else if (EPI == 1) {
      const float gt = bf16_to_f32(f32_to_bf16(v0[i] + b0));
      const float up = bf16_to_f32(f32_to_bf16(v1[i] + b1));
      yrow[c0 + r] = f32_to_bf16(gt * __builtin_amdgcn_rcpf(1.f + __expf(-gt)) * up);
    } else {
      const int head = c0 >> 7;
      const int d = (c0 & 127) + r;  // 0..63
      const uint16_t x1 = f32_to_bf16(v0[i] + b0), x2 = f32_to_bf16(v1[i] + b1);
      if (head < a.nh + a.nkv) {
        const float* cs = a.cos_sin + (size_t)a.positions[m] * 128;
        const float cv = cs[d], sv = cs[64 + d];
        const float f1 = bf16_to_f32(x1), f2 = bf16_to_f32(x2);
        const uint16_t o1 = f32_to_bf16(f1 * cv - f2 * sv);
        const uint16_t o2 = f32_to_bf16(f2 * cv + f1 * sv);
        if (head < a.nh) {
          yrow[c0 + r] = o1;
          yrow[c1 + r] = o2;
        } else {
          yrow[c0 + r] = x1;
          yrow[c1 + r] = x2;
          const int slot = a.slots[m];
          if (slot >= 0) {
            const int bs = 1 << a.bs_log2;
            const size_t base = (((size_t)(slot >> a.bs_log2) * a.nkv + (head - a.nh)) * bs + (slot & (bs - 1))) * 128;
            a.k_cache[base + d] = o1;
            a.k_cache[base + d + 64] = o2;
          }
        }
      } else {
        yrow[c0 + r] = x1;
        yrow[c1 + r] = x2;
        const int slot = a.slots[m];
        if (slot >= 0) {
          const int bs = 1 << a.bs_log2;
          const size_t base =
              (((size_t)(slot >> a.bs_log2) * a.nkv + (head - a.nh - a.nkv)) * bs + (slot & (bs - 1))) * 128;
          a.v_cache[base + d] = x1;
          a.v_cache[base + d + 64] = x2;
        }
      }
    }
  }
}

template <int PRO, int EPI>
int launch(const FusedArgs& a, int nblocks, hipStream_t s) {
  // 8 waves x 2 K-steps per group (the skinny kernel's best M <= 16 config)
  fused_skinny_kernel<8, 2, PRO, EPI><<<dim3(nblocks), 512, 0, s>>>(a);
  DGI_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// pro: 0 none, 1 rmsnorm(x), 2 add + rmsnorm; epi: 0 store, 1 SwiGLU, 2 RoPE + KV write.
// N = output columns of y covered by the pairs: epi 0 -> N columns (pairs of adjacent 16-col
// tiles), epi 1 -> N = I gate columns (up rows at I + c), epi 2 -> N = (nh + 2 nkv) * 128.
extern "C" int dgi_fused_skinny(const void* x, int ldx, const void* res, int ldr, void* res_out,
                                const void* gamma, float eps, const void* w, const void* bias, void* y,
                                int ldy, int M, int N, int K, int pro, int epi, const int* positions,
                                const float* cos_sin, const int* slots, void* k_cache, void* v_cache, int nh,
                                int nkv, int block_size, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 16) return -2;
  if (K % 1024 || ldx % 8 || (pro == 2 && ldr % 8)) return -3;
  FusedArgs a{(const uint16_t*)x, ldx, (const uint16_t*)res, ldr, (uint16_t*)res_out, (const uint16_t*)gamma,
              eps, (const uint16_t*)w, (const uint16_t*)bias, (uint16_t*)y, ldy, M, K, 1, 32, 16,
              positions, cos_sin, slots, (uint16_t*)k_cache, (uint16_t*)v_cache, nh, nkv, 0};
  int nblocks;
  if (epi == 0) {
    if (N % 32) return -4;
    nblocks = N / 32;
  } else if (epi == 1) {
    if (N % 16) return -4;
    a.gstride = 16;
    a.pair_off = N;
    nblocks = N / 16;
  } else if (epi == 2) {
    if (N != (nh + 2 * nkv) * 128) return -4;
    int bl = 0;
    while ((1 << bl) < block_size) ++bl;
    if ((1 << bl) != block_size) return -4;
    a.bs_log2 = bl;
    a.tpg = 4;
    a.gstride = 128;
    a.pair_off = 64;
    nblocks = N / 32;
  } else {
    return -5;
  }
  if (pro < 0 || pro > 2) return -5;
#define DGI_FS(P, E) if (pro == P && epi == E) return launch<P, E>(a, nblocks, s);
  DGI_FS(0, 0) DGI_FS(1, 0) DGI_FS(2, 0)
  DGI_FS(0, 1) DGI_FS(1, 1) DGI_FS(2, 1)
  DGI_FS(0, 2) DGI_FS(1, 2) DGI_FS(2, 2)
#undef DGI_FS
  return -5;
}
