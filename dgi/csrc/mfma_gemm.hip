// dgi/csrc/mfma_gemm.hip — LDS-tiled MFMA GEMM for prefill / mixed-step projections
// (SURVEY K3/K8/K11), with an optional fused SwiGLU epilogue.
//
//   epi 0:  Y[M, N]  = X[M, K] · W[N, K]^T
//   epi 1:  Y[M, I]  = silu(X · Wg^T) * (X · Wu^T)   with W = [Wg; Wu] (2I x K, the
//           layout of the model's fused gate_up weight)
//
// bf16 in/out, fp32 accumulate.  Written for gfx950 (CDNA4), one 512-thread
// workgroup (8 waves) per CU:
//
//  * 256 x 256 output tile, K step 64, two LDS stages of X and W tiles
//    (2 x 64 KB): the whole 160 KB LDS budget goes to one deep tile, so every
//    staged byte feeds 256 MFMA columns;
//  * global -> LDS by `global_load_lds_dwordx4` (16 B per lane, no VGPR
//    round trip).  The LDS image is lane-linear (128-byte rows of 64 k), so
//    the bank-conflict swizzle is applied to the per-lane SOURCE address:
//    16-byte chunk c of row r holds logical k-chunk c ^ ((r >> 1) & 7), which
//    makes every 16-lane ds_read_b128 group of a fragment read hit 16
//    distinct bank slots;
//  * wave tile 128 (M) x 64 (N): 8 x 4 accumulators of
//    v_mfma_f32_16x16x32_bf16 with W as the A operand and X as the B
//    operand, so each lane ends up with 4 consecutive output COLUMNS of one
//    row (8-byte stores) — and, for SwiGLU, with the gate and up values of
//    the same column in the same lane and register;
//  * one barrier per K step (behind an explicit vmcnt(0): hipcc does not wait
//    for global_load_lds before a barrier on its own): fragments of k-half 1 are read while the
//    MFMAs of k-half 0 run, the barrier retires the next stage's loads and
//    everyone's reads of the current stage, then the stage after next is
//    issued into the stage just consumed while k-half 1's MFMAs run;
//  * XCD-aware tile order: blocks that share an XCD (b % 8) take a
//    contiguous run of tiles, M-fastest, so the 8 row tiles that reuse one
//    W tile run side by side on one L2.
//
// Requirements (checked by the host): N % 256 == 0 (epi 1: I % 128 == 0),
// K % 64 == 0, ldx % 8 == 0, ldy % 4 == 0.  Any M: rows past M are clamped
// on load and skipped on store.
#include "common.h"

#include <type_traits>

using namespace dgi;

namespace {

constexpr int kBM = 256;
constexpr int kBK = 64;
constexpr int kTileBytes = kBM * kBK * 2;      // 32 KB: one operand, one stage
constexpr int kStageBytes = 2 * kTileBytes;    // X tile + W tile

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

__device__ __forceinline__ void glds16(const uint16_t* src, char* lds) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds, 16, 0, 0);
}

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

// Lane holds rows m0 + 128 wm + 16 i + (lane & 15), columns 4 (lane >> 4) + 0..3 of each 16x16 tile.
// Two neighbouring tiles (A, B) are stored as ONE 16-byte store per lane: v_permlane16_swap
// trades A's columns of the odd 16-lane rows for B's columns of the even rows, so lane group
// g ends up with 8 consecutive columns — A 0-7 (g 0), B 0-7 (g 1), A 8-15 (g 2), B 8-15 (g 3) —
// and every row of a store instruction writes 64 contiguous bytes (half the store
// instructions of 8-byte stores; the store tail of a tile's epilogue is issue-bound).
__device__ __forceinline__ void store_pair16(uint16_t* yrow, int n0, int g, const float (&a)[4], const float (&b)[4]) {
  const uint32_t a01 = pack_bf16x2(a[0], a[1]), a23 = pack_bf16x2(a[2], a[3]);
  const uint32_t b01 = pack_bf16x2(b[0], b[1]), b23 = pack_bf16x2(b[2], b[3]);
  const auto s0 = __builtin_amdgcn_permlane16_swap(a01, b01, false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(a23, b23, false, false);
  uint4 v;
  v.x = s0[0];
  v.y = s1[0];
  v.z = s0[1];
  v.w = s1[1];
  *(uint4*)(yrow + n0 + 16 * (g & 1) + 4 * (g & 2)) = v;
}

// Epilogue kinds of the ping-pong kernel (the other schedules take 0 and 1):
//   0 plain store;  1 SwiGLU over [gate; up];
//   2 residual:  Y <- Y + acc in place (Y is the residual stream), and the tile's per-row sum of
//     squares of the new bf16 values to ss[m * ss_ld + tn] — the partial RMS statistics of the
//     next RMSNorm, reduced in a fixed order (deterministic, no atomics);
//   3 / 4 normalised plain / SwiGLU:  acc scaled per row by rstd[m] = rsqrt(sum_j ss[m, j] / K + eps)
//     before the store / activation.  With the RMSNorm gain folded into the weights
//     (W' = W * diag(gamma), LlamaModel.fold_norms) this is rmsnorm(x) * gamma @ W^T without
//     the normalised copy of x: the norm kernels between the projections disappear.
//   5 normalised qkv with the RoPE + paged-KV epilogue: the rstd-scaled tile is rounded to bf16
//     into LDS, then q heads are rotated (NeoX pairs d, d + 64 of each 128-dim head) in place in Y
//     and k (rotated) / v heads go straight to the paged cache at each row's slot — the separate
//     rope_cache kernel and its read-back of the qkv tensor disappear (k / v columns of Y are not
//     written: attention reads them from the cache).
template <int EPI>
struct EpiKind {
  static constexpr bool swiglu = EPI == 1 || EPI == 4;
  static constexpr bool norm = EPI == 3 || EPI == 4 || EPI == 5;
  static constexpr bool res = EPI == 2;
  static constexpr bool rope = EPI == 5;
};

constexpr int kRopeLd = 264;                    // LDS row stride (elements) of the RoPE tile image
constexpr int kRopeBytes = 256 * kRopeLd * 2;   // 135,168: the staging stages plus 4 KB

// store_pair16's column exchange on fp32 values: f[0..7] are the lane's 8 consecutive columns
// (A 0-7 for lane group 0, B 0-7 for 1, A 8-15 for 2, B 8-15 for 3) starting at
// n0 + 16 (g & 1) + 4 (g & 2)
__device__ __forceinline__ void swap_pair(const float (&a)[4], const float (&b)[4], float (&f)[8]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[e]), __float_as_uint(b[e]), false, false);
    f[e] = __uint_as_float(s[0]);
    f[4 + e] = __uint_as_float(s[1]);
  }
}

// rs: the tile's 256 per-row rstd values (LDS) for EPI 3 / 4
template <int EPI>
__device__ __forceinline__ void epilogue(const f32x4 (&acc)[8][4], uint16_t* __restrict__ Y, int ldy, int M, int m0,
                                         int tn, int wm, int wn, int lane, const float* rs = nullptr) {
  const int r16 = lane & 15;
  const int g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + r16;
    // the swap partners (lanes l, l ^ 16) hold the same row, so a row past M drops both together
    if (m >= M) continue;
    uint16_t* yrow = Y + (size_t)m * ldy;
    float sc = 1.f;
    if constexpr (EpiKind<EPI>::norm) sc = rs[wm * 128 + i * 16 + r16];
    if constexpr (EpiKind<EPI>::swiglu) {
      float o[2][4];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f32x4 gt = acc[i][j], u = acc[i][j + 2];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if constexpr (EpiKind<EPI>::norm)
            o[j][e] = silu(gt[e] * sc) * (u[e] * sc);
          else
            o[j][e] = silu(gt[e]) * u[e];
        }
      }
      store_pair16(yrow, tn * 128 + wn * 32, g, o[0], o[1]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        float x0[4], x1[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          x0[e] = acc[i][j][e] * sc;
          x1[e] = acc[i][j + 1][e] * sc;
        }
        store_pair16(yrow, tn * 256 + wn * 64 + j * 16, g, x0, x1);
      }
    }
  }
}

// EPI 2: Y <- bf16(Y + acc) and ss[m * ss_ld + tn] = sum over the tile's 256 columns of the new
// values squared.  Per row: each lane sums its 16 columns, the 4 lane groups of a wave combine by
// shuffles, the 4 waves of a row band through LDS (ssl: 4 x 256 floats), in a fixed order.
// Every wave of the block must call it (one barrier).
__device__ __forceinline__ void epilogue_res(const f32x4 (&acc)[8][4], uint16_t* __restrict__ Y, int ldy, int M,
                                             int m0, int tn, int wm, int wn, int lane, float* ssl,
                                             float* __restrict__ ss, int ss_ld) {
  const int r16 = lane & 15;
  const int g = lane >> 4;
  const int cbase = tn * 256 + wn * 64 + 16 * (g & 1) + 4 * (g & 2);
  // rows in batches of 4: the batch's 8 residual loads are all issued before the first is used
  // (a load-use per 16-byte chunk would serialise 16 memory round trips per lane)
#pragma unroll
  for (int i0 = 0; i0 < 8; i0 += 4) {
    uint4 old[4][2];
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int m = m0 + wm * 128 + (i0 + ii) * 16 + r16;
      const uint16_t* yrow = Y + (size_t)min(m, M - 1) * ldy + cbase;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) old[ii][jj] = *(const uint4*)(yrow + jj * 32);
    }
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int i = i0 + ii;
      const int m = m0 + wm * 128 + i * 16 + r16;
      float part = 0.f;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int j = 2 * jj;
        float x0[4], x1[4], f[8], o[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          x0[e] = acc[i][j][e];
          x1[e] = acc[i][j + 1][e];
        }
        swap_pair(x0, x1, f);
        const u32x4 ov = {old[ii][jj].x, old[ii][jj].y, old[ii][jj].z, old[ii][jj].w};
        unpack8(ov, o);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += f[e];
        const u32x4 nv = pack8(o);
        if (m < M) *(uint4*)(Y + (size_t)m * ldy + cbase + jj * 32) = uint4{nv[0], nv[1], nv[2], nv[3]};
        float r[8];
        unpack8(nv, r);               // the rounded values the next norm reads
#pragma unroll
        for (int e = 0; e < 8; ++e) part += r[e] * r[e];
      }
      part += __shfl_xor(part, 16, 64);
      part += __shfl_xor(part, 32, 64);
      if (g == 0) ssl[wn * 256 + wm * 128 + i * 16 + r16] = part;
    }
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t < 256 && m0 + t < M)
    ss[(size_t)(m0 + t) * ss_ld + tn] = ((ssl[t] + ssl[256 + t]) + ssl[512 + t]) + ssl[768 + t];
}

template <int EPI, int SCHED>
__global__ __launch_bounds__(512) void mfma_gemm_kernel(const uint16_t* __restrict__ X, int ldx,
                                                         const uint16_t* __restrict__ W,
                                                         uint16_t* __restrict__ Y, int ldy, int M, int I, int K,
                                                         int tiles_m, int tiles_total) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kStageBytes];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;

  // XCD-aware, bijective block -> tile map (blocks b and b + 8 share an XCD)
  const int b = blockIdx.x;
  const int xcd = b & 7, li = b >> 3;
  const int q8 = tiles_total >> 3, r8 = tiles_total & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + li;
  const int tm = t % tiles_m, tn = t / tiles_m;
  const int m0 = tm * kBM;

  // ---- staging map: lane-linear LDS image, swizzled global source
  const int q = tid >> 3;                         // row within each 64-row slab
  const int lc = (tid & 7) ^ ((tid >> 4) & 7);    // logical k-chunk this lane fetches
  const int xq = m0 + q;                          // rows xq + 64 i (clamped to M - 1 at issue)
  const uint16_t* const xsrc = X + lc * 8;
  // W rows: epi 0 -> n0 + 64 i + q; epi 1 -> slab i = wave column i: 32 gate rows then the
  // matching 32 up rows, so accumulator columns 0-1 (gate) pair with 2-3 (up) in one wave
  int wrow0, wstep;
  if (EPI == 1) {
    wrow0 = tn * 128 + (q < 32 ? q : I + q - 32);
    wstep = 32;
  } else {
    wrow0 = tn * 256 + q;
    wstep = 64;
  }
  const uint16_t* wsrc = W + (size_t)wrow0 * K + lc * 8;
  const size_t wslab = (size_t)wstep * K;
  char* const lds_x = smem + w * 1024;               // + stage * kStageBytes + i * 8 KB
  char* const lds_w = smem + kTileBytes + w * 1024;

  auto issue = [&](int kt, int stage) {
    const int k0 = kt * kBK;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds16(xsrc + min(xq + i * 64, M - 1) * ldx + k0, lds_x + stage * kStageBytes + i * 8192);
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(wsrc + i * wslab + k0, lds_w + stage * kStageBytes + i * 8192);
  };

  // ---- fragment read map (bytes inside one operand tile)
  const int r16 = lane & 15;
  const int sw = (lane >> 1) & 7;
  const int ph0 = ((lane >> 4) ^ sw) * 16;           // k-half 0: chunks 0-3
  const int ph1 = ((4 + (lane >> 4)) ^ sw) * 16;     // k-half 1: chunks 4-7
  const int xbase = (wm * 128 + r16) * 128;
  const int wbase = kTileBytes + (wn * 64 + r16) * 128;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 xa[8], wa[4], xb[8], wb[4];
  auto read = [&](int stage, int ph, bf16x8* xf, bf16x8* wf) {
    const char* s = smem + stage * kStageBytes;
#pragma unroll
    for (int j = 0; j < 4; ++j) wf[j] = *(const bf16x8*)(s + wbase + j * 2048 + ph);
#pragma unroll
    for (int i = 0; i < 8; ++i) xf[i] = *(const bf16x8*)(s + xbase + i * 2048 + ph);
  };
  auto mma = [&](const bf16x8* xf, const bf16x8* wf) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
  };

  const int nt = K / kBK;
  issue(0, 0);
  if (nt > 1) issue(1, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  read(0, ph0, xa, wa);
  if (SCHED == 0) {
    for (int kt = 0; kt < nt; ++kt) {
      const int st = kt & 1;
      read(st, ph1, xb, wb);
      __builtin_amdgcn_s_setprio(1);
      mma(xa, wa);
      __builtin_amdgcn_s_setprio(0);
      // next stage landed: hipcc does not count global_load_lds as an LDS write
      // before a barrier, so the wave's own loads are retired explicitly
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();        // every wave's loads landed; every wave done reading this stage
      if (kt + 2 < nt) issue(kt + 2, st);
      if (kt + 1 < nt) read(st ^ 1, ph0, xa, wa);
      __builtin_amdgcn_s_setprio(1);
      mma(xb, wb);
      __builtin_amdgcn_s_setprio(0);
    }
  } else {
    // Same schedule with the memory instructions spread between the MFMAs
    // (sched_group_barrier): k-half 1's 12 fragment reads ride 2 MFMAs each,
    // and after the barrier every global_load_lds and k-half 0 fragment read
    // of the next step is paired with MFMAs instead of issuing as one burst.
    // The loop is peeled so each body is one scheduling region (no s_setprio
    // inside: it would split the region and pin the bursts in place).
    auto body = [&](int kt, auto issue_next, auto read_next) {
      const int st = kt & 1;
      read(st, ph1, xb, wb);
      mma(xa, wa);
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (decltype(issue_next)::value) issue(kt + 2, st);
      if constexpr (decltype(read_next)::value) read(st ^ 1, ph0, xa, wa);
      mma(xb, wb);
      if constexpr (decltype(issue_next)::value) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 1);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 1);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 1);
      } else if constexpr (decltype(read_next)::value) {
#pragma unroll
        for (int i = 0; i < 12; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 1);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 1);
      }
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    int kt = 0;
    for (; kt + 2 < nt; ++kt) body(kt, T_{}, T_{});
    if (kt + 1 < nt) body(kt++, F_{}, T_{});
    body(kt, F_{}, F_{});
  }

  epilogue<EPI>(acc, Y, ldy, M, m0, tn, wm, wn, lane);
}


// ---------------------------------------------------------------------------
// Half tile (sched 4, epi 0): a 128 x 128 output tile on 4 waves (2 x 2 of 64 x 64), the same
// lane-linear LDS image, source-side swizzle and fragment map as mfma_gemm_kernel, two 32 KB
// stages (two workgroups per CU).  For row counts whose 256 x 256 tiles fill a fraction of the
// chip — the decode role's qkv / o at 512 rows: 80 / 64 tiles on 256 CUs, where the full tile
// needs a split-K round trip (0.84 PF/s) and hipBLASLt reaches 0.86-0.90 — the half tile gives
// 320 / 256 whole tiles (profiles/r5_pd/README.md §10).
constexpr int kHM = 128;
constexpr int kHTile = kHM * kBK * 2;     // 16 KB: one operand, one stage
constexpr int kHStage = 2 * kHTile;       // X tile + W tile

__global__ __launch_bounds__(256) void mfma_gemm_half_kernel(const uint16_t* __restrict__ X, int ldx,
                                                             const uint16_t* __restrict__ W,
                                                             uint16_t* __restrict__ Y, int ldy, int M, int K,
                                                             int tiles_m, int tiles_total) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kHStage];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;

  // XCD-aware, bijective block -> tile map (blocks b and b + 8 share an XCD), M-fastest
  const int b = blockIdx.x;
  const int xcd = b & 7, li = b >> 3;
  const int q8 = tiles_total >> 3, r8 = tiles_total & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + li;
  const int tm = t % tiles_m, tn = t / tiles_m;
  const int m0 = tm * kHM;

  // staging: pass i moves rows 32 i .. 32 i + 31 of each operand (one 1 KB wave-instruction per
  // 8 rows); physical 16-byte chunk c of row r holds logical k-chunk c ^ ((r >> 1) & 7)
  const int q = tid >> 3;
  const int lc = (tid & 7) ^ ((tid >> 4) & 7);
  const int xq = m0 + q;
  const uint16_t* const xsrc = X + lc * 8;
  const uint16_t* const wsrc = W + (size_t)(tn * kHM + q) * K + lc * 8;
  const size_t wslab = (size_t)32 * K;
  char* const lds_x = smem + w * 1024;
  char* const lds_w = smem + kHTile + w * 1024;

  auto issue = [&](int kt, int stage) {
    const int k0 = kt * kBK;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds16(xsrc + (size_t)min(xq + i * 32, M - 1) * ldx + k0, lds_x + stage * kHStage + i * 4096);
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(wsrc + i * wslab + k0, lds_w + stage * kHStage + i * 4096);
  };

  const int r16 = lane & 15;
  const int sw = (lane >> 1) & 7;
  const int ph0 = ((lane >> 4) ^ sw) * 16;
  const int ph1 = ((4 + (lane >> 4)) ^ sw) * 16;
  const int xbase = (wm * 64 + r16) * 128;
  const int wbase = kHTile + (wn * 64 + r16) * 128;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 xa[4], wa[4], xb[4], wb[4];
  auto read = [&](int stage, int ph, bf16x8* xf, bf16x8* wf) {
    const char* sp = smem + stage * kHStage;
#pragma unroll
    for (int j = 0; j < 4; ++j) wf[j] = *(const bf16x8*)(sp + wbase + j * 2048 + ph);
#pragma unroll
    for (int i = 0; i < 4; ++i) xf[i] = *(const bf16x8*)(sp + xbase + i * 2048 + ph);
  };
  auto mma = [&](const bf16x8* xf, const bf16x8* wf) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
  };

  const int nt = K / kBK;
  issue(0, 0);
  if (nt > 1) issue(1, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  read(0, ph0, xa, wa);
  for (int kt = 0; kt < nt; ++kt) {
    const int st = kt & 1;
    read(st, ph1, xb, wb);
    mma(xa, wa);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's next-stage loads landed
    __syncthreads();                                    // everyone's landed; stage st fully read
    if (kt + 2 < nt) issue(kt + 2, st);
    if (kt + 1 < nt) read(st ^ 1, ph0, xa, wa);
    mma(xb, wb);
  }

  const int g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + r16;
    if (m >= M) continue;
    uint16_t* yrow = Y + (size_t)m * ldy;
#pragma unroll
    for (int j = 0; j < 4; j += 2) {
      float x0[4], x1[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x0[e] = acc[i][j][e];
        x1[e] = acc[i][j + 1][e];
      }
      store_pair16(yrow, tn * kHM + wn * 64 + j * 16, g, x0, x1);
    }
  }
}

// ---------------------------------------------------------------------------
// Ring schedule (sched 2): the K loop advances in 32-deep sub-steps through a
// ring of four 32 KB LDS slots (X 256 x 32 and W 256 x 32, 64-byte rows).
// Sub-step u computes on fragments of u already in registers, reads u + 1's
// fragments, and refills the slot u itself came from with u + 4 — so three
// sub-steps of loads stay in flight across every barrier (counted
// s_waitcnt vmcnt(8), never 0 in the steady state, raw s_barrier) and each
// sub-step's 4 global_load_lds, 12 ds_read_b128 and 32 MFMAs are issued
// interleaved.  64-byte rows: chunk c of row r holds k-chunk c ^ f((r >> 2) & 3)
// with f = {0, 2, 3, 1}, conflict-free for the ds_read_b128 lane groups.
template <int EPI>
__global__ __launch_bounds__(512) void mfma_gemm_ring_kernel(const uint16_t* __restrict__ X, int ldx,
                                                              const uint16_t* __restrict__ W,
                                                              uint16_t* __restrict__ Y, int ldy, int M, int I,
                                                              int K, int tiles_m, int tiles_total) {
  constexpr int kSlot = 32768;        // X 16 KB + W 16 KB
  constexpr int kHalf = 16384;
  __shared__ __attribute__((aligned(16))) char smem[4 * kSlot];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;

  const int b = blockIdx.x;
  const int xcd = b & 7, li = b >> 3;
  const int q8 = tiles_total >> 3, r8 = tiles_total & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + li;
  const int tm = t % tiles_m, tn = t / tiles_m;
  const int m0 = tm * kBM;

  // staging: instruction i covers tile rows 128 i + (tid >> 2), 16-byte chunk tid & 3
  const int rq = tid >> 2;
  const int quad = (tid >> 4) & 3;
  const int lc = (tid & 3) ^ ((0x1320 >> (quad * 4)) & 3);
  const int xq = m0 + rq;
  const uint16_t* const xsrc = X + lc * 8;
  int wrow0, wstep;
  if (EPI == 1) {            // tile row r -> wave column r >> 6; 32 gate rows then the 32 matching up rows
    const int qq = rq & 63;
    wrow0 = tn * 128 + (rq >> 6) * 32 + (qq < 32 ? qq : I + qq - 32);
    wstep = 64;              // +128 tile rows = +2 wave columns = +64 weight rows
  } else {
    wrow0 = tn * 256 + rq;
    wstep = 128;
  }
  const uint16_t* const wsrc = W + (size_t)wrow0 * K + lc * 8;
  const size_t wslab = (size_t)wstep * K;
  char* const lds_x = smem + w * 1024;
  char* const lds_w = smem + kHalf + w * 1024;

  auto issue = [&](int u) {
    const int k0 = u * 32;
    const int slot = (u & 3) * kSlot;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      glds16(xsrc + min(xq + i * 128, M - 1) * ldx + k0, lds_x + slot + i * 8192);
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(wsrc + i * wslab + k0, lds_w + slot + i * 8192);
  };

  const int r16 = lane & 15;
  const int ph = ((lane >> 4) ^ ((0x1320 >> (((lane >> 2) & 3) * 4)) & 3)) * 16;
  const int xbase = (wm * 128 + r16) * 64 + ph;
  const int wbase = kHalf + (wn * 64 + r16) * 64 + ph;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 xa[8], wa[4], xb[8], wb[4];
  auto read = [&](int u, bf16x8* xf, bf16x8* wf) {
    const char* s = smem + (u & 3) * kSlot;
#pragma unroll
    for (int j = 0; j < 4; ++j) wf[j] = *(const bf16x8*)(s + wbase + j * 1024);
#pragma unroll
    for (int i = 0; i < 8; ++i) xf[i] = *(const bf16x8*)(s + xbase + i * 1024);
  };
  auto mma = [&](const bf16x8* xf, const bf16x8* wf) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
  };
  // steady-state sub-step (u + 4 < nu): compute on (xc, wc) = fragments of u, read u + 1 into
  // (xn, wn_), refill slot u with u + 4 — branch-free, so the interleave below is one region
  auto steady = [&](int u, bf16x8* xc, bf16x8* wc, bf16x8* xn, bf16x8* wn_) {
    // the refill goes first: each global_load_lds rewrites M0, and hipcc waits for every
    // outstanding LDS op before an M0 write, so issued behind the fragment reads it would
    // serialise them
    issue(u + 4);
    read(u + 1, xn, wn_);
    mma(xc, wc);
    __builtin_amdgcn_sched_group_barrier(0x020, 4, 0);
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // slot u + 2 landed; u + 3, u + 4 in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // the last (up to 4) sub-steps: no refills, the in-flight slots drain
  auto tail = [&](int u, int nu, bf16x8* xc, bf16x8* wc, bf16x8* xn, bf16x8* wn_) {
    if (u + 1 < nu) read(u + 1, xn, wn_);
    mma(xc, wc);
    __builtin_amdgcn_sched_barrier(0);
    if (u + 3 < nu)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  const int nu = K / 32;
  for (int u = 0; u < 4 && u < nu; ++u) issue(u);
  // slots 0 and 1 landed (2 and 3 may still be in flight)
  if (nu >= 4)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  read(0, xa, wa);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();          // every wave holds slot 0 in registers: it may be refilled
  __builtin_amdgcn_sched_barrier(0);
  // nu is even (K % 64 == 0): steady pairs while both sub-steps refill, then drain in pairs
  int u = 0;
  for (; u + 5 < nu; u += 2) {
    steady(u, xa, wa, xb, wb);
    steady(u + 1, xb, wb, xa, wa);
  }
  for (; u < nu; u += 2) {
    tail(u, nu, xa, wa, xb, wb);
    tail(u + 1, nu, xb, wb, xa, wa);
  }
  epilogue<EPI>(acc, Y, ldy, M, m0, tn, wm, wn, lane);
}

// ---------------------------------------------------------------------------
// Ping-pong schedule (sched 3).  Same tile, LDS image and fragment map as the
// kernel above, but each K tile runs as 4 phases of 16 MFMAs per wave and the two
// wave groups of a SIMD (waves 0-3: rows 0-127, waves 4-7: rows 128-255) are
// staggered by one barrier: while one wave of a SIMD issues its fragment reads
// and staging loads ("R" section), its partner runs its MFMAs ("M" section),
// and every section ends at a raw s_barrier.  The phases of tile t, per wave
// (Xa / Xb = first / second 64 of the wave's 128 X rows, Wa / Wb = first /
// second 32 of its 64 W rows):
//
//   phase  reads        MFMAs      staging (slab = 64 rows x 64 k, one glds)   wait before the barrier
//   0      Xa, Wa (12)  Xa x Wa    W2, W3 of t+1
//   1      Wb (4)       Xa x Wb    X3 of t+1, X0 of t+2                      vmcnt(7): X1, X3 of t landed
//   2      Xb (8)       Xb x Wb    X1 of t+1, X2 of t+2
//   3      -            Xb x Wa    W0, W1 of t+2                             vmcnt(6): all but X1, X3 of t+1
//
// Every slab is refilled at least two sections after the last read of the
// slab it replaces (WAR; each wave retires its reads with lgkmcnt(0) at the
// top of the following M section) and waited for by every wave before the
// barrier that precedes its first read (RAW): staging loads stay 3-6 phases in
// flight and vmcnt never drains to 0 in the steady state.  The last two tiles
// issue less and wait with smaller counts (MODE 1, 2).  A work item is any even
// number (>= 2) of K tiles of one output tile.
//
// Work decomposition.  When the output tiles are a multiple of the CU count
// (or many waves of it) every block owns whole tiles (grid = tiles).  Otherwise
// the launch is persistent (grid = P blocks, P = CUs) and hybrid split-K: the
// first `rem` = tiles % P tiles are cut along K into `splits` (2-4) pieces of
// 128-deep units, piece j of tile t going to block g = j * rem + t, so the
// blocks of one XCD (consecutive g) work on neighbouring tiles over the SAME K
// range and share their X / W slabs in L2 (a stream-K split, whose pieces start
// at staggered K offsets, measured slower for that reason); every block then
// owns `full` whole tiles.  A piece that finishes its K range takes an arrival
// ticket (one relaxed counter add).  Every piece but the last to arrive stores its
// fp32 partial tile to its block's workspace slab with write-through (sc1) stores and
// publishes it (every wave drains its stores, then a relaxed add on the tile's
// "written" counter; no release fence, which would write back the whole L2).  The
// last piece waits until the others' slabs are written, acquires, folds every
// piece's partial in piece order (s_0 + s_1 + ..: deterministic whichever piece
// arrived last), writes the bf16 tile and resets both counters for the next launch.
// Pieces 0 and 1 keep their own partial in registers (s_0 + s_1 == s_1 + s_0 in
// IEEE arithmetic, so it enters the fold at its place); a later piece stores its
// slab too (a prefix register set spills).  The wait cannot deadlock for any block placement or dispatch
// order: every piece it waits for has already taken its ticket, so it is resident
// and has only its slab store left.  The wait is bounded (a broken counter ends as
// a wrong tile, not a hung GPU).  This saves the last piece's slab store and one slab
// read on the tile's critical path (pp_split_probe: the split-K round trip cost
// ~30 us per GEMM at the decode role's 512 rows).
struct PPArgs {
  const uint16_t* X;
  const uint16_t* W;
  uint16_t* Y;
  float* ws;     // one 256 x 256 fp32 slab per block (hybrid launches)
  int* cnt;      // per split tile: arrivals at [t], slabs written at [P + t]; zero between launches
  int ldx, ldy, M, I, K, tiles_m, tiles_total;
  int rem, splits, full, P;   // P == 0: one tile per block (grid = tiles)
  int ovl;                    // issue the next tile's prologue before the current epilogue
  float* ss;                  // EPI 2: per-row partial sums of squares out; EPI 3 / 4: in
  int ss_ld;                  // row stride of ss (EPI 2: its column is the N tile; EPI 3 / 4: partials per row)
  float inv_k, eps;           // EPI 3 / 4: rstd = rsqrt(sum * inv_k + eps)
  // EPI 5: RoPE table [positions, 128] (64 cos | 64 sin), per-row positions / cache slots, caches
  // [blocks, nkv, bs, 128], q / kv column counts
  const int* pos;
  const float* cs;
  const int* slots;
  uint16_t* kc;
  uint16_t* vc;
  int qcols, kvcols, nkv, bs;
};

// EPI 5 (see EpiKind): T is the LDS tile image (256 rows x kRopeLd), rs the tile's rstd.  Every wave
// of the block calls it (two barriers).
__device__ __forceinline__ void epilogue_rope(const f32x4 (&acc)[8][4], const PPArgs& a, int m0, int tn, int wm,
                                              int wn, int lane, const float* rs, uint16_t* T) {
  const int r16 = lane & 15;
  const int g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int rl = wm * 128 + i * 16 + r16;
    const float sc = rs[rl];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint2 v;
      v.x = pack_bf16x2(acc[i][j][0] * sc, acc[i][j][1] * sc);
      v.y = pack_bf16x2(acc[i][j][2] * sc, acc[i][j][3] * sc);
      *(uint2*)(T + rl * kRopeLd + wn * 64 + j * 16 + 4 * g) = v;
    }
  }
  __syncthreads();
  const int t = threadIdx.x;
  const int rl = t >> 1, half = t & 1;      // two lanes per row, 32 of the 64 pairs of each head
  const int m = m0 + rl;
  const int col0 = tn * 256;
  const int kind = col0 < a.qcols ? 0 : col0 < a.qcols + a.kvcols ? 1 : 2;    // q, k or v heads
  const int slot = (m < a.M && kind) ? a.slots[m] : 0;
  if (m < a.M && slot >= 0) {
    const int blk = kind ? slot / a.bs : 0;
    const int off = kind ? slot - blk * a.bs : 0;
    const float* cs = a.cs + (size_t)a.pos[m] * 128;
    const int head0 = kind == 1 ? (col0 - a.qcols) >> 7 : (col0 - a.qcols - a.kvcols) >> 7;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int d = half * 32 + c * 8;
      float cv[8], sv[8];
      if (kind != 2) {
        *(float4*)cv = *(const float4*)(cs + d);
        *(float4*)(cv + 4) = *(const float4*)(cs + d + 4);
        *(float4*)sv = *(const float4*)(cs + 64 + d);
        *(float4*)(sv + 4) = *(const float4*)(cs + 64 + d + 4);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint16_t* tp = T + rl * kRopeLd + h * 128 + d;
        const u32x4 p0 = *(const u32x4*)tp, p1 = *(const u32x4*)(tp + 64);
        u32x4 o0 = p0, o1 = p1;
        if (kind != 2) {
          float x0[8], x1[8], y0[8], y1[8];
          unpack8(p0, x0);
          unpack8(p1, x1);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            y0[e] = x0[e] * cv[e] - x1[e] * sv[e];
            y1[e] = x1[e] * cv[e] + x0[e] * sv[e];
          }
          o0 = pack8(y0);
          o1 = pack8(y1);
        }
        uint16_t* dst;
        if (kind == 0)
          dst = a.Y + (size_t)m * a.ldy + col0 + h * 128 + d;
        else
          dst = (kind == 1 ? a.kc : a.vc) + (((size_t)blk * a.nkv + head0 + h) * a.bs + off) * 128 + d;
        *(u32x4*)dst = o0;
        *(u32x4*)(dst + 64) = o1;
      }
    }
  }
  __syncthreads();   // the image is read before the next work item's staging rewrites LDS
}

// buffer resource word 3 of a raw (stride 0, byte-addressed) buffer on gfx9, and the cache
// policy bit of a write-through (sc1) access
constexpr int kRsrcWord3 = 0x00020000;
constexpr int kSc1 = 16;

// The work items of one block (see "Work decomposition" above): its one tile
// (P == 0), its split-K piece, then its whole tiles.  prologue(tm, tn, kb) issues the
// staging loads of output tile (tm, tn) from K tile kb on, body(tm, tn, kb, L, ov) accumulates
// L K tiles into the caller's registers; slab_store(store16) moves them to a 256 x 256 fp32 slab
// through store16(e, v) (16-byte element e of this thread; NT threads interleaved by 16 bytes),
// slab_sum(load16, own, n) folds the n pieces' slabs (load16(piece, e)) in piece order into them,
// they being piece own; epi stores the bf16 tile.  With a.ovl,
// the next whole tile's prologue is issued before the current whole tile's epilogue
// (which does not touch LDS: the body ends with every LDS read retired), so its first
// K tiles load while the stores drain.
template <int NT, class Pro, class Body, class Store, class Sum, class Epi>
__device__ __forceinline__ void drive(const PPArgs& a, char* smem, Pro&& prologue, Body&& body, Store&& slab_store,
                                      Sum&& slab_sum, Epi&& epi) {
  const int tid = threadIdx.x;
  const int nt = a.K / kBK;
  const int nt2 = nt >> 1;                    // 128-deep units per tile
  // persistent hybrid: block g (blocks that share an XCD take consecutive g)
  const int g = (blockIdx.x & 7) * (a.P >> 3) + (blockIdx.x >> 3);
  bool split = a.rem && g < a.rem * a.splits;
  int k = 0;
  // next work item: tile t, K tiles kb .. kb + L - 1; t < 0 when the block is done
  struct Item {
    int t, kb, L;
    bool piece;
  };
  auto next = [&]() -> Item {
    if (a.P == 0) {
      if (k++) return Item{-1, 0, 0, false};
      const int b = blockIdx.x, T = a.tiles_total;
      const int xcd = b & 7, li = b >> 3;
      const int q8 = T >> 3, r8 = T & 7;
      return Item{(xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + li, 0, nt, false};
    }
    if (split) {
      split = false;
      const int j = g / a.rem;
      const int u0 = j * nt2 / a.splits, u1 = (j + 1) * nt2 / a.splits;
      return Item{g - j * a.rem, 2 * u0, 2 * (u1 - u0), true};
    }
    if (k < a.full) return Item{a.rem + (k++) * a.P + g, 0, nt, false};
    return Item{-1, 0, 0, false};
  };
  Item cur = next();
  if (cur.t < 0) return;
  prologue(cur.t % a.tiles_m, cur.t / a.tiles_m, cur.kb);
  bool ov = false;
  for (;;) {
    const int tm = cur.t % a.tiles_m, tn = cur.t / a.tiles_m;
    body(tm, tn, cur.kb, cur.L, ov);
    const Item nx = next();
    // overlap only between whole tiles whose epilogue stores every row (fixed store count)
    ov = a.ovl && nx.t >= 0 && !cur.piece && !nx.piece && (tm + 1) * kBM <= a.M;
    if (ov) prologue(nx.t % a.tiles_m, nx.t / a.tiles_m, nx.kb);
    bool store = true;
    if (cur.piece) {
      const int t = cur.t;
      const int own = g / a.rem;                // this block's piece of tile t
      // slab offsets from a laundered thread id: otherwise hipcc hoists every per-lane
      // address out of the work-item loop and spills them
      int lt = tid;
      asm volatile("" : "+v"(lt));
      const int lo = lt * 16;
      if (tid == 0) {
        const int old = __hip_atomic_fetch_add(a.cnt + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *(volatile int*)smem = old == a.splits - 1;
      }
      __syncthreads();
      store = *(volatile int*)smem;
      __syncthreads();          // flag read by every wave before the next item's staging overwrites it
      // every piece but the last stores its slab; so does a last piece past the second (its
      // registers cannot enter the fold without a prefix register set)
      if (!store || own >= 2) {
        // publish: write-through (sc1) 16-byte stores drained by every wave, then one relaxed
        // counter add — no release fence (an agent release writes back the whole L2)
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(a.ws + (size_t)g * 65536), 0, 65536 * 4, kRsrcWord3);
        slab_store([&](int e, const f32x4& v) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, e * NT * 16 + lo, 0, kSc1);
        });
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0 && !store)
          __hip_atomic_fetch_add(a.cnt + a.P + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (store) {
        if (tid == 0) {
          bool landed = false;
          for (int spin = 0; spin < (1 << 22) && !landed; ++spin) {
            landed = __hip_atomic_load(a.cnt + a.P + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= a.splits - 1;
            if (!landed) __builtin_amdgcn_s_sleep(2);
          }
          // a wait that ran out (a broken counter): counted in the workspace's error word, which
          // dgi_gemm_split_timeouts reads (DGI_DEBUG_SYNC checks it after every GEMM)
          if (!landed) __hip_atomic_fetch_add(a.cnt - 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_store(a.cnt + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.cnt + a.P + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        slab_sum([&](int jj, int e) {
          const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
              (void*)(a.ws + (size_t)(jj * a.rem + t) * 65536), 0, 65536 * 4, kRsrcWord3);
          return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rl, e * NT * 16 + lo, 0, 0));
        }, own >= 2 ? -1 : own, a.splits);
        // a real s_waitcnt (not inline asm) so that the waitcnt pass knows the accumulators are
        // written: otherwise it merges this path's pending loads into the epilogue as vmcnt(0)
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
      }
    }
    if (store) epi(tm, tn);
    if (nx.t < 0) break;
    if (!ov) prologue(nx.t % a.tiles_m, nx.t / a.tiles_m, nx.kb);
    cur = nx;
  }
}

// PRIO: 0 = s_setprio 1 around each MFMA cluster (keeps hipcc from moving MFMAs across the
// barriers; the instructions themselves are near free); 1 = static s_setprio 1 for waves 4-7
// (the second-dispatched half) and no per-cluster flips; 2 = no s_setprio.
// PH: phases per K tile, 4 (16 MFMAs per section, the table above) or 2 (32 MFMAs per
// section, half the barrier hand-offs):
//
//   phase  reads             MFMAs          staging                       wait before the barrier
//   0      Xa, Wa, Wb (16)   Xa x (Wa, Wb)  W0-3, X2 of t+1               vmcnt(6): X1, X3 of t landed
//   1      Xb (8)            Xb x (Wa, Wb)  X3, X1 of t+1, X0 of t+2      vmcnt(3): all but X3, X1 of t+1
template <int EPI, int PRIO, int PH>
__global__ __launch_bounds__(512) void mfma_gemm_pp_kernel(PPArgs a) {
  // EPI 2: per-wave row partials of the sum of squares; EPI 3 / 4: two slots of the tile's rstd
  // (slot per work item: a fast wave may start the next item while others still store this one).
  // Carved from the one LDS array: with a second __shared__ object hipcc's waitcnt pass can no
  // longer tell the staging DMA from other LDS traffic and waits vmcnt(0) before every fragment
  // read of the K loop (measured: the gate_up kernel 349 -> 517 us at 512 rows).
  constexpr int kEpBytes = EpiKind<EPI>::res ? 4096 : EpiKind<EPI>::norm ? 2048 : 0;
  constexpr int kMainBytes = EpiKind<EPI>::rope ? kRopeBytes : 2 * kStageBytes;
  __shared__ __attribute__((aligned(16))) char smem[kMainBytes + kEpBytes];
  float* const ep_lds = (float*)(smem + kMainBytes);
  int rs_slot = 0;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const int M = a.M, K = a.K, ldx = a.ldx;

  char* const lds_x = smem + w * 1024;
  char* const lds_w = smem + kTileBytes + w * 1024;
  const int r16 = lane & 15;
  const int sw = (lane >> 1) & 7;
  const int ph0 = ((lane >> 4) ^ sw) * 16;
  const int ph1 = ((4 + (lane >> 4)) ^ sw) * 16;
  const int xbase = (wm * 128 + r16) * 128;
  const int wbase = kTileBytes + (wn * 64 + r16) * 128;

  f32x4 acc[8][4];
  bf16x8 xa[4][2], xb[4][2], wa[2][2], wb[2][2];
  // x fragments of row tiles i0 .. i0 + 3, w fragments of row tiles j0, j0 + 1; both k halves
  auto rx = [&](int st, int i0, bf16x8 (&f)[4][2]) {
    const char* s = smem + st * kStageBytes + xbase + i0 * 2048;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[i][0] = *(const bf16x8*)(s + i * 2048 + ph0);
      f[i][1] = *(const bf16x8*)(s + i * 2048 + ph1);
    }
  };
  auto rw = [&](int st, int j0, bf16x8 (&f)[2][2]) {
    const char* s = smem + st * kStageBytes + wbase + j0 * 2048;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      f[j][0] = *(const bf16x8*)(s + j * 2048 + ph0);
      f[j][1] = *(const bf16x8*)(s + j * 2048 + ph1);
    }
  };
  auto mma = [&](int i0, int j0, const bf16x8 (&xf)[4][2], const bf16x8 (&wf)[2][2]) {
    if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][h], xf[i][h], acc[i0 + i][j0 + j], 0, 0, 0);
    if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(0);
  };
  if constexpr (PRIO == 1) {
    if (wm == 1) __builtin_amdgcn_s_setprio(1);
  }
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  // staging sources of the current work item (set by prologue)
  const uint16_t* xs[4];
  const uint16_t* wsrc = a.W;
  size_t wslab = 0;
  // slab i (rows 64 i .. 64 i + 63) of local K tile kt into LDS stage st
  auto gx = [&](int kt, int i, int st) { glds16(xs[i] + kt * kBK, lds_x + st * kStageBytes + i * 8192); };
  auto gw = [&](int kt, int i, int st) { glds16(wsrc + i * wslab + kt * kBK, lds_w + st * kStageBytes + i * 8192); };

  // the staging loads that precede K tile 0 of output tile (tm, tn), K tiles from kb on
  // (PH == 2: 9 loads, PH == 4: 12; the body retires the oldest 6 before its first read)
  // per-lane terms of the prologue and epilogue from a laundered thread id: hipcc would otherwise
  // keep them live across the K loop and spill them, and the reload's vmcnt(0) would drain the
  // next tile's staging loads before the epilogue
  auto fresh_tid = [&]() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
  };
  auto set_src = [&](int tm, int tn, int kb) {
    const int m0 = tm * kBM;
    const int tq = fresh_tid();
    const int q = tq >> 3, lc = (tq & 7) ^ ((tq >> 4) & 7);
#pragma unroll
    for (int i = 0; i < 4; ++i) xs[i] = a.X + (size_t)min(m0 + q + i * 64, M - 1) * ldx + lc * 8 + kb * kBK;
    int wrow0, wstep;
    if (EpiKind<EPI>::swiglu) {
      wrow0 = tn * 128 + (q < 32 ? q : a.I + q - 32);
      wstep = 32;
    } else {
      wrow0 = tn * 256 + q;
      wstep = 64;
    }
    wsrc = a.W + (size_t)wrow0 * K + lc * 8 + kb * kBK;
    wslab = (size_t)wstep * K;
  };
  auto prologue = [&](int tm, int tn, int kb) {
    set_src(tm, tn, kb);
    if constexpr (PH == 2) {
      gx(0, 0, 0); gw(0, 0, 0); gw(0, 1, 0); gw(0, 2, 0); gw(0, 3, 0); gx(0, 2, 0);
      gx(0, 3, 0); gx(0, 1, 0); gx(1, 0, 1);
    } else {
      gx(0, 0, 0); gx(0, 2, 0); gw(0, 0, 0); gw(0, 1, 0); gw(0, 2, 0); gw(0, 3, 0);
      gx(0, 3, 0); gx(1, 0, 1); gx(0, 1, 0); gx(1, 2, 1); gw(1, 0, 1); gw(1, 1, 1);
    }
  };

  // acc = X[tile rows] . W[tile cols]^T over K tiles kb .. kb + L - 1 (L even, >= 4) after
  // prologue(tm, tn, kb); the sources are recomputed here so that they are not live across an
  // overlapped epilogue (whose register pressure otherwise makes hipcc reuse store-data
  // registers, each reuse a vmcnt(0)).
  // ov: the previous tile's epilogue (8 16-byte stores per thread for EPI 1, 16 for EPI 0; all its rows inside M) was
  // issued between the prologue and this call, so the first wait counts those stores too
  // (vector memory operations retire in issue order)
  auto body = [&](int tm, int tn, int kb, int L, bool ov) {
    set_src(tm, tn, kb);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (EpiKind<EPI>::norm) {
      // the tile's row statistics: partial sums in a fixed order, rstd into this item's LDS slot
      // (visible to every wave by the K loop's barriers; the epilogue reads it)
      rs_slot ^= 1;
      const int t = fresh_tid();
      // two lanes per row, each summing half of its partials (float4 loads, all in flight
      // together: ss_ld % 8 == 0, <= 32), then one exchange — a fixed order on every run
      const int m = min(tm * kBM + (t >> 1), M - 1);
      const int per = a.ss_ld >> 3;
      const f32x4* sp = (const f32x4*)(a.ss + (size_t)m * a.ss_ld) + (t & 1) * per;
      f32x4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = j < per ? sp[j] : f32x4{0.f, 0.f, 0.f, 0.f};
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
      const float o2 = __shfl_xor(s, 1, 64);
      s = (t & 1) ? o2 + s : s + o2;
      if (!(t & 1)) ep_lds[rs_slot * 256 + (t >> 1)] = rsqrtf(s * a.inv_k + a.eps);
    }

    // one K tile; ST = its LDS stage, MODE 0: t + 2 < L, 1: t + 2 == L, 2: t + 1 == L
    auto tile = [&](int t, auto ST_, auto MODE_) {
      constexpr int ST = decltype(ST_)::value, MODE = decltype(MODE_)::value;
      // phase 0
      if constexpr (MODE < 2) { gw(t + 1, 2, ST ^ 1); gw(t + 1, 3, ST ^ 1); }
      rw(ST, 0, wa);
      rx(ST, 0, xa);
      barrier();
      mma(0, 0, xa, wa);
      barrier();
      // phase 1
      if constexpr (MODE < 2) gx(t + 1, 3, ST ^ 1);
      if constexpr (MODE == 0) gx(t + 2, 0, ST);
      rw(ST, 2, wb);
      if constexpr (MODE == 0) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      else if constexpr (MODE == 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      barrier();
      mma(0, 2, xa, wb);
      barrier();
      // phase 2
      if constexpr (MODE < 2) gx(t + 1, 1, ST ^ 1);
      if constexpr (MODE == 0) gx(t + 2, 2, ST);
      rx(ST, 4, xb);
      barrier();
      mma(4, 2, xb, wb);
      barrier();
      // phase 3
      if constexpr (MODE == 0) { gw(t + 2, 0, ST); gw(t + 2, 1, ST); }
      if constexpr (MODE == 0) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if constexpr (MODE == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      barrier();
      mma(4, 0, xb, wa);
      barrier();
    };

    // the same K tile in two phases of 32 MFMAs (PH == 2)
    auto tile2 = [&](int t, auto ST_, auto MODE_) {
      constexpr int ST = decltype(ST_)::value, MODE = decltype(MODE_)::value;
      // phase 0
      if constexpr (MODE < 2) {
        gw(t + 1, 0, ST ^ 1); gw(t + 1, 1, ST ^ 1); gw(t + 1, 2, ST ^ 1); gw(t + 1, 3, ST ^ 1);
        gx(t + 1, 2, ST ^ 1);
      }
      rw(ST, 0, wa);
      rw(ST, 2, wb);
      rx(ST, 0, xa);
      if constexpr (MODE < 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      barrier();
      mma(0, 0, xa, wa);
      mma(0, 2, xa, wb);
      barrier();
      // phase 1
      if constexpr (MODE < 2) { gx(t + 1, 3, ST ^ 1); gx(t + 1, 1, ST ^ 1); }
      if constexpr (MODE == 0) gx(t + 2, 0, ST);
      rx(ST, 4, xb);
      if constexpr (MODE == 0) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else if constexpr (MODE == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      barrier();
      mma(4, 0, xb, wa);
      mma(4, 2, xb, wb);
      barrier();
    };

    using Z = std::integral_constant<int, 0>;
    using O = std::integral_constant<int, 1>;
    using T2 = std::integral_constant<int, 2>;
    if constexpr (PH == 2) {
      if (!ov) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else if constexpr (EpiKind<EPI>::swiglu) asm volatile("s_waitcnt vmcnt(11)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(19)" ::: "memory");
      barrier();
      if (wm == 1) barrier();     // stagger: waves 4-7 run one section behind
      int t = 0;
      for (; t + 4 <= L; t += 2) {
        tile2(t, Z{}, Z{});
        tile2(t + 1, O{}, Z{});
      }
      tile2(t, Z{}, O{});
      tile2(t + 1, O{}, T2{});
    } else {
      if (!ov) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if constexpr (EpiKind<EPI>::swiglu) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
      barrier();
      if (wm == 1) barrier();     // stagger: waves 4-7 run one section behind
      int t = 0;
      for (; t + 4 <= L; t += 2) {
        tile(t, Z{}, Z{});
        tile(t + 1, O{}, Z{});
      }
      tile(t, Z{}, O{});
      tile(t + 1, O{}, T2{});
    }
    if (wm == 0) barrier();     // pairs with the last barrier of waves 4-7: every LDS read retired
  };

  drive<512>(a, smem, prologue, body,
             [&](auto&& store16) {
#pragma unroll
               for (int i = 0; i < 8; ++i)
#pragma unroll
                 for (int j = 0; j < 4; ++j) store16(i * 4 + j, acc[i][j]);
             },
             [&](auto&& load16, int own, int n) {
               // the left fold s_0 + s_1 + .. of every piece in order; with own 0 / 1 the registers are
               // s_own (x + y == y + x exactly: s_0 + s_1 == s_1 + s_0), with own < 0 every slab is read.
               // 16 loads in flight per batch (a load-add pair per element serialises on vmcnt(0); the
               // fragment registers are free here).  A prefix register set for own >= 2 spills (hipcc).
               if (own < 0) {
#pragma unroll
                 for (int i = 0; i < 8; ++i)
#pragma unroll
                   for (int j = 0; j < 4; ++j) acc[i][j] = load16(0, i * 4 + j);
               }
               for (int jj = own == 1 ? 0 : 1; jj < n; ++jj) {
                 if (jj == own) continue;
#pragma unroll
                 for (int i0 = 0; i0 < 8; i0 += 4) {
                   f32x4 v[4][4];
#pragma unroll
                   for (int i = 0; i < 4; ++i)
#pragma unroll
                     for (int j = 0; j < 4; ++j) v[i][j] = load16(jj, (i0 + i) * 4 + j);
#pragma unroll
                   for (int i = 0; i < 4; ++i)
#pragma unroll
                     for (int j = 0; j < 4; ++j) acc[i0 + i][j] += v[i][j];
                 }
               }
             },
             [&](int tm, int tn) {
               const int te = fresh_tid();
               if constexpr (EpiKind<EPI>::res)
                 epilogue_res(acc, a.Y, a.ldy, M, tm * kBM, tn, (te >> 8) & 1, (te >> 6) & 3, te & 63, ep_lds, a.ss,
                              a.ss_ld);
               else if constexpr (EpiKind<EPI>::rope)
                 epilogue_rope(acc, a, tm * kBM, tn, (te >> 8) & 1, (te >> 6) & 3, te & 63, ep_lds + rs_slot * 256,
                               (uint16_t*)smem);
               else
                 epilogue<EPI>(acc, a.Y, a.ldy, M, tm * kBM, tn, (te >> 8) & 1, (te >> 6) & 3, te & 63,
                               ep_lds + rs_slot * 256);
             });
}

// Per-device split-K workspace (one fp32 slab per block + two counters per tile),
// allocated on first use outside stream capture.  Shared by every stream of
// the process: the engine issues its projection GEMMs on one stream at a time.
struct SkWorkspace {
  float* ws = nullptr;
  int* cnt = nullptr;   // 2 P counters, preceded by the error word cnt[-1] (timed-out waits)
  int P = 0;
};

SkWorkspace g_sk_per_dev[64];

SkWorkspace* sk_peek(int dev) { return g_sk_per_dev[dev].ws ? &g_sk_per_dev[dev] : nullptr; }

SkWorkspace* sk_workspace(hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  SkWorkspace& w = g_sk_per_dev[dev];
  if (w.ws) return &w;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 8) return nullptr;
  const int P = cus & ~7;
  float* ws = nullptr;
  int* cnt = nullptr;
  if (hipMalloc(&ws, (size_t)P * 65536 * sizeof(float)) != hipSuccess) return nullptr;
  if (hipMalloc(&cnt, (size_t)(2 * P + 1) * sizeof(int)) != hipSuccess ||
      hipMemset(cnt, 0, (size_t)(2 * P + 1) * sizeof(int)) != hipSuccess) {
    hipFree(ws);
    return nullptr;
  }
  w.ws = ws;
  w.cnt = cnt + 1;
  w.P = P;
  return &w;
}

// Split-K waits of this device that ran out since the last reset (0 unless a counter broke).
int sk_timeouts(bool reset) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
  SkWorkspace* w = sk_peek(dev);
  if (!w) return 0;
  int v = 0;
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&v, w->cnt - 1, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  if (reset && v && hipMemset(w->cnt - 1, 0, sizeof(int)) != hipSuccess) return -1;
  return v;
}

// CUs the persistent / split-K launches size their grid for (0 = all of the device's): a GEMM
// issued on a CU-masked stream (two-batch-overlap decode steps keep a few CUs of every XCD for
// attention) must not launch one block per device CU, or the blocks past the mask run as a
// second round.  Set by the host around such a step (dgi_set_gemm_cus).
int g_cu_limit = 0;

// skmode 0: whole tiles only; 1: hybrid split-K when the tiles leave the last wave at most half
// full (and fewer than 8 full waves); 2: hybrid whenever tiles % CUs leaves room for 2 splits
struct NormArgs {
  float* ss = nullptr;
  int ss_ld = 0;
  float inv_k = 0.f, eps = 0.f;
  const int* pos = nullptr;
  const float* cs = nullptr;
  const int* slots = nullptr;
  uint16_t* kc = nullptr;
  uint16_t* vc = nullptr;
  int qcols = 0, kvcols = 0, nkv = 0, bs = 0;
};

template <int EPI>
void launch_pp(const void* x, int ldx, const void* w, void* y, int ldy, int M, int I, int K, int tiles_m, int total,
               int skmode, int prio, hipStream_t s, const NormArgs& na = NormArgs{}) {
  decltype(&mfma_gemm_pp_kernel<EPI, 0, 2>) kern;
  if constexpr (EPI >= 2)       // the fused-norm epilogues: default priority scheme only
    kern = (prio & 4) ? mfma_gemm_pp_kernel<EPI, 0, 2> : mfma_gemm_pp_kernel<EPI, 0, 4>;
  else
    kern = (prio & 4) ? (prio & 3) == 1   ? mfma_gemm_pp_kernel<EPI, 1, 2>
                        : (prio & 3) == 2 ? mfma_gemm_pp_kernel<EPI, 2, 2>
                                          : mfma_gemm_pp_kernel<EPI, 0, 2>
                      : (prio & 3) == 1   ? mfma_gemm_pp_kernel<EPI, 1, 4>
                      : (prio & 3) == 2   ? mfma_gemm_pp_kernel<EPI, 2, 4>
                                          : mfma_gemm_pp_kernel<EPI, 0, 4>;
  // EPI 2 reads the tile it stores (in place) and EPI 5 stages its tile through the staging LDS: no
  // overlap of the next tile's loads with their epilogues
  PPArgs a{(const uint16_t*)x, (const uint16_t*)w, (uint16_t*)y, nullptr, nullptr, ldx, ldy, M, I, K, tiles_m, total,
           0, 0, 0, 0, !(prio & 8) && EPI != 2 && EPI != 5, na.ss, na.ss_ld, na.inv_k, na.eps,
           na.pos, na.cs, na.slots, na.kc, na.vc, na.qcols, na.kvcols, na.nkv, na.bs};
  const int nt = K / kBK;
  SkWorkspace* sk = ((skmode || a.ovl) && nt >= 8) ? sk_workspace(s) : nullptr;
  if (sk) {
    const int P = (g_cu_limit >= 8 && g_cu_limit < sk->P) ? (g_cu_limit & ~7) : sk->P;
    const int full = total / P, rem = total % P;
    const int splits = rem ? min(4, P / rem) : 0;
    if (skmode && splits >= 2 && (full < 8 || skmode == 2)) {
      a.ws = sk->ws;
      a.cnt = sk->cnt;
      a.rem = rem;
      a.splits = splits;
      a.full = full;
      a.P = P;
      kern<<<dim3(P), 512, 0, s>>>(a);
      return;
    }
    if (a.ovl && rem == 0 && full >= 2) {
      // whole waves of tiles: persistent, so each block's next tile loads under this one's epilogue
      a.full = full;
      a.P = P;
      kern<<<dim3(P), 512, 0, s>>>(a);
      return;
    }
  }
  kern<<<dim3(total), 512, 0, s>>>(a);
}

template <int EPI, int SCHED>
void launch(const void* x, int ldx, const void* w, void* y, int ldy, int M, int I, int K, int tiles_m, int total,
            int skmode, int prio, hipStream_t s) {
  if (SCHED == 3)
    launch_pp<EPI>(x, ldx, w, y, ldy, M, I, K, tiles_m, total, skmode, prio, s);
  else if (SCHED == 2)
    mfma_gemm_ring_kernel<EPI><<<dim3(total), 512, 0, s>>>((const uint16_t*)x, ldx, (const uint16_t*)w,
                                                          (uint16_t*)y, ldy, M, I, K, tiles_m, total);
  else
    mfma_gemm_kernel<EPI, SCHED><<<dim3(total), 512, 0, s>>>((const uint16_t*)x, ldx, (const uint16_t*)w,
                                                            (uint16_t*)y, ldy, M, I, K, tiles_m, total);
}

}  // namespace

// epi & 1: 0 = Y[M, N] = X W^T with N = rows of W; 1 = Y[M, I] = SwiGLU with W = [gate; up] (2I rows).
// epi >> 4: K-loop schedule (0 = compiler order, 1 = interleaved, 2 = 4-slot ring of 32-deep sub-steps,
// 3 = ping-pong wave groups, 4 phases per K tile, 4 = 128 x 128 half tile, epi 0 only).  (epi >> 8) & 3: stream-K policy of schedule 3
// (0 = auto, 1 = off, 2 = whenever the tiles leave the last wave part-empty).  (epi >> 10) & 3:
// s_setprio variant of schedule 3, (epi >> 12) & 1: two 32-MFMA phases per K tile, (epi >> 13) & 1:
// four 16-MFMA phases (default: two up to M = 2560, see mfma_gemm_pp_kernel), (epi >> 14) & 1: no
// cross-tile overlap (next tile's prologue after the epilogue; whole waves of tiles not persistent).
extern "C" void dgi_set_gemm_cus(int cus) { g_cu_limit = cus; }

extern "C" int dgi_gemm_split_timeouts(int reset) { return sk_timeouts(reset != 0); }

// The fused-RMSNorm GEMMs (ping-pong schedule): kind 2 = residual (y += x w^T in place, row
// partial sums of squares to ss[:, N / 256 columns]), 3 = y = rstd * x w^T, 4 = SwiGLU of
// rstd * x [gate; up]^T, with rstd from the ss_ld partials per row of ss.  phases: 0 auto, 2, 4.
extern "C" int dgi_mfma_gemm_norm(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K,
                                  int kind, float* ss, int ss_ld, float inv_k, float eps, int phases, hipStream_t s) {
  if (M <= 0) return 0;
  if (kind < 2 || kind > 4 || K % (2 * kBK) || K < 4 * kBK || ldx % 8 || ldy % 4 || N % 256 || !ss || ss_ld <= 0)
    return -3;
  if (kind == 2 && ss_ld < N / 256) return -3;
  if (kind != 2 && (ss_ld % 8 || ss_ld > 32)) return -3;
  int prio = (phases == 2 || (phases == 0 && M <= 2560)) ? 4 : 0;
  const int I = kind == 4 ? N / 2 : 0;
  const int tiles_n = kind == 4 ? I / 128 : N / 256;
  const int tiles_m = (M + kBM - 1) / kBM;
  const int total = tiles_m * tiles_n;
  NormArgs na;
  na.ss = ss;
  na.ss_ld = ss_ld;
  na.inv_k = inv_k;
  na.eps = eps;
  if (kind == 2)
    launch_pp<2>(x, ldx, w, y, ldy, M, I, K, tiles_m, total, 1, prio, s, na);
  else if (kind == 3)
    launch_pp<3>(x, ldx, w, y, ldy, M, I, K, tiles_m, total, 1, prio, s, na);
  else
    launch_pp<4>(x, ldx, w, y, ldy, M, I, K, tiles_m, total, 1, prio, s, na);
  DGI_CHECK_LAUNCH();
  return 0;
}

// The normalised qkv projection with the RoPE + paged-KV epilogue (EPI 5): y = rstd * x w^T with the
// q heads rotated in place (y's k / v columns are left unwritten), k (rotated) and v written to the
// caches [blocks, nkv, bs, 128] at slots[m] (< 0: skipped).  Head dim 128, full NeoX rotary;
// nh * 128 and nkv * 128 multiples of 256.
extern "C" int dgi_mfma_gemm_norm_rope(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K,
                                       float* ss, int ss_ld, float inv_k, float eps, const int* pos,
                                       const float* cos_sin, const int* slots, void* k_cache, void* v_cache,
                                       int nh, int nkv, int block_size, int phases, hipStream_t s) {
  if (M <= 0) return 0;
  if (K % (2 * kBK) || K < 4 * kBK || ldx % 8 || ldy % 8 || N % 256 || !ss || ss_ld % 8 || ss_ld > 32 || ss_ld <= 0)
    return -3;
  if ((nh * 128) % 256 || (nkv * 128) % 256 || N != (nh + 2 * nkv) * 128 || block_size <= 0) return -3;
  int prio = (phases == 2 || (phases == 0 && M <= 2560)) ? 4 : 0;
  const int tiles_m = (M + kBM - 1) / kBM;
  const int total = tiles_m * (N / 256);
  NormArgs na;
  na.ss = ss;
  na.ss_ld = ss_ld;
  na.inv_k = inv_k;
  na.eps = eps;
  na.pos = pos;
  na.cs = cos_sin;
  na.slots = slots;
  na.kc = (uint16_t*)k_cache;
  na.vc = (uint16_t*)v_cache;
  na.qcols = nh * 128;
  na.kvcols = nkv * 128;
  na.nkv = nkv;
  na.bs = block_size;
  launch_pp<5>(x, ldx, w, y, ldy, M, 0, K, tiles_m, total, 1, prio, s, na);
  DGI_CHECK_LAUNCH();
  return 0;
}

extern "C" int dgi_mfma_gemm(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K,
                             int epi, hipStream_t s) {
  if (M <= 0) return 0;
  const int swiglu = epi & 15;
  int sched = (epi >> 4) & 15;
  if (sched == 4) {             // half tile: plain GEMM, N % 128
    if (swiglu || K % kBK || ldx % 8 || ldy % 4 || N % kHM) return -3;
    const int tiles_m = (M + kHM - 1) / kHM;
    const int total = tiles_m * (N / kHM);
    mfma_gemm_half_kernel<<<dim3(total), 256, 0, s>>>((const uint16_t*)x, ldx, (const uint16_t*)w, (uint16_t*)y,
                                                      ldy, M, K, tiles_m, total);
    DGI_CHECK_LAUNCH();
    return 0;
  }
  if (K % kBK || ldx % 8 || ldy % 4 || N % 256) return -3;
  const int skmode = ((epi >> 8) & 3) == 0 ? 1 : ((epi >> 8) & 3) == 1 ? 0 : 2;
  int prio = ((epi >> 10) & 7) | (((epi >> 14) & 1) << 3);
  // phases per K tile: (epi >> 13) & 1 forces 4; otherwise 2 up to 10 row tiles (M <= 2560: the
  // 2-phase body measured 2-4 % faster there) and 4 above (its deeper prefetch wins at M = 4096)
  if (!((epi >> 13) & 1) && !(prio & 4) && M <= 2560) prio |= 4;
  if (swiglu > 1 || sched > 3) return -4;
  if (sched == 3 && (K % (2 * kBK) || K < 4 * kBK)) sched = 1;   // ping-pong needs an even count of >= 4 K tiles
  const int I = swiglu ? N / 2 : 0;
  const int tiles_n = swiglu ? I / 128 : N / 256;
  const int tiles_m = (M + kBM - 1) / kBM;
  const int total = tiles_m * tiles_n;
  if (swiglu)
    (sched == 3 ? launch<1, 3> : sched == 2 ? launch<1, 2> : sched ? launch<1, 1> : launch<1, 0>)(
        x, ldx, w, y, ldy, M, I, K, tiles_m, total, skmode, prio, s);
  else
    (sched == 3 ? launch<0, 3> : sched == 2 ? launch<0, 2> : sched ? launch<0, 1> : launch<0, 0>)(
        x, ldx, w, y, ldy, M, I, K, tiles_m, total, skmode, prio, s);
  DGI_CHECK_LAUNCH();
  return 0;
}
