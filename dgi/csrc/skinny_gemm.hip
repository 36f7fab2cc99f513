// dgi/csrc/skinny_gemm.hip — weight-streaming GEMM for decode-sized M.
//
// Y[M, N] = X[M, K] · W[N, K]^T (+ bias[N]), bf16 in/out, fp32 accumulate, M <= 32.
//
// At decode batch sizes every projection is a read of its weight matrix:
// the FLOPs are free and the kernel's job is to keep HBM3E streaming.
// hipBLASLt's tiles for M = 1..32 leave most of the ~6 TB/s unused, so this
// kernel is shaped around the weight stream instead of the output tile:
//
//  * one workgroup per 16·NT output columns, NW waves splitting K between them;
//  * lane l reads 32 contiguous bytes of weight row n0 + (l & 15) per
//    64-deep K step: the 4 lane groups cover a full 128-byte line of each
//    of the 16 rows, loaded straight to VGPRs (no LDS round trip — the
//    operand is used once) with nontemporal loads, U steps in flight;
//  * those 8+8 bf16 are exactly the B fragments of two
//    v_mfma_f32_16x16x32_bf16 (lane holds B[k = 8(l>>4)+j][col l&15]); the
//    K order inside a step is permuted identically for X, which a dot
//    product does not see.  X rows (A fragments, 16 per MFMA, zero above M)
//    come from L2 — X is tiny and every workgroup reads the same bytes;
//  * the NW partial 16x16 tiles are summed through LDS and the epilogue adds
//    the bias and rounds to bf16.
// MT = 2 handles 17..32 rows with the same weight registers (two A tiles);
// NT > 1 column tiles per wave reuse each X fragment NT times.  Loads run
// D - 1 groups of U K-steps ahead of the MFMAs (register ring, D = 2 is the
// double buffer).
#include "common.h"

using namespace dgi;

namespace {

// Fragments of U K-steps: W for NT column tiles, X for MT row tiles.
template <int MT, int NT, int U>
struct Frag {
  u32x4 w[U][NT][2];
  u32x4 x[U][MT][2];
};

template <int NW, int MT, int NT, int U, int D>
__global__ __launch_bounds__(NW * 64) void skinny_gemm_kernel(
    const uint16_t* __restrict__ X, int ldx, const uint16_t* __restrict__ W,
    const uint16_t* __restrict__ bias, uint16_t* __restrict__ Y, int ldy, int M, int K) {
  __shared__ f32x4 red[NW][MT * NT][64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int n0 = blockIdx.x * 16 * NT;
  // host guarantees nsteps % (NW * U) == 0: every group is full, no predicates in the stream
  const int ngroups = (K >> 6) / (NW * U);
  const uint16_t* wrow = W + (size_t)(n0 + r) * K + g * 16 + (size_t)w * 64;
  const size_t wtile = (size_t)16 * K;  // next column tile
  const uint16_t* xrow[MT];
  bool xval[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + r;
    xval[mt] = m < M;
    xrow[mt] = X + (size_t)(xval[mt] ? m : 0) * ldx + g * 16 + w * 64;
  }
  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto load = [&](Frag<MT, NT, U>& f, int grp) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t off = ((size_t)grp * NW * U + (size_t)u * NW) * 64;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const u32x4* p = reinterpret_cast<const u32x4*>(wrow + nt * wtile + off);
        f.w[u][nt][0] = __builtin_nontemporal_load(p);
        f.w[u][nt][1] = __builtin_nontemporal_load(p + 1);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        if (xval[mt]) {
          const u32x4* p = reinterpret_cast<const u32x4*>(xrow[mt] + off);
          f.x[u][mt][0] = p[0];
          f.x[u][mt][1] = p[1];
        } else {
          f.x[u][mt][0] = u32x4{0u, 0u, 0u, 0u};
          f.x[u][mt][1] = u32x4{0u, 0u, 0u, 0u};
        }
      }
    }
  };
  auto compute = [&](const Frag<MT, NT, U>& f) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(f.x[u][mt][0]),
                                                                as_bf16x8(f.w[u][nt][0]), acc[mt][nt], 0, 0, 0);
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(f.x[u][mt][1]),
                                                                as_bf16x8(f.w[u][nt][1]), acc[mt][nt], 0, 0, 0);
        }
  };
  // register ring of D groups: D - 1 in flight ahead of the one being multiplied
  Frag<MT, NT, U> ring[D];
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (d < ngroups) load(ring[d], d);
  for (int base = 0; base < ngroups; base += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      if (base + d < ngroups) {  // uniform
        compute(ring[d]);
        if (base + D + d < ngroups) load(ring[d], base + D + d);
      }
    }
  }

#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) red[w][mt * NT + nt][lane] = acc[mt][nt];
  __syncthreads();
  // wave w (< MT*NT) sums the NW partial tiles of output tile w
  if (w >= MT * NT) return;
  f32x4 v = red[0][w][lane];
#pragma unroll
  for (int j = 1; j < NW; ++j) v += red[j][w][lane];
  const int mt = w / NT, nt = w % NT;
  const int col = n0 + nt * 16 + r;
  const float b = bias ? bf16_to_f32(bias[col]) : 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mt * 16 + g * 4 + i;
    if (m < M) Y[(size_t)m * ldy + col] = f32_to_bf16(v[i] + b);
  }
}

template <int NW, int MT, int NT, int U, int D = 2>
int launch(const void* x, int ldx, const void* w, const void* bias, void* y, int ldy, int M, int N, int K,
           hipStream_t s) {
  if (N % (16 * NT) || (K / 64) % (NW * U)) return -5;
  skinny_gemm_kernel<NW, MT, NT, U, D><<<dim3(N / (16 * NT)), NW * 64, 0, s>>>(
      (const uint16_t*)x, ldx, (const uint16_t*)w, (const uint16_t*)bias, (uint16_t*)y, ldy, M, K);
  DGI_CHECK_LAUNCH();
  return 0;
}

template <int MT>
int dispatch(int cfg, const void* x, int ldx, const void* w, const void* bias, void* y, int ldy, int M, int N,
             int K, hipStream_t s) {
  switch (cfg) {
    case 1: return launch<16, MT, 1, 1>(x, ldx, w, bias, y, ldy, M, N, K, s);
    case 2: return launch<8, MT, 2, 2>(x, ldx, w, bias, y, ldy, M, N, K, s);
    case 3: return launch<16, MT, 2, 1>(x, ldx, w, bias, y, ldy, M, N, K, s);
    case 4: return launch<8, MT, 1, 2>(x, ldx, w, bias, y, ldy, M, N, K, s);
    case 5: return MT == 1 ? launch<16, 1, 4, 1>(x, ldx, w, bias, y, ldy, M, N, K, s)   // MT 2 would spill
                           : launch<16, MT, 2, 1>(x, ldx, w, bias, y, ldy, M, N, K, s);
    case 6: return launch<4, MT, 2, 4>(x, ldx, w, bias, y, ldy, M, N, K, s);
    // deeper rings: more bytes in flight per wave for short kernels (o-proj) and long K (down)
    case 7: return launch<8, MT, 1, 1, 4>(x, ldx, w, bias, y, ldy, M, N, K, s);
    case 8: return launch<8, MT, 1, 2, 4>(x, ldx, w, bias, y, ldy, M, N, K, s);
    case 9: return launch<4, MT, 1, 2, 4>(x, ldx, w, bias, y, ldy, M, N, K, s);
    case 10: return launch<4, MT, 1, 1, 8>(x, ldx, w, bias, y, ldy, M, N, K, s);
    case 11: return launch<8, MT, 1, 1, 8>(x, ldx, w, bias, y, ldy, M, N, K, s);
    default: return -4;
  }
}

}  // namespace

// cfg selects (waves per workgroup, column tiles per wave, K-steps per group);
// 0 = pick from the shape.  Requires K % 1024 == 0 (16 K-steps per group).
extern "C" int dgi_skinny_gemm(const void* x, int ldx, const void* w, const void* bias, void* y, int ldy, int M,
                               int N, int K, int cfg, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 32) return -2;
  if (K % 1024 || N % 16 || ldx % 8) return -3;
  // 8 waves x 2 K-steps per group, one column tile per wave: the fastest or
  // within 3 % of it on every 8B / 70B projection shape at M <= 8
  if (cfg == 0) cfg = 4;
  return M > 16 ? dispatch<2>(cfg, x, ldx, w, bias, y, ldy, M, N, K, s)
                : dispatch<1>(cfg, x, ldx, w, bias, y, ldy, M, N, K, s);
}
