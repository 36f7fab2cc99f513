// dgi/csrc/skinny_gemm.hip — weight-streaming GEMM for decode-sized M.
//
// Y[M, N] = X[M, K] · W[N, K]^T (+ bias[N]), bf16 in/out, fp32 accumulate, M <= 32.
//
// At decode batch sizes every projection is a read of its weight matrix:
// the FLOPs are free and the kernel's job is to keep HBM3E streaming.
// hipBLASLt's tiles for M = 1..32 leave most of the ~6 TB/s unused, so this
// kernel is shaped around the weight stream instead of the output tile:
//
//  * one workgroup per 16 output columns, NW waves splitting K between them
//    (NW picked by the host so the grid holds ~16 waves per CU);
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
// MT = 2 handles 17..32 rows with the same weight registers (two A tiles).
#include "common.h"

using namespace dgi;

namespace {

template <int NW, int MT, int U>
__global__ __launch_bounds__(NW * 64) void skinny_gemm_kernel(
    const uint16_t* __restrict__ X, int ldx, const uint16_t* __restrict__ W,
    const uint16_t* __restrict__ bias, uint16_t* __restrict__ Y, int ldy, int M, int K) {
  __shared__ f32x4 red[NW][MT][64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int nsteps = K >> 6;
  const uint16_t* wrow = W + (size_t)(n0 + r) * K + g * 16;
  const uint16_t* xrow[MT];
  bool xval[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + r;
    xval[mt] = m < M;
    xrow[mt] = X + (size_t)(xval[mt] ? m : 0) * ldx + g * 16;
  }
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int s0 = w; s0 < nsteps; s0 += NW * U) {
    u32x4 wb[U][2];
    u32x4 xa[U][MT][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ks = s0 + u * NW;
      if (ks < nsteps) {
        const u32x4* p = reinterpret_cast<const u32x4*>(wrow + (size_t)ks * 64);
        wb[u][0] = __builtin_nontemporal_load(p);
        wb[u][1] = __builtin_nontemporal_load(p + 1);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ks = s0 + u * NW;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        if (ks < nsteps && xval[mt]) {
          const u32x4* p = reinterpret_cast<const u32x4*>(xrow[mt] + (size_t)ks * 64);
          xa[u][mt][0] = p[0];
          xa[u][mt][1] = p[1];
        } else {
          xa[u][mt][0] = u32x4{0u, 0u, 0u, 0u};
          xa[u][mt][1] = u32x4{0u, 0u, 0u, 0u};
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ks = s0 + u * NW;
      if (ks < nsteps) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xa[u][mt][0]), as_bf16x8(wb[u][0]),
                                                            acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xa[u][mt][1]), as_bf16x8(wb[u][1]),
                                                            acc[mt], 0, 0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) red[w][mt][lane] = acc[mt];
  __syncthreads();
  if (w >= MT) return;
  // wave w < MT sums the NW partial tiles of row tile w
  f32x4 v = red[0][w][lane];
#pragma unroll
  for (int j = 1; j < NW; ++j) v += red[j][w][lane];
  const int col = n0 + r;
  const float b = bias ? bf16_to_f32(bias[col]) : 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = w * 16 + g * 4 + i;
    if (m < M) Y[(size_t)m * ldy + col] = f32_to_bf16(v[i] + b);
  }
}

template <int MT>
int launch(const void* x, int ldx, const void* w, const void* bias, void* y, int ldy, int M, int N, int K,
           int nw, hipStream_t s) {
  const dim3 grid(N / 16);
  const auto X = (const uint16_t*)x;
  const auto Wp = (const uint16_t*)w;
  const auto B = (const uint16_t*)bias;
  const auto Y = (uint16_t*)y;
  switch (nw) {
    case 16: skinny_gemm_kernel<16, MT, 2><<<grid, 1024, 0, s>>>(X, ldx, Wp, B, Y, ldy, M, K); break;
    case 8: skinny_gemm_kernel<8, MT, 4><<<grid, 512, 0, s>>>(X, ldx, Wp, B, Y, ldy, M, K); break;
    case 4: skinny_gemm_kernel<4, MT, 4><<<grid, 256, 0, s>>>(X, ldx, Wp, B, Y, ldy, M, K); break;
    default: return -4;
  }
  DGI_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// nw = waves per workgroup (4, 8 or 16); 0 = choose so the grid holds ~16 waves per CU.
extern "C" int dgi_skinny_gemm(const void* x, int ldx, const void* w, const void* bias, void* y, int ldy, int M,
                               int N, int K, int nw, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 32) return -2;
  if (K % 64 || N % 16 || ldx % 8) return -3;
  if (nw == 0) {
    const int tiles = N / 16;
    const int steps = K / 64;
    nw = 4;
    while (nw < 16 && tiles * nw < 256 * 16 && steps >= nw * 2 * 4) nw *= 2;
  }
  return M > 16 ? launch<2>(x, ldx, w, bias, y, ldy, M, N, K, nw, s)
                : launch<1>(x, ldx, w, bias, y, ldy, M, N, K, nw, s);
}
