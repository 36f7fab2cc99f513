// dgi/csrc/rmsnorm.hip — RMSNorm and fused residual-add + RMSNorm.
//
// Replaces the RMSNorm modules that the reference executes inside HF Llama
// layers (worker/distributed/model_shard.py:209-226).  One 256-thread
// workgroup per row; the row lives in registers (16-byte bf16x8 loads, NC
// chunks per thread) so the residual stream is read once and written once.
#include "common.h"

using namespace dgi;

template <int NC, bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_kernel(
    uint16_t* out, uint16_t* x, uint16_t* __restrict__ residual,
    const uint16_t* __restrict__ w, int H, float eps) {
  const int row = blockIdx.x;
  const int tid = threadIdx.x;
  const int nchunk = H >> 3;
  u32x4* xr = reinterpret_cast<u32x4*>(x + (size_t)row * H);
  u32x4* rr = ADD ? reinterpret_cast<u32x4*>(residual + (size_t)row * H) : nullptr;
  u32x4* orow = reinterpret_cast<u32x4*>(out + (size_t)row * H);
  const u32x4* wr = reinterpret_cast<const u32x4*>(w);

  // every load of the row (x, residual, weight) is issued before any use, so a
  // thread has 3*NC 16-byte loads in flight instead of one dependent chain
  u32x4 xa[NC], ra[NC], wa[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = tid + c * 256;
    if (i < nchunk) {
      xa[c] = xr[i];
      if (ADD) ra[c] = rr[i];
      wa[c] = wr[i];
    }
  }
  float v[NC][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = tid + c * 256;
    if (i < nchunk) {
      unpack8(xa[c], v[c]);
      if (ADD) {
        float r[8];
        unpack8(ra[c], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] += r[j];
        // The residual stream is kept in bf16 (what the next layer adds to).
        u32x4 p = pack8(v[c]);
        rr[i] = p;
        unpack8(p, v[c]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[c][j] * v[c][j];
    }
  }
  __shared__ float red[4];
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float inv = rsqrtf(tot / (float)H + eps);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = tid + c * 256;
    if (i < nchunk) {
      float wf[8];
      unpack8(wa[c], wf);
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[c][j] * inv * wf[j];
      orow[i] = pack8(o);
    }
  }
}

template <bool ADD>
static int launch_rms(uint16_t* out, uint16_t* x, uint16_t* residual, const uint16_t* w, int T,
                      int H, float eps, hipStream_t s) {
  const int nchunk = H / 8;
  const int nc = (nchunk + 255) / 256;
  dim3 grid(T), block(256);
  if (T == 0) return 0;
  switch (nc) {
    case 1: rmsnorm_kernel<1, ADD><<<grid, block, 0, s>>>(out, x, residual, w, H, eps); break;
    case 2: rmsnorm_kernel<2, ADD><<<grid, block, 0, s>>>(out, x, residual, w, H, eps); break;
    case 3: rmsnorm_kernel<3, ADD><<<grid, block, 0, s>>>(out, x, residual, w, H, eps); break;
    case 4: rmsnorm_kernel<4, ADD><<<grid, block, 0, s>>>(out, x, residual, w, H, eps); break;
    case 5: case 6: case 7: case 8:
      rmsnorm_kernel<8, ADD><<<grid, block, 0, s>>>(out, x, residual, w, H, eps); break;
    default: return -1;
  }
  DGI_CHECK_LAUNCH();
  return 0;
}

extern "C" int dgi_rmsnorm(void* out, const void* x, const void* w, int T, int H, float eps,
                           hipStream_t s) {
  if (H % 8) return -2;
  return launch_rms<false>((uint16_t*)out, (uint16_t*)x, nullptr, (const uint16_t*)w, T, H, eps, s);
}

// residual <- x + residual ; x <- rmsnorm(residual) * w   (both in place)
extern "C" int dgi_fused_add_rmsnorm(void* x, void* residual, const void* w, int T, int H,
                                     float eps, hipStream_t s) {
  if (H % 8) return -2;
  return launch_rms<true>((uint16_t*)x, (uint16_t*)x, (uint16_t*)residual, (const uint16_t*)w, T,
                          H, eps, s);
}
