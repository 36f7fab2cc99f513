// dgi/csrc/sampler.hip — on-device token selection.
//
// Greedy argmax and temperature sampling by the Gumbel-max trick in one pass
// over the logits row, so no host sync and no softmax materialisation.  The
// reference samples inside HF generate / vLLM SamplingParams
// (worker/engines/llm.py:62-69, worker/engines/llm_vllm.py:144-151) and
// argmax/multinomial in speculative.py:444-449.
// top-k / top-p filtering, when requested, is a per-row logit threshold
// computed by topkp_thresh_kernel below; sample_kernel skips every element
// under it (rows with top_k/top_p disabled get -inf and skip nothing).
//
// Also: per-row top-k (k <= 16) candidate extraction used by the EAGLE draft
// tree builder (K13): each workgroup keeps a wave-level sorted list.
#include "common.h"

using namespace dgi;

namespace {

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

template <typename T>
__device__ __forceinline__ float load_logit(const T* p, int i);
template <>
__device__ __forceinline__ float load_logit<float>(const float* p, int i) { return p[i]; }
template <>
__device__ __forceinline__ float load_logit<uint16_t>(const uint16_t* p, int i) { return bf16_to_f32(p[i]); }

// Logits arrive as 16-byte vectors (8 bf16 or 4 fp32) when the row allows it:
// one workgroup streams a 128k-vocab row (256 KB bf16) with 4 vectors in
// flight per thread instead of 125 dependent 2-byte loads.
template <typename T>
__device__ __forceinline__ float vec_elem(const u32x4& v, int j);
template <>
__device__ __forceinline__ float vec_elem<float>(const u32x4& v, int j) { return __uint_as_float(v[j]); }
template <>
__device__ __forceinline__ float vec_elem<uint16_t>(const u32x4& v, int j) {
  const uint32_t w = v[j >> 1];
  return __uint_as_float((j & 1) ? (w & 0xffff0000u) : (w << 16));
}

template <typename T, typename F>
__device__ __forceinline__ void scan_row(const T* lp, int V, int stride, F&& f) {
  constexpr int E = 16 / sizeof(T);
  const bool vec = (stride % E == 0) && ((reinterpret_cast<uintptr_t>(lp) & 15) == 0);
  const int nvec = vec ? V / E : 0;
  const int nt = blockDim.x;
  for (int c0 = threadIdx.x; c0 < nvec; c0 += nt * 4) {
    u32x4 buf[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = c0 + u * nt;
      if (c < nvec) buf[u] = reinterpret_cast<const u32x4*>(lp)[c];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = c0 + u * nt;
      if (c < nvec) {
#pragma unroll
        for (int j = 0; j < E; ++j) f(vec_elem<T>(buf[u], j), c * E + j);
      }
    }
  }
  for (int i = nvec * E + threadIdx.x; i < V; i += nt) f(load_logit<T>(lp, i), i);
}

template <typename T>
__global__ __launch_bounds__(1024) void sample_kernel(const T* __restrict__ logits, int V, int stride,
                                                      const float* __restrict__ temperature,
                                                      const long long* __restrict__ seeds,
                                                      long long step, const float* __restrict__ thresh,
                                                      long long* __restrict__ out) {
  const int row = blockIdx.x;
  const T* lp = logits + (size_t)row * stride;
  const float temp = temperature ? temperature[row] : 0.f;
  const bool greedy = temp <= 1e-5f;
  const float inv_t = greedy ? 1.f : 1.f / temp;
  const uint32_t seed = seeds ? (uint32_t)(seeds[row] * 2654435761ull) ^ (uint32_t)(step * 40503u) : 0u;
  float best = -INFINITY;
  int best_i = 0x7fffffff;
  if (greedy) {
    scan_row<T>(lp, V, stride, [&](float v, int i) {
      if (v > best || (v == best && i < best_i)) { best = v; best_i = i; }
    });
  } else {
    const float th = thresh ? thresh[row] : -INFINITY;
    scan_row<T>(lp, V, stride, [&](float v, int i) {
      if (v < th) return;  // outside the top-k / top-p set
      const uint32_t h = hash32(seed ^ hash32((uint32_t)i + 0x9e3779b9u));
      const float u = ((h >> 8) + 0.5f) * (1.0f / 16777216.0f);
      v = v * inv_t - __logf(-__logf(u));
      if (v > best || (v == best && i < best_i)) { best = v; best_i = i; }
    });
  }
  // wave reduce
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(best_i, o, 64);
    if (ob > best || (ob == best && oi < best_i)) { best = ob; best_i = oi; }
  }
  __shared__ float sb[16];
  __shared__ int si[16];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sb[w] = best; si[w] = best_i; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = blockDim.x >> 6;
    for (int k = 1; k < nw; ++k)
      if (sb[k] > best || (sb[k] == best && si[k] < best_i)) { best = sb[k]; best_i = si[k]; }
    out[row] = best_i == 0x7fffffff ? 0 : best_i;
  }
}

// Small batches: a row split over C workgroups of SP_CHUNK logits each (one 128k-vocab row
// on one workgroup is ~16 dependent rounds of loads, 15.5 us on the 8B decode step,
// profiles/r5_decode/decode8b_b1_step_breakdown_r5.md).  Each part writes its (best, index);
// the final kernel reduces the C parts of a row on one wave.  The Gumbel noise depends only on
// (seed, step, index), so the pick is the single-workgroup kernel's, ties to the lower index.
constexpr int SP_NT = 256;
constexpr int SP_CHUNK = 8192;

template <typename T>
__global__ __launch_bounds__(SP_NT) void sample_part_kernel(const T* __restrict__ logits, int V, int stride,
                                                            const float* __restrict__ temperature,
                                                            const long long* __restrict__ seeds, long long step,
                                                            const float* __restrict__ thresh, float* __restrict__ pv,
                                                            int* __restrict__ pi) {
  const int c = blockIdx.x, row = blockIdx.y, C = gridDim.x;
  const int lo = c * SP_CHUNK;
  const int n = min(V - lo, SP_CHUNK);
  const T* lp = logits + (size_t)row * stride + lo;
  const float temp = temperature ? temperature[row] : 0.f;
  const bool greedy = temp <= 1e-5f;
  const float inv_t = greedy ? 1.f : 1.f / temp;
  const uint32_t seed = seeds ? (uint32_t)(seeds[row] * 2654435761ull) ^ (uint32_t)(step * 40503u) : 0u;
  float best = -INFINITY;
  int best_i = 0x7fffffff;
  if (greedy) {
    scan_row<T>(lp, n, stride, [&](float v, int i) {
      i += lo;
      if (v > best || (v == best && i < best_i)) { best = v; best_i = i; }
    });
  } else {
    const float th = thresh ? thresh[row] : -INFINITY;
    scan_row<T>(lp, n, stride, [&](float v, int i) {
      i += lo;
      if (v < th) return;
      const uint32_t h = hash32(seed ^ hash32((uint32_t)i + 0x9e3779b9u));
      const float u = ((h >> 8) + 0.5f) * (1.0f / 16777216.0f);
      v = v * inv_t - __logf(-__logf(u));
      if (v > best || (v == best && i < best_i)) { best = v; best_i = i; }
    });
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(best_i, o, 64);
    if (ob > best || (ob == best && oi < best_i)) { best = ob; best_i = oi; }
  }
  __shared__ float sb[SP_NT / 64];
  __shared__ int si[SP_NT / 64];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sb[w] = best; si[w] = best_i; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < SP_NT / 64; ++k)
      if (sb[k] > best || (sb[k] == best && si[k] < best_i)) { best = sb[k]; best_i = si[k]; }
    pv[(size_t)row * C + c] = best;
    pi[(size_t)row * C + c] = best_i;
  }
}

// one wave per row over its C parts (C <= 64 * 4)
__global__ __launch_bounds__(64) void sample_final_kernel(const float* __restrict__ pv, const int* __restrict__ pi,
                                                          int C, long long* __restrict__ out) {
  const int row = blockIdx.x, lane = threadIdx.x;
  float best = -INFINITY;
  int best_i = 0x7fffffff;
  for (int c = lane; c < C; c += 64) {
    const float v = pv[(size_t)row * C + c];
    const int i = pi[(size_t)row * C + c];
    if (v > best || (v == best && i < best_i)) { best = v; best_i = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(best_i, o, 64);
    if (ob > best || (ob == best && oi < best_i)) { best = ob; best_i = oi; }
  }
  if (lane == 0) out[row] = best_i == 0x7fffffff ? 0 : best_i;
}

// top-k (k <= 16) per row: values + indices, descending.  One 256-thread
// block per row; each thread keeps its own sorted top-k, then a tree merge in LDS.
template <typename T>
__global__ __launch_bounds__(256) void topk_kernel(const T* __restrict__ logits, int V, int stride,
                                                   int K, float* __restrict__ out_v,
                                                   long long* __restrict__ out_i) {
  const int row = blockIdx.x;
  const T* lp = logits + (size_t)row * stride;
  float tv[16];
  int ti[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) { tv[k] = -INFINITY; ti[k] = 0x7fffffff; }
  scan_row<T>(lp, V, stride, [&](float v, int i) {
    if (v > tv[K - 1]) {
      int k = K - 1;
      while (k > 0 && tv[k - 1] < v) { tv[k] = tv[k - 1]; ti[k] = ti[k - 1]; --k; }
      tv[k] = v; ti[k] = i;
    }
  });
  __shared__ float sv[256 * 16];
  __shared__ int si[256 * 16];
  for (int k = 0; k < K; ++k) { sv[threadIdx.x * 16 + k] = tv[k]; si[threadIdx.x * 16 + k] = ti[k]; }
  __syncthreads();
  for (int half = 128; half > 0; half >>= 1) {
    if (threadIdx.x < half) {
      const float* a = sv + threadIdx.x * 16;
      const int* ai = si + threadIdx.x * 16;
      const float* bv = sv + (threadIdx.x + half) * 16;
      const int* bi = si + (threadIdx.x + half) * 16;
      float mv[16]; int mi[16];
      int x = 0, y = 0;
      for (int k = 0; k < K; ++k) {
        const bool takea = (a[x] > bv[y]) || (a[x] == bv[y] && ai[x] <= bi[y]);
        if (takea) { mv[k] = a[x]; mi[k] = ai[x]; ++x; } else { mv[k] = bv[y]; mi[k] = bi[y]; ++y; }
      }
      for (int k = 0; k < K; ++k) { sv[threadIdx.x * 16 + k] = mv[k]; si[threadIdx.x * 16 + k] = mi[k]; }
    }
    __syncthreads();
  }
  if (threadIdx.x < K) {
    out_v[(size_t)row * K + threadIdx.x] = sv[threadIdx.x];
    out_i[(size_t)row * K + threadIdx.x] = si[threadIdx.x];
  }
}


// ---------------------------------------------------------------------------
// Top-k of log_softmax(row) straight from bf16 logits (EAGLE draft expansion), without
// materialising the fp32 log-probs: log_softmax is monotone, so the top-k indices are the
// logits' and only the k winners need `v - logsumexp(row)`.
//
// Stage 1, grid (C chunks, B rows): each workgroup scans one chunk of a row with 16-byte
// loads, keeping a per-thread top-k and an online (max, sum of exp) pair, merges them in
// LDS and writes the chunk's top-k + (max, sum).  Stage 2, one workgroup per row: merges
// the C x k candidates and the C partial sums.  A 128k-vocab row is 16 workgroups instead
// of one (round 5 trace: the one-block-per-row kernel plus torch's log_softmax took 222 us
// per draft depth at 3 rows).  Ties: lower index first (as topk_kernel).
constexpr int TK_NT = 256;
constexpr int TK_CHUNK = 2048;   // elements per stage-1 workgroup: one 16-byte load per thread

// Sorted (descending) per-thread list of KP entries in registers; every index below is a
// compile-time constant after unrolling (a runtime-K insertion loop compiles to select chains
// over all 16 slots per element).  A new element sinks below equal ones (ties: earlier first).
template <int KP>
__device__ __forceinline__ void tk_insert(float (&tv)[KP], int (&ti)[KP], float v, int i) {
  if (v > tv[KP - 1] || (v == tv[KP - 1] && i < ti[KP - 1])) {
    tv[KP - 1] = v;
    ti[KP - 1] = i;
#pragma unroll
    for (int j = KP - 1; j > 0; --j) {
      if (tv[j] > tv[j - 1] || (tv[j] == tv[j - 1] && ti[j] < ti[j - 1])) {
        const float tvv = tv[j]; tv[j] = tv[j - 1]; tv[j - 1] = tvv;
        const int tii = ti[j]; ti[j] = ti[j - 1]; ti[j - 1] = tii;
      }
    }
  }
}

// block-wide merge of the per-thread lists: each wave reduces its 64 lists with xor
// shuffles (the partner's list inserted into this lane's, all indices compile-time), then
// thread 0 merges the NW wave winners through LDS.  Result valid on thread 0.
template <int KP>
__device__ __forceinline__ void tk_merge2(float (&a)[KP], int (&ai)[KP], const float (&b)[KP], const int (&bi)[KP]) {
#pragma unroll
  for (int k = 0; k < KP; ++k) tk_insert<KP>(a, ai, b[k], bi[k]);
}

template <int KP>
__device__ __forceinline__ void tk_block_reduce(float (&tv)[KP], int (&ti)[KP], float& m, float& sum,
                                                float* s_v, int* s_i, float* s_m, float* s_s) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    float ov[KP];
    int oi[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) { ov[k] = __shfl_xor(tv[k], off); oi[k] = __shfl_xor(ti[k], off); }
    tk_merge2<KP>(tv, ti, ov, oi);
    const float om = __shfl_xor(m, off), os = __shfl_xor(sum, off);
    const float nm = fmaxf(m, om);
    sum = (sum > 0.f ? sum * __expf(m - nm) : 0.f) + (os > 0.f ? os * __expf(om - nm) : 0.f);
    m = nm;
  }
  constexpr int NW = TK_NT / 64;
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < KP; ++k) { s_v[w * KP + k] = tv[k]; s_i[w * KP + k] = ti[k]; }
    s_m[w] = m;
    s_s[w] = sum;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int ww = 1; ww < NW; ++ww) {
      float ov[KP];
      int oi[KP];
#pragma unroll
      for (int k = 0; k < KP; ++k) { ov[k] = s_v[ww * KP + k]; oi[k] = s_i[ww * KP + k]; }
      tk_merge2<KP>(tv, ti, ov, oi);
      const float om = s_m[ww], os = s_s[ww];
      const float nm = fmaxf(m, om);
      sum = (sum > 0.f ? sum * __expf(m - nm) : 0.f) + (os > 0.f ? os * __expf(om - nm) : 0.f);
      m = nm;
    }
  }
}

template <int KP>
__global__ __launch_bounds__(TK_NT) void topk_lse_part_kernel(const uint16_t* __restrict__ logits, int V, int stride,
                                                              float* __restrict__ ws_v, int* __restrict__ ws_i,
                                                              float* __restrict__ ws_ms) {
  const int c = blockIdx.x, C = gridDim.x, row = blockIdx.y;
  const uint16_t* lp = logits + (size_t)row * stride;
  const int lo = c * TK_CHUNK, hi = min(V, lo + TK_CHUNK);
  float tv[KP];
  int ti[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) { tv[k] = -INFINITY; ti[k] = 0x7fffffff; }
  float m = -INFINITY, sum = 0.f;
  auto take = [&](float v, int i) {
    if (v > m) {                       // online logsumexp (finite logits; -inf entries add nothing)
      sum = (sum > 0.f ? sum * __expf(m - v) : 0.f) + 1.f;
      m = v;
    } else if (v > -INFINITY) {
      sum += __expf(v - m);
    }
    tk_insert<KP>(tv, ti, v, i);
  };
  const int i = lo + 8 * threadIdx.x;
  if (i + 8 <= hi) {
    const u32x4 p = *reinterpret_cast<const u32x4*>(lp + i);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      take(__uint_as_float(p[j] << 16), i + 2 * j);
      take(__uint_as_float(p[j] & 0xffff0000u), i + 2 * j + 1);
    }
  } else {
    for (int j = i; j < hi; ++j) take(bf16_to_f32(lp[j]), j);
  }
  __shared__ float s_v[(TK_NT / 64) * KP], s_m[TK_NT / 64], s_s[TK_NT / 64];
  __shared__ int s_i[(TK_NT / 64) * KP];
  tk_block_reduce<KP>(tv, ti, m, sum, s_v, s_i, s_m, s_s);
  if (threadIdx.x == 0) {
    const size_t o = (size_t)row * C + c;
#pragma unroll
    for (int k = 0; k < KP; ++k) { ws_v[o * 16 + k] = tv[k]; ws_i[o * 16 + k] = ti[k]; }
    ws_ms[2 * o] = m;
    ws_ms[2 * o + 1] = sum;
  }
}

template <int KP>
__global__ __launch_bounds__(TK_NT) void topk_lse_final_kernel(int C, int K, const float* __restrict__ ws_v,
                                                               const int* __restrict__ ws_i,
                                                               const float* __restrict__ ws_ms,
                                                               float* __restrict__ out_v,
                                                               long long* __restrict__ out_i) {
  const int row = blockIdx.x;
  float tv[KP];
  int ti[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) { tv[k] = -INFINITY; ti[k] = 0x7fffffff; }
  float m = -INFINITY, sum = 0.f;
  for (int cc = threadIdx.x; cc < C; cc += TK_NT) {      // one chunk's list per thread
    const size_t o = (size_t)row * C + cc;
    float ov[KP];
    int oi[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) { ov[k] = ws_v[o * 16 + k]; oi[k] = ws_i[o * 16 + k]; }
    tk_merge2<KP>(tv, ti, ov, oi);
    const float om = ws_ms[2 * o], os = ws_ms[2 * o + 1];
    const float nm = fmaxf(m, om);
    sum = (sum > 0.f ? sum * __expf(m - nm) : 0.f) + (os > 0.f ? os * __expf(om - nm) : 0.f);
    m = nm;
  }
  __shared__ float s_v[(TK_NT / 64) * KP], s_m[TK_NT / 64], s_s[TK_NT / 64];
  __shared__ int s_i[(TK_NT / 64) * KP];
  tk_block_reduce<KP>(tv, ti, m, sum, s_v, s_i, s_m, s_s);
  if (threadIdx.x == 0) {
    const float lse = m + __logf(sum);
    for (int k = 0; k < K; ++k) {
      out_v[(size_t)row * K + k] = tv[k] - lse;
      out_i[(size_t)row * K + k] = ti[k];
    }
  }
}

// ---------------------------------------------------------------------------
// top-k / top-p (nucleus) cut as one logit threshold per row.
//
// With u > t "strictly greater", an element v is kept iff
//   #{u > v} < top_k   and   sum_{u > v} exp((u - max) / T) <= top_p * Z_k
// (HF / vLLM order: temperature, then top-k, then top-p over the top-k
// survivors renormalised: Z_k is the mass of {v : #{u > v} < top_k}, found by a
// count-only search first).  Both sides are monotone in v, so the kept set is
// {v >= v*}.  v* is bracketed by a 16-way interval search
// over [min, max]: every pass streams the row once and evaluates the count and
// mass above 16 candidate cuts in registers (no sort, no atomics, no
// materialised softmax), so a 128k-vocab row costs at most NPASS + 2 L2-resident scans (bf16 rows
// usually stop after 3 passes, once the interval is narrower than one bf16 ulp).
// The sampler then skips v < thresh.  Ties at the cut are all kept; when the
// final interval still holds several distinct values (fp32 logits closer than
// range / 16^NPASS) the cut keeps all of them — a superset by construction.
constexpr int NCUT = 16;
constexpr int NPASS = 6;

template <int N>
__device__ __forceinline__ void block_sum(float (&v)[N], float* red /* [16][N] */) {
#pragma unroll
  for (int j = 0; j < N; ++j)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[j] += __shfl_xor(v[j], o, 64);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int j = 0; j < N; ++j) red[w * N + j] = v[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < N; ++j) {
    float a = 0.f;
    for (int k = 0; k < nw; ++k) a += red[k * N + j];
    v[j] = a;
  }
}

__device__ __forceinline__ float block_minmax(float v, bool is_max, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float u = __shfl_xor(v, o, 64);
    v = is_max ? fmaxf(v, u) : fminf(v, u);
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float a = red[0];
  for (int k = 1; k < nw; ++k) a = is_max ? fmaxf(a, red[k]) : fminf(a, red[k]);
  return a;
}

template <typename T>
__global__ __launch_bounds__(1024) void topkp_thresh_kernel(const T* __restrict__ logits, int V, int stride,
                                                            const float* __restrict__ temperature,
                                                            const long long* __restrict__ top_k,
                                                            const float* __restrict__ top_p,
                                                            float* __restrict__ thresh) {
  __shared__ float red[16 * (2 * NCUT + 1)];
  const int row = blockIdx.x;
  const T* lp = logits + (size_t)row * stride;
  const float temp = temperature ? temperature[row] : 1.f;
  const long long kraw = top_k ? top_k[row] : 0;
  const float p = top_p ? top_p[row] : 1.f;
  const long long kk = (kraw <= 0 || kraw > V) ? (long long)V : kraw;
  if (temp <= 1e-5f || (kk >= V && p >= 1.f)) {  // greedy or no filter
    if (threadIdx.x == 0) thresh[row] = -INFINITY;
    return;
  }
  const float sc = 1.4426950408889634f / temp;  // exp((u - max) / T) = exp2((u - max) * sc)
  constexpr float kRel = sizeof(T) == 2 ? 1.f / 512.f : 1.f / 33554432.f;

  float vmax = -INFINITY, vmin = INFINITY;
  scan_row<T>(lp, V, stride, [&](float v, int) {
    if (v > -INFINITY && v < INFINITY) { vmax = fmaxf(vmax, v); vmin = fminf(vmin, v); }
  });
  vmax = block_minmax(vmax, true, red);
  vmin = block_minmax(vmin, false, red);
  if (!(vmax > vmin)) {  // constant (or empty) row: nothing to cut
    if (threadIdx.x == 0) thresh[row] = -INFINITY;
    return;
  }
  // ---- top-k cut (count-only interval search): the nucleus is renormalised over it
  float kcut = -INFINITY;
  if (kk < V) {
    float lo = vmin, hi = vmax;
    bool keep_all = false;
    for (int pass = 0; pass < NPASS; ++pass) {
      const float step = (hi - lo) * (1.f / NCUT);
      float cnt[NCUT];
#pragma unroll
      for (int j = 0; j < NCUT; ++j) cnt[j] = 0.f;
      scan_row<T>(lp, V, stride, [&](float v, int) {
        if (!(v > lo)) return;
#pragma unroll
        for (int j = 0; j < NCUT; ++j) cnt[j] += v > lo + step * j ? 1.f : 0.f;
      });
      block_sum<NCUT>(cnt, red);
      if (pass == 0 && cnt[0] < (float)kk) { keep_all = true; break; }   // top-k keeps every element
      int jl = 0;
#pragma unroll
      for (int j = 1; j < NCUT; ++j)
        if (!(cnt[j] < (float)kk)) jl = j;
      const float nlo = lo + step * jl;
      hi = (jl == NCUT - 1) ? hi : lo + step * (jl + 1);
      lo = nlo;
      if (!(hi > lo) || (hi - lo) < fminf(fabsf(lo), fabsf(hi)) * kRel) break;
    }
    if (!keep_all) {
      float vk = INFINITY;
      scan_row<T>(lp, V, stride, [&](float v, int) {
        if (v > lo && v <= hi) vk = fminf(vk, v);
      });
      vk = block_minmax(vk, false, red);
      kcut = vk < INFINITY ? vk : hi;
    }
  }

  float lo = vmin, hi = vmax, pz = 0.f;
  for (int pass = 0; pass < NPASS; ++pass) {
    const float step = (hi - lo) * (1.f / NCUT);
    float acc[2 * NCUT + 1];  // counts | masses | Z
#pragma unroll
    for (int j = 0; j < 2 * NCUT + 1; ++j) acc[j] = 0.f;
    float z = 0.f;
    scan_row<T>(lp, V, stride, [&](float v, int) {
      if (pass == 0 && v >= kcut && v < INFINITY) z += exp2f((v - vmax) * sc);   // Z_k
      if (!(v > lo)) return;  // never above any cut of this pass (and not -inf / NaN)
      const float e = exp2f((fminf(v, vmax) - vmax) * sc);
#pragma unroll
      for (int j = 0; j < NCUT; ++j) {
        const bool gt = v > lo + step * j;
        acc[j] += gt ? 1.f : 0.f;
        acc[NCUT + j] += gt ? e : 0.f;
      }
    });
    acc[2 * NCUT] = z;
    block_sum<2 * NCUT + 1>(acc, red);
    if (pass == 0) {
      pz = p * acc[2 * NCUT];
      // cut 0 is vmin itself: if it passes, every finite element is kept
      if (acc[0] < (float)kk && acc[NCUT] <= pz) {
        if (threadIdx.x == 0) thresh[row] = -INFINITY;
        return;
      }
    }
    int jl = 0;  // largest failing cut (cut 0 == lo always fails)
#pragma unroll
    for (int j = 1; j < NCUT; ++j)
      if (!(acc[j] < (float)kk && acc[NCUT + j] <= pz)) jl = j;
    const float nlo = lo + step * jl;
    hi = (jl == NCUT - 1) ? hi : lo + step * (jl + 1);
    lo = nlo;
    // stop once (lo, hi] can hold at most one representable value of T
    // (bf16: 8-bit mantissa, spacing >= |x| 2^-8 > width; fp32 rarely gets here)
    if (!(hi > lo) || (hi - lo) < fminf(fabsf(lo), fabsf(hi)) * kRel) break;
  }
  // v* = smallest element value in (lo, hi]
  float vs = INFINITY;
  scan_row<T>(lp, V, stride, [&](float v, int) {
    if (v > lo && v <= hi) vs = fminf(vs, v);
  });
  vs = block_minmax(vs, false, red);
  if (threadIdx.x == 0) thresh[row] = vs < INFINITY ? vs : hi;
}

}  // namespace

// floats of workspace dgi_sample's split path needs for B rows of V logits (0: no split)
extern "C" int dgi_sample_ws_floats(int B, int V) {
  if (B > 32 || V < 2 * SP_CHUNK) return 0;
  return 2 * B * ((V + SP_CHUNK - 1) / SP_CHUNK);
}

extern "C" int dgi_sample(const void* logits, int is_bf16, int B, int V, int stride,
                          const float* temperature, const long long* seeds, long long step,
                          const float* thresh, long long* out, void* ws, hipStream_t s) {
  if (B == 0) return 0;
  if (ws && dgi_sample_ws_floats(B, V) > 0) {
    const int C = (V + SP_CHUNK - 1) / SP_CHUNK;
    float* pv = reinterpret_cast<float*>(ws);
    int* pi = reinterpret_cast<int*>(pv + (size_t)B * C);
    const dim3 grid(C, B);
    if (is_bf16)
      sample_part_kernel<uint16_t><<<grid, SP_NT, 0, s>>>((const uint16_t*)logits, V, stride, temperature, seeds,
                                                         step, thresh, pv, pi);
    else
      sample_part_kernel<float><<<grid, SP_NT, 0, s>>>((const float*)logits, V, stride, temperature, seeds, step,
                                                      thresh, pv, pi);
    DGI_CHECK_LAUNCH();
    sample_final_kernel<<<B, 64, 0, s>>>(pv, pi, C, out);
    DGI_CHECK_LAUNCH();
    return 0;
  }
  if (is_bf16)
    sample_kernel<uint16_t><<<B, 1024, 0, s>>>((const uint16_t*)logits, V, stride, temperature, seeds, step,
                                               thresh, out);
  else
    sample_kernel<float><<<B, 1024, 0, s>>>((const float*)logits, V, stride, temperature, seeds, step, thresh,
                                            out);
  DGI_CHECK_LAUNCH();
  return 0;
}

extern "C" int dgi_topk(const void* logits, int is_bf16, int B, int V, int stride, int K,
                        float* out_v, long long* out_i, hipStream_t s) {
  if (B == 0) return 0;
  if (K < 1 || K > 16) return -2;
  if (is_bf16)
    topk_kernel<uint16_t><<<B, 256, 0, s>>>((const uint16_t*)logits, V, stride, K, out_v, out_i);
  else
    topk_kernel<float><<<B, 256, 0, s>>>((const float*)logits, V, stride, K, out_v, out_i);
  DGI_CHECK_LAUNCH();
  return 0;
}

// workspace: (B * C * 16) floats + (B * C * 16) ints + (B * C * 2) floats, C = ceil(V / TK_CHUNK)
extern "C" int dgi_topk_logprobs_ws_floats(int B, int V) {
  const int C = (V + TK_CHUNK - 1) / TK_CHUNK;
  return B * C * (16 + 16 + 2);
}

extern "C" int dgi_topk_logprobs(const void* logits, int B, int V, int stride, int K, float* ws, float* out_v,
                                 long long* out_i, hipStream_t s) {
  if (B == 0) return 0;
  if (K < 1 || K > 8) return -2;     // wider draft expansions use log_softmax + topk_kernel
  if (stride % 8 || V < 1) return -3;
  const int C = (V + TK_CHUNK - 1) / TK_CHUNK;
  float* ws_v = ws;
  int* ws_i = reinterpret_cast<int*>(ws + (size_t)B * C * 16);
  float* ws_ms = ws + (size_t)B * C * 32;
#define DGI_TKL(KPV)                                                                                         \
  topk_lse_part_kernel<KPV><<<dim3(C, B), TK_NT, 0, s>>>((const uint16_t*)logits, V, stride, ws_v, ws_i, ws_ms); \
  DGI_CHECK_LAUNCH();                                                                                         \
  topk_lse_final_kernel<KPV><<<B, TK_NT, 0, s>>>(C, K, ws_v, ws_i, ws_ms, out_v, out_i);                      \
  DGI_CHECK_LAUNCH();
  if (K <= 1) { DGI_TKL(1) } else if (K <= 2) { DGI_TKL(2) } else if (K <= 4) { DGI_TKL(4) } else { DGI_TKL(8) }
#undef DGI_TKL
  return 0;
}

extern "C" int dgi_topkp_threshold(const void* logits, int is_bf16, int B, int V, int stride,
                                   const float* temperature, const long long* top_k, const float* top_p,
                                   float* thresh, hipStream_t s) {
  if (B == 0) return 0;
  if (V < 1) return -2;
  if (is_bf16)
    topkp_thresh_kernel<uint16_t><<<B, 1024, 0, s>>>((const uint16_t*)logits, V, stride, temperature, top_k,
                                                     top_p, thresh);
  else
    topkp_thresh_kernel<float><<<B, 1024, 0, s>>>((const float*)logits, V, stride, temperature, top_k, top_p,
                                                  thresh);
  DGI_CHECK_LAUNCH();
  return 0;
}
