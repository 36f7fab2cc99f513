// dgi/csrc/tree.hip — EAGLE draft-tree mask and verification.
//
// The reference builds the tree attention mask with an O(N*depth) Python loop
// (worker/engines/speculative.py:184-213), compares target logits at node i
// with draft token i (off by one, :419-454) and traces the accepted path on
// the host (:215-245).  Here both steps run on device, one wave per sequence,
// with the tree held as a parent array (node 0 = the root = last accepted
// token, parent[n] < n for n > 0, at most 64 nodes):
//   tree_mask   : anc[n] = bitmask of ancestors-or-self of n  (feeds the
//                 tree mode of prefill_attention.hip)
//   tree_verify : node n (n>0) matches iff draft[n] == target_argmax[parent[n]];
//                 it is accepted iff every ancestor-or-self except the root
//                 matches: (anc[n] & ~match) == 0.  The deepest accepted node
//                 (ties -> lowest index) gives the path; the bonus token is
//                 target_argmax at that node.  Outputs accept length, the path
//                 node ids (for KV compaction) and the accepted token ids.
#include "common.h"

using namespace dgi;

namespace {

__global__ __launch_bounds__(64) void tree_mask_kernel(const int* __restrict__ parent, int N,
                                                       unsigned long long* __restrict__ anc,
                                                       int* __restrict__ depth) {
  const int b = blockIdx.x;
  const int n = threadIdx.x;
  if (n >= N) return;
  const int* par = parent + (size_t)b * N;
  unsigned long long m = 1ull << n;
  int d = 0;
  int p = par[n];
  while (p >= 0 && d < 64) { m |= 1ull << p; p = par[p]; ++d; }
  anc[(size_t)b * 64 + n] = m;
  if (depth) depth[(size_t)b * N + n] = d;
}

__global__ __launch_bounds__(64) void tree_verify_kernel(
    const int* __restrict__ parent, const long long* __restrict__ draft,
    const long long* __restrict__ target, int N, const unsigned long long* __restrict__ anc,
    const int* __restrict__ depth, int* __restrict__ accept_len, int* __restrict__ path,
    long long* __restrict__ out_tokens, int max_path) {
  const int b = blockIdx.x;
  const int n = threadIdx.x;
  const bool live = n < N;
  const int* par = parent + (size_t)b * N;
  bool match = false;
  if (live) {
    if (n == 0) match = true;
    else match = draft[(size_t)b * N + n] == target[(size_t)b * N + par[n]];
  }
  const unsigned long long match_bits = __ballot(match);
  unsigned long long a = live ? anc[(size_t)b * 64 + n] : 0ull;
  const bool ok = live && ((a & ~match_bits) == 0ull);
  const int d = live ? depth[(size_t)b * N + n] : -1;
  // deepest accepted node, lowest index on ties: key = d * 64 + (63 - n)
  int key = ok ? d * 64 + (63 - n) : -1;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) key = max(key, __shfl_xor(key, o, 64));
  const int best = 63 - (key & 63);
  const int bd = key >> 6;
  if (n == 0) {
    accept_len[b] = bd;  // number of accepted draft tokens (root excluded)
    // path from root to best; fill from the leaf upwards
    int node = best;
    for (int k = bd; k >= 0; --k) {
      if (k < max_path) {
        path[(size_t)b * max_path + k] = node;
        // accepted token at depth k is draft[node] (k>0); the bonus follows
        if (k > 0) out_tokens[(size_t)b * (max_path + 1) + k - 1] = draft[(size_t)b * N + node];
      }
      node = node > 0 ? par[node] : 0;
    }
    if (bd < max_path + 1) out_tokens[(size_t)b * (max_path + 1) + bd] = target[(size_t)b * N + best];
  }
}

}  // namespace

extern "C" int dgi_tree_mask(const int* parent, int B, int N, unsigned long long* anc, int* depth,
                             hipStream_t s) {
  if (B == 0) return 0;
  if (N > 64) return -2;
  tree_mask_kernel<<<B, 64, 0, s>>>(parent, N, anc, depth);
  DGI_CHECK_LAUNCH();
  return 0;
}

extern "C" int dgi_tree_verify(const int* parent, const long long* draft, const long long* target,
                               int B, int N, const unsigned long long* anc, const int* depth,
                               int* accept_len, int* path, long long* out_tokens, int max_path,
                               hipStream_t s) {
  if (B == 0) return 0;
  if (N > 64) return -2;
  tree_verify_kernel<<<B, 64, 0, s>>>(parent, draft, target, N, anc, depth, accept_len, path,
                                      out_tokens, max_path);
  DGI_CHECK_LAUNCH();
  return 0;
}
