// dgi/csrc/bindings.cpp — registers the gfx950 kernels as torch.ops.dgi.*.
//
// Every op launches on the current HIP stream and allocates nothing, so the
// whole decode step can be captured into a hipGraph (torch.cuda.CUDAGraph on
// ROCm).  Shapes are checked here, on the host, before any launch: a kernel
// never sees operands that disagree with its grid.
#include <cstdlib>
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

extern "C" {
int dgi_rmsnorm(void* out, const void* x, const void* w, int T, int H, float eps, hipStream_t s);
int dgi_fused_add_rmsnorm(void* x, void* residual, const void* w, int T, int H, float eps,
                          hipStream_t s);
int dgi_rope_cache(void* qkv, int T, int qkv_stride, const int* positions, const float* cos_sin,
                   int nh, int nkv, int hd, int rd, int mode, const int* slot_mapping, void* k_cache,
                   void* v_cache, int block_size, hipStream_t s);
int dgi_paged_decode(const void* q, int q_stride, const void* k_cache, const void* v_cache,
                     const int* block_tables, int bt_stride, const int* context_lens, void* out,
                     int out_stride, float* part_o, float* part_lse, int* counters, int B, int nh, int nkv,
                     int hd, int block_size, int max_splits, int part_size, float scale, hipStream_t s);
int dgi_paged_prefill(const void* q, int q_stride, const void* k_cache, const void* v_cache,
                      const int* block_tables, int bt_stride, const int* cu_seqlens_q,
                      const int* context_lens, const int* tiles, int n_tiles, void* out,
                      int out_stride, int nh, int nkv, int hd, int block_size, float scale,
                      const unsigned long long* tree_mask, int tree_n, int tile_rows, hipStream_t s);
int dgi_silu_mul(const void* gu, void* out, int T, int I, hipStream_t s);
int dgi_skinny_gemm(const void* x, int ldx, const void* w, const void* bias, void* y, int ldy, int M,
                    int N, int K, int nw, hipStream_t s);
int dgi_mfma_gemm(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int epi,
                  hipStream_t s);
void dgi_set_gemm_cus(int cus);
int dgi_gemm_split_timeouts(int reset);
int dgi_mfma_gemm_norm(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int kind,
                       float* ss, int ss_ld, float inv_k, float eps, int phases, hipStream_t s);
int dgi_mfma_gemm_norm_rope(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, float* ss,
                            int ss_ld, float inv_k, float eps, const int* pos, const float* cos_sin, const int* slots,
                            void* k_cache, void* v_cache, int nh, int nkv, int block_size, int phases, hipStream_t s);
int dgi_fused_skinny(const void* x, int ldx, const void* res, int ldr, void* res_out, const void* gamma,
                     float eps, const void* w, const void* bias, void* y, int ldy, int M, int N, int K, int pro,
                     int epi, const int* positions, const float* cos_sin, const int* slots, void* k_cache,
                     void* v_cache, int nh, int nkv, int block_size, int cfg, hipStream_t s);
int dgi_sample(const void* logits, int is_bf16, int B, int V, int stride, const float* temperature,
               const long long* seeds, long long step, const float* thresh, long long* out, void* ws, hipStream_t s);
int dgi_sample_ws_floats(int B, int V);
int dgi_topkp_threshold(const void* logits, int is_bf16, int B, int V, int stride, const float* temperature,
                        const long long* top_k, const float* top_p, float* thresh, hipStream_t s);
int dgi_topk(const void* logits, int is_bf16, int B, int V, int stride, int K, float* out_v,
             long long* out_i, hipStream_t s);
int dgi_topk_logprobs_ws_floats(int B, int V);
int dgi_topk_logprobs(const void* logits, int B, int V, int stride, int K, float* ws, float* out_v,
                      long long* out_i, hipStream_t s);
int dgi_kv_gather(const void* cache, const int* ids, int n, int LK, int num_blocks, int page_elems,
                  void* buf, int block_major, hipStream_t s);
int dgi_kv_scatter(void* cache, const int* ids, int n, int LK, int num_blocks, int page_elems,
                   const void* buf, int block_major, hipStream_t s);
int dgi_mall_prefetch(const void* base, const int* rows, int nrows, int row_bytes, int blocks, void* sink,
                      hipStream_t s);
int dgi_kv_slot_copy(void* cache, const int* src, const int* dst, int n, int LK, int num_blocks, int nkv, int bs,
                     int hd, void* buf, hipStream_t s);
int dgi_kv_copy(void* cache, const int* src, const int* dst, int n, int LK, int num_blocks,
                int page_elems, hipStream_t s);
int dgi_tree_mask(const int* parent, int B, int N, unsigned long long* anc, int* depth,
                  hipStream_t s);
int dgi_tree_verify(const int* parent, const long long* draft, const long long* target, int B,
                    int N, const unsigned long long* anc, const int* depth, int* accept_len,
                    int* path, long long* out_tokens, int max_path, hipStream_t s);
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "dgi kernel ", what, " failed with code ", rc,
              rc > 0 ? (std::string(" (") + hipGetErrorString((hipError_t)rc) + ")") : std::string());
}

void check_dev(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
}
void check_bf16(const at::Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16");
}
void check_i32(const at::Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kInt, name, " must be int32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void rmsnorm(at::Tensor out, const at::Tensor& x, const at::Tensor& w, double eps) {
  check_bf16(out, "out"); check_bf16(x, "x"); check_bf16(w, "w");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && w.is_contiguous());
  const int H = (int)x.size(-1);
  TORCH_CHECK(w.numel() == H && out.numel() == x.numel());
  check_rc(dgi_rmsnorm(out.data_ptr(), x.data_ptr(), w.data_ptr(), (int)(x.numel() / H), H,
                       (float)eps, cur_stream()), "rmsnorm");
}

void fused_add_rmsnorm(at::Tensor x, at::Tensor residual, const at::Tensor& w, double eps) {
  check_bf16(x, "x"); check_bf16(residual, "residual"); check_bf16(w, "w");
  TORCH_CHECK(x.is_contiguous() && residual.is_contiguous() && w.is_contiguous());
  const int H = (int)x.size(-1);
  TORCH_CHECK(w.numel() == H && residual.numel() == x.numel());
  check_rc(dgi_fused_add_rmsnorm(x.data_ptr(), residual.data_ptr(), w.data_ptr(),
                                 (int)(x.numel() / H), H, (float)eps, cur_stream()),
           "fused_add_rmsnorm");
}

// k_cache / v_cache: [num_blocks, nkv, bs, hd] (contiguous per-layer views)
// cos_sin: [max_pos, rd] fp32 (rd/2 cos | rd/2 sin); rd = rotary dims (<= hd);
// mode 0 = NeoX pairing, 1 = interleaved (GPT-J / GLM)
void rope_cache(at::Tensor qkv, const at::Tensor& positions, const at::Tensor& cos_sin, int64_t nh,
                int64_t nkv, int64_t hd, const at::Tensor& slot_mapping, at::Tensor k_cache,
                at::Tensor v_cache, int64_t mode) {
  check_bf16(qkv, "qkv"); check_i32(positions, "positions"); check_i32(slot_mapping, "slot_mapping");
  check_bf16(k_cache, "k_cache"); check_bf16(v_cache, "v_cache");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() && cos_sin.size(1) <= hd);
  TORCH_CHECK(positions.numel() == 0 || cos_sin.dim() == 2);
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1 && qkv.size(1) >= (nh + 2 * nkv) * hd);
  TORCH_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous());
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == nkv && k_cache.size(3) == hd);
  const int T = (int)qkv.size(0);
  TORCH_CHECK(positions.numel() == T && slot_mapping.numel() == T);
  check_rc(dgi_rope_cache(qkv.data_ptr(), T, (int)qkv.stride(0), positions.data_ptr<int>(),
                          cos_sin.data_ptr<float>(), (int)nh, (int)nkv, (int)hd, (int)cos_sin.size(1),
                          (int)mode, slot_mapping.data_ptr<int>(), k_cache.data_ptr(), v_cache.data_ptr(),
                          (int)k_cache.size(2), cur_stream()),
           "rope_cache");
}

// q: [B, >= nh*hd] rows (row stride = q.stride(0)); out: [B, nh*hd]
void paged_decode(at::Tensor out, const at::Tensor& q, const at::Tensor& k_cache,
                  const at::Tensor& v_cache, const at::Tensor& block_tables,
                  const at::Tensor& context_lens, at::Tensor part_o, at::Tensor part_lse,
                  int64_t nh, int64_t nkv, int64_t max_splits, int64_t part_size, double scale,
                  const c10::optional<at::Tensor>& counters) {
  check_bf16(out, "out"); check_bf16(q, "q"); check_bf16(k_cache, "k_cache"); check_bf16(v_cache, "v_cache");
  check_i32(block_tables, "block_tables"); check_i32(context_lens, "context_lens");
  TORCH_CHECK(q.dim() == 2 && q.stride(1) == 1 && out.dim() == 2 && out.stride(1) == 1);
  const int hd = (int)k_cache.size(3);
  const int B = (int)q.size(0);
  TORCH_CHECK(q.size(1) >= nh * hd && out.size(1) >= nh * hd && out.size(0) == B);
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) >= B && context_lens.numel() >= B);
  TORCH_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous() && k_cache.size(1) == nkv);
  if (max_splits > 1) {
    TORCH_CHECK(part_o.scalar_type() == at::kFloat && part_lse.scalar_type() == at::kFloat);
    TORCH_CHECK(part_o.numel() >= (int64_t)B * nh * max_splits * hd);
    TORCH_CHECK(part_lse.numel() >= (int64_t)B * nh * max_splits);
  }
  int* cnt = nullptr;
  if (counters.has_value() && counters->defined() && max_splits > 1) {
    check_i32(*counters, "counters");
    TORCH_CHECK(counters->numel() >= (int64_t)B * nkv, "paged_decode: counters need B * nkv zeros");
    cnt = counters->data_ptr<int>();
  }
  check_rc(dgi_paged_decode(q.data_ptr(), (int)q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                            block_tables.data_ptr<int>(), (int)block_tables.stride(0),
                            context_lens.data_ptr<int>(), out.data_ptr(), (int)out.stride(0),
                            max_splits > 1 ? part_o.data_ptr<float>() : nullptr,
                            max_splits > 1 ? part_lse.data_ptr<float>() : nullptr, cnt, B, (int)nh,
                            (int)nkv, hd, (int)k_cache.size(2), (int)max_splits, (int)part_size,
                            (float)scale, cur_stream()),
           "paged_decode");
}

void paged_prefill(at::Tensor out, const at::Tensor& q, const at::Tensor& k_cache,
                   const at::Tensor& v_cache, const at::Tensor& block_tables,
                   const at::Tensor& cu_seqlens_q, const at::Tensor& context_lens,
                   const at::Tensor& tiles, int64_t nh, int64_t nkv, double scale,
                   const c10::optional<at::Tensor>& tree_mask, int64_t tree_n, int64_t tile_rows) {
  check_bf16(out, "out"); check_bf16(q, "q"); check_bf16(k_cache, "k_cache"); check_bf16(v_cache, "v_cache");
  check_i32(block_tables, "block_tables"); check_i32(cu_seqlens_q, "cu_seqlens_q");
  check_i32(context_lens, "context_lens"); check_i32(tiles, "tiles");
  TORCH_CHECK(q.dim() == 2 && q.stride(1) == 1 && out.dim() == 2 && out.stride(1) == 1);
  const int hd = (int)k_cache.size(3);
  TORCH_CHECK(q.size(1) >= nh * hd && out.size(1) >= nh * hd && out.size(0) == q.size(0));
  TORCH_CHECK(tiles.dim() == 2 && tiles.size(1) == 2);
  TORCH_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous() && k_cache.size(1) == nkv);
  const unsigned long long* tm = nullptr;
  if (tree_mask.has_value() && tree_mask->defined()) {
    TORCH_CHECK(tree_mask->scalar_type() == at::kLong && tree_mask->is_contiguous());
    TORCH_CHECK(tree_mask->size(-1) == 64 && tree_mask->numel() >= 64 * (cu_seqlens_q.numel() - 1));
    tm = reinterpret_cast<const unsigned long long*>(tree_mask->data_ptr<int64_t>());
  }
  check_rc(dgi_paged_prefill(q.data_ptr(), (int)q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                             block_tables.data_ptr<int>(), (int)block_tables.stride(0),
                             cu_seqlens_q.data_ptr<int>(), context_lens.data_ptr<int>(),
                             tiles.data_ptr<int>(), (int)tiles.size(0), out.data_ptr(),
                             (int)out.stride(0), (int)nh, (int)nkv, hd, (int)k_cache.size(2),
                             (float)scale, tm, (int)tree_n, (int)tile_rows, cur_stream()),
           "paged_prefill");
}

void silu_mul(at::Tensor out, const at::Tensor& gu) {
  check_bf16(out, "out"); check_bf16(gu, "gu");
  TORCH_CHECK(gu.is_contiguous() && out.is_contiguous());
  const int I = (int)out.size(-1);
  TORCH_CHECK(gu.size(-1) == 2 * I && gu.numel() == 2 * out.numel());
  check_rc(dgi_silu_mul(gu.data_ptr(), out.data_ptr(), (int)(out.numel() / I), I, cur_stream()),
           "silu_mul");
}

void skinny_gemm(at::Tensor out, const at::Tensor& x, const at::Tensor& w,
                 const c10::optional<at::Tensor>& bias, int64_t cfg) {
  check_bf16(out, "out"); check_bf16(x, "x"); check_bf16(w, "w");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "skinny_gemm: 2-D operands");
  TORCH_CHECK(x.stride(1) == 1 && out.stride(1) == 1 && w.is_contiguous(), "skinny_gemm: row-major operands");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && out.size(0) == M && out.size(1) == N, "skinny_gemm: shape mismatch");
  TORCH_CHECK(M <= 32 && K % 1024 == 0 && N % 16 == 0 && x.stride(0) % 8 == 0, "skinny_gemm: M<=32, K%1024, N%16");
  const void* b = nullptr;
  if (bias.has_value()) {
    check_bf16(*bias, "bias");
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == N);
    b = bias->data_ptr();
  }
  check_rc(dgi_skinny_gemm(x.data_ptr(), (int)x.stride(0), w.data_ptr(), b, out.data_ptr(), (int)out.stride(0),
                           (int)M, (int)N, (int)K, (int)cfg, cur_stream()),
           "skinny_gemm");
}

// LDS-tiled MFMA GEMM (prefill / mixed steps): epi 0 out = x w^T; epi 1 out = SwiGLU with w = [gate; up].
void mfma_gemm(at::Tensor out, const at::Tensor& x, const at::Tensor& w, int64_t epi) {
  check_bf16(out, "out"); check_bf16(x, "x"); check_bf16(w, "w");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "mfma_gemm: 2-D operands");
  TORCH_CHECK(x.device() == w.device() && x.device() == out.device(), "mfma_gemm: operands on one device");
  TORCH_CHECK(x.stride(1) == 1 && out.stride(1) == 1 && w.is_contiguous(), "mfma_gemm: row-major operands");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && out.size(0) == M, "mfma_gemm: shape mismatch");
  TORCH_CHECK((epi & 15) <= 1 && ((epi >> 4) & 15) <= 4 && ((epi >> 8) & 3) <= 2 && ((epi >> 10) & 3) <= 2 && (epi >> 15) == 0,
              "mfma_gemm: epi 0 (store) or 1 (SwiGLU), + 16 * schedule + 256 * stream-K mode");
  TORCH_CHECK(((epi >> 4) & 15) != 4 || (epi & 15) == 0, "mfma_gemm: schedule 4 (half tile) is a plain GEMM");
  TORCH_CHECK(out.size(1) == ((epi & 15) == 1 ? N / 2 : N), "mfma_gemm: output columns");
  TORCH_CHECK(N % 256 == 0 && K % 64 == 0 && x.stride(0) % 8 == 0 && out.stride(0) % 4 == 0,
              "mfma_gemm: N%256, K%64, ldx%8, ldy%4");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(out.data_ptr()) % 8 == 0, "mfma_gemm: operand alignment");
  TORCH_CHECK((int64_t)M * x.stride(0) < (1LL << 31), "mfma_gemm: activation too large for 32-bit offsets");
  check_rc(dgi_mfma_gemm(x.data_ptr(), (int)x.stride(0), w.data_ptr(), out.data_ptr(), (int)out.stride(0), (int)M,
                         (int)N, (int)K, (int)epi, cur_stream()),
           "mfma_gemm");
}

// Fused-RMSNorm MFMA GEMMs (ping-pong schedule, dgi/csrc/mfma_gemm.hip): kind 2 residual
// (out += x w^T in place, per-row partial sums of squares -> ss[:, N / 256]); 3 out = rstd * x w^T;
// 4 out = SwiGLU(rstd * x [gate; up]^T); rstd = rsqrt(sum(ss[m, :]) * inv_k + eps).
void mfma_gemm_norm(at::Tensor out, const at::Tensor& x, const at::Tensor& w, int64_t kind, at::Tensor ss,
                    double inv_k, double eps, int64_t phases) {
  check_bf16(out, "out"); check_bf16(x, "x"); check_bf16(w, "w");
  TORCH_CHECK(ss.scalar_type() == at::kFloat && ss.dim() == 2 && ss.is_contiguous(), "mfma_gemm_norm: ss fp32 [M, n]");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "mfma_gemm_norm: 2-D operands");
  TORCH_CHECK(x.device() == w.device() && x.device() == out.device() && ss.device() == x.device(),
              "mfma_gemm_norm: operands on one device");
  TORCH_CHECK(x.stride(1) == 1 && out.stride(1) == 1 && w.is_contiguous(), "mfma_gemm_norm: row-major operands");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(kind >= 2 && kind <= 4, "mfma_gemm_norm: kind 2 (residual), 3 (norm), 4 (norm + SwiGLU)");
  TORCH_CHECK(w.size(1) == K && out.size(0) == M && ss.size(0) >= M, "mfma_gemm_norm: shape mismatch");
  TORCH_CHECK(out.size(1) == (kind == 4 ? N / 2 : N), "mfma_gemm_norm: output columns");
  TORCH_CHECK(kind != 2 || ss.size(1) >= N / 256, "mfma_gemm_norm: ss needs N / 256 columns");
  TORCH_CHECK(kind == 2 || (ss.size(1) % 8 == 0 && ss.size(1) <= 32), "mfma_gemm_norm: ss columns % 8, <= 32");
  TORCH_CHECK(N % 256 == 0 && K % 128 == 0 && K >= 256 && x.stride(0) % 8 == 0 && out.stride(0) % 4 == 0,
              "mfma_gemm_norm: N%256, K%128, ldx%8, ldy%4");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "mfma_gemm_norm: operand alignment");
  TORCH_CHECK((int64_t)M * x.stride(0) < (1LL << 31) && (int64_t)M * out.stride(0) < (1LL << 31),
              "mfma_gemm_norm: activation too large for 32-bit offsets");
  check_rc(dgi_mfma_gemm_norm(x.data_ptr(), (int)x.stride(0), w.data_ptr(), out.data_ptr(), (int)out.stride(0), (int)M,
                              (int)N, (int)K, (int)kind, ss.data_ptr<float>(), (int)ss.size(1), (float)inv_k,
                              (float)eps, (int)phases, cur_stream()),
           "mfma_gemm_norm");
}

// The normalised qkv projection with the RoPE + paged-KV epilogue (mfma_gemm.hip EPI 5).
void mfma_gemm_norm_rope(at::Tensor out, const at::Tensor& x, const at::Tensor& w, at::Tensor ss, double inv_k,
                         double eps, const at::Tensor& positions, const at::Tensor& cos_sin,
                         const at::Tensor& slot_mapping, at::Tensor k_cache, at::Tensor v_cache, int64_t nh,
                         int64_t nkv, int64_t phases) {
  check_bf16(out, "out"); check_bf16(x, "x"); check_bf16(w, "w"); check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  TORCH_CHECK(ss.scalar_type() == at::kFloat && ss.dim() == 2 && ss.is_contiguous() && ss.size(1) % 8 == 0 &&
              ss.size(1) <= 32, "mfma_gemm_norm_rope: ss fp32 [M, n], n % 8, <= 32");
  TORCH_CHECK(positions.scalar_type() == at::kInt && slot_mapping.scalar_type() == at::kInt &&
              positions.is_contiguous() && slot_mapping.is_contiguous(), "mfma_gemm_norm_rope: int32 positions / slots");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.dim() == 2 && cos_sin.size(1) == 128 &&
              cos_sin.is_contiguous(), "mfma_gemm_norm_rope: cos_sin fp32 [max_pos, 128]");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == nkv && k_cache.size(3) == 128 && k_cache.is_contiguous() &&
              v_cache.sizes() == k_cache.sizes() && v_cache.is_contiguous(),
              "mfma_gemm_norm_rope: caches [blocks, nkv, bs, 128]");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2 && x.stride(1) == 1 && out.stride(1) == 1 &&
              w.is_contiguous(), "mfma_gemm_norm_rope: row-major 2-D operands");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && out.size(0) == M && out.size(1) == N && ss.size(0) >= M &&
              positions.size(0) >= M && slot_mapping.size(0) >= M, "mfma_gemm_norm_rope: shape mismatch");
  TORCH_CHECK(N == (nh + 2 * nkv) * 128 && (nh * 128) % 256 == 0 && (nkv * 128) % 256 == 0,
              "mfma_gemm_norm_rope: fused qkv of 128-dim heads, head groups of 256 columns");
  TORCH_CHECK(K % 128 == 0 && K >= 256 && x.stride(0) % 8 == 0 && out.stride(0) % 8 == 0,
              "mfma_gemm_norm_rope: K%128, ldx%8, ldy%8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "mfma_gemm_norm_rope: operand alignment");
  TORCH_CHECK((int64_t)M * x.stride(0) < (1LL << 31) && (int64_t)M * out.stride(0) < (1LL << 31),
              "mfma_gemm_norm_rope: activation too large for 32-bit offsets");
  check_rc(dgi_mfma_gemm_norm_rope(x.data_ptr(), (int)x.stride(0), w.data_ptr(), out.data_ptr(), (int)out.stride(0),
                                   (int)M, (int)N, (int)K, ss.data_ptr<float>(), (int)ss.size(1), (float)inv_k,
                                   (float)eps, positions.data_ptr<int>(), cos_sin.data_ptr<float>(),
                                   slot_mapping.data_ptr<int>(), k_cache.data_ptr(), v_cache.data_ptr(), (int)nh,
                                   (int)nkv, (int)k_cache.size(2), (int)phases, cur_stream()),
           "mfma_gemm_norm_rope");
}

// Decode GEMM with fused RMSNorm prologue (pro 1: norm, 2: residual add + norm -> res_out) and
// epilogue (epi 0: store, 1: SwiGLU over the [gate; up] rows, 2: RoPE + paged KV write).
void fused_skinny(at::Tensor y, const at::Tensor& x, const c10::optional<at::Tensor>& res,
                  const c10::optional<at::Tensor>& res_out, const c10::optional<at::Tensor>& gamma, double eps,
                  const at::Tensor& w, const c10::optional<at::Tensor>& bias, int64_t pro, int64_t epi,
                  const c10::optional<at::Tensor>& positions, const c10::optional<at::Tensor>& cos_sin,
                  const c10::optional<at::Tensor>& slots, const c10::optional<at::Tensor>& k_cache,
                  const c10::optional<at::Tensor>& v_cache, int64_t nh, int64_t nkv, int64_t cfg) {
  check_bf16(y, "y"); check_bf16(x, "x"); check_bf16(w, "w");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 2, "fused_skinny: 2-D operands");
  TORCH_CHECK(x.stride(1) == 1 && y.stride(1) == 1 && w.is_contiguous() && x.stride(0) % 8 == 0);
  const int64_t M = x.size(0), K = x.size(1), R = w.size(0);
  TORCH_CHECK(w.size(1) == K && y.size(0) == M && M <= 16 && K % 1024 == 0, "fused_skinny: M<=16, K%1024");
  TORCH_CHECK(x.device() == w.device() && y.device() == w.device());
  int64_t N = R;
  if (epi == 1) {
    TORCH_CHECK(R % 2 == 0 && y.size(1) == R / 2, "fused_skinny: SwiGLU output is [M, I] for [2I, K] weights");
    N = R / 2;
  } else {
    TORCH_CHECK(y.size(1) == R, "fused_skinny: y must be [M, N]");
  }
  const void* rp = nullptr;
  void* rop = nullptr;
  int ldr = 0;
  const void* gp = nullptr;
  if (pro >= 1) {
    TORCH_CHECK(gamma.has_value() && gamma->defined());
    check_bf16(*gamma, "gamma");
    TORCH_CHECK(gamma->is_contiguous() && gamma->numel() == K);
    gp = gamma->data_ptr();
  }
  if (pro == 2) {
    TORCH_CHECK(res.has_value() && res_out.has_value() && res->defined() && res_out->defined());
    check_bf16(*res, "res"); check_bf16(*res_out, "res_out");
    TORCH_CHECK(res->sizes() == x.sizes() && res_out->sizes() == x.sizes() && res->stride(1) == 1 &&
                res_out->stride(1) == 1 && res->stride(0) == res_out->stride(0) && res->stride(0) % 8 == 0);
    TORCH_CHECK(res_out->data_ptr() != res->data_ptr() && res_out->data_ptr() != x.data_ptr(),
                "fused_skinny: res_out must not alias x or res");
    rp = res->data_ptr();
    rop = res_out->data_ptr();
    ldr = (int)res->stride(0);
  }
  const void* b = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_bf16(*bias, "bias");
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == R);
    b = bias->data_ptr();
  }
  const int* pos = nullptr;
  const float* cs = nullptr;
  const int* sl = nullptr;
  void* kc = nullptr;
  void* vc = nullptr;
  int bsz = 16;
  if (epi == 2) {
    TORCH_CHECK(positions.has_value() && cos_sin.has_value() && slots.has_value() && k_cache.has_value() &&
                v_cache.has_value());
    check_i32(*positions, "positions"); check_i32(*slots, "slots");
    check_bf16(*k_cache, "k_cache"); check_bf16(*v_cache, "v_cache");
    TORCH_CHECK(positions->numel() >= M && slots->numel() >= M);
    TORCH_CHECK(cos_sin->scalar_type() == at::kFloat && cos_sin->is_contiguous() && cos_sin->dim() == 2 &&
                cos_sin->size(1) == 128, "fused_skinny: RoPE epilogue needs full 128-dim rotary");
    TORCH_CHECK(k_cache->is_contiguous() && v_cache->is_contiguous() && k_cache->dim() == 4 &&
                k_cache->size(1) == nkv && k_cache->size(3) == 128 && v_cache->sizes() == k_cache->sizes());
    TORCH_CHECK(R == (nh + 2 * nkv) * 128);
    pos = positions->data_ptr<int>();
    cs = cos_sin->data_ptr<float>();
    sl = slots->data_ptr<int>();
    kc = k_cache->data_ptr();
    vc = v_cache->data_ptr();
    bsz = (int)k_cache->size(2);
  }
  check_rc(dgi_fused_skinny(x.data_ptr(), (int)x.stride(0), rp, ldr, rop, gp, (float)eps, w.data_ptr(), b,
                            y.data_ptr(), (int)y.stride(0), (int)M, (int)N, (int)K, (int)pro, (int)epi, pos, cs,
                            sl, kc, vc, (int)nh, (int)nkv, bsz, (int)cfg, cur_stream()),
           "fused_skinny");
}

void sample(at::Tensor out, const at::Tensor& logits, const c10::optional<at::Tensor>& temperature,
            const c10::optional<at::Tensor>& seeds, int64_t step, const c10::optional<at::Tensor>& thresh) {
  check_dev(logits, "logits");
  TORCH_CHECK(out.scalar_type() == at::kLong && out.is_contiguous());
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1);
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat);
  const int B = (int)logits.size(0);
  TORCH_CHECK(out.numel() >= B);
  const float* tp = nullptr;
  const long long* sp = nullptr;
  if (temperature.has_value() && temperature->defined()) {
    TORCH_CHECK(temperature->scalar_type() == at::kFloat && temperature->numel() >= B &&
                temperature->is_contiguous() && temperature->device() == logits.device());
    tp = temperature->data_ptr<float>();
  }
  if (seeds.has_value() && seeds->defined()) {
    TORCH_CHECK(seeds->scalar_type() == at::kLong && seeds->numel() >= B && seeds->is_contiguous() &&
                seeds->device() == logits.device());
    sp = reinterpret_cast<const long long*>(seeds->data_ptr<int64_t>());
  }
  const float* thp = nullptr;
  if (thresh.has_value() && thresh->defined()) {
    TORCH_CHECK(thresh->scalar_type() == at::kFloat && thresh->numel() >= B && thresh->is_contiguous() &&
                thresh->device() == logits.device());
    thp = thresh->data_ptr<float>();
  }
  // small batches split each row over several workgroups (DGI_SAMPLE_SPLIT=0: one per row)
  static const bool split = [] {
    const char* e = std::getenv("DGI_SAMPLE_SPLIT");
    return !(e && e[0] == '0');
  }();
  const int wsf = split ? dgi_sample_ws_floats(B, (int)logits.size(1)) : 0;
  at::Tensor ws;
  if (wsf > 0) ws = at::empty({wsf}, logits.options().dtype(at::kFloat));
  check_rc(dgi_sample(logits.data_ptr(), logits.scalar_type() == at::kBFloat16, B,
                      (int)logits.size(1), (int)logits.stride(0), tp, sp, step, thp,
                      reinterpret_cast<long long*>(out.data_ptr<int64_t>()), wsf > 0 ? ws.data_ptr() : nullptr,
                      cur_stream()),
           "sample");
}

void topkp_threshold(at::Tensor thresh, const at::Tensor& logits, const at::Tensor& temperature,
                     const at::Tensor& top_k, const at::Tensor& top_p) {
  check_dev(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1);
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat);
  const int B = (int)logits.size(0);
  TORCH_CHECK(thresh.scalar_type() == at::kFloat && thresh.is_contiguous() && thresh.numel() >= B);
  TORCH_CHECK(temperature.scalar_type() == at::kFloat && temperature.is_contiguous() && temperature.numel() >= B);
  TORCH_CHECK(top_k.scalar_type() == at::kLong && top_k.is_contiguous() && top_k.numel() >= B);
  TORCH_CHECK(top_p.scalar_type() == at::kFloat && top_p.is_contiguous() && top_p.numel() >= B);
  TORCH_CHECK(thresh.device() == logits.device() && temperature.device() == logits.device() &&
              top_k.device() == logits.device() && top_p.device() == logits.device());
  check_rc(dgi_topkp_threshold(logits.data_ptr(), logits.scalar_type() == at::kBFloat16, B, (int)logits.size(1),
                               (int)logits.stride(0), temperature.data_ptr<float>(),
                               reinterpret_cast<const long long*>(top_k.data_ptr<int64_t>()),
                               top_p.data_ptr<float>(), thresh.data_ptr<float>(), cur_stream()),
           "topkp_threshold");
}

void topk(at::Tensor out_v, at::Tensor out_i, const at::Tensor& logits, int64_t k) {
  check_dev(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1);
  const int B = (int)logits.size(0);
  TORCH_CHECK(out_v.scalar_type() == at::kFloat && out_i.scalar_type() == at::kLong);
  TORCH_CHECK(out_v.numel() >= B * k && out_i.numel() >= B * k);
  check_rc(dgi_topk(logits.data_ptr(), logits.scalar_type() == at::kBFloat16, B, (int)logits.size(1),
                    (int)logits.stride(0), (int)k, out_v.data_ptr<float>(),
                    reinterpret_cast<long long*>(out_i.data_ptr<int64_t>()), cur_stream()),
           "topk");
}

// top-k of log_softmax(logits) (bf16 logits, fp32 log-probs of the k winners)
void topk_logprobs(at::Tensor out_v, at::Tensor out_i, const at::Tensor& logits, int64_t k) {
  check_dev(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1 && logits.scalar_type() == at::kBFloat16);
  const int B = (int)logits.size(0), V = (int)logits.size(1);
  TORCH_CHECK(out_v.scalar_type() == at::kFloat && out_i.scalar_type() == at::kLong);
  TORCH_CHECK(out_v.numel() >= B * k && out_i.numel() >= B * k && out_v.is_contiguous() && out_i.is_contiguous());
  at::Tensor ws = at::empty({std::max(1, dgi_topk_logprobs_ws_floats(B, V))}, logits.options().dtype(at::kFloat));
  check_rc(dgi_topk_logprobs(logits.data_ptr(), B, V, (int)logits.stride(0), (int)k, ws.data_ptr<float>(),
                             out_v.data_ptr<float>(), reinterpret_cast<long long*>(out_i.data_ptr<int64_t>()),
                             cur_stream()),
           "topk_logprobs");
}

// cache: [L, 2, NB, nkv, bs, hd]; buf: [L, 2, n, nkv, bs, hd], or [n, L, 2, nkv, bs, hd] when block_major
void kv_gather(at::Tensor buf, const at::Tensor& cache, const at::Tensor& ids, bool block_major) {
  check_dev(cache, "cache"); check_i32(ids, "ids");
  TORCH_CHECK(cache.is_contiguous() && buf.is_contiguous() && cache.dim() == 6);
  const int n = (int)ids.numel();
  const int LK = (int)(cache.size(0) * cache.size(1));
  const int NB = (int)cache.size(2);
  const int page = (int)(cache.size(3) * cache.size(4) * cache.size(5));
  TORCH_CHECK(buf.numel() >= (int64_t)LK * n * page && buf.scalar_type() == cache.scalar_type());
  check_rc(dgi_kv_gather(cache.data_ptr(), ids.data_ptr<int>(), n, LK, NB, page, buf.data_ptr(),
                         block_major ? 1 : 0, cur_stream()), "kv_gather");
}

void kv_scatter(at::Tensor cache, const at::Tensor& ids, const at::Tensor& buf, bool block_major) {
  check_dev(cache, "cache"); check_i32(ids, "ids");
  TORCH_CHECK(cache.is_contiguous() && buf.is_contiguous() && cache.dim() == 6);
  const int n = (int)ids.numel();
  const int LK = (int)(cache.size(0) * cache.size(1));
  const int NB = (int)cache.size(2);
  const int page = (int)(cache.size(3) * cache.size(4) * cache.size(5));
  TORCH_CHECK(buf.numel() >= (int64_t)LK * n * page && buf.scalar_type() == cache.scalar_type());
  check_rc(dgi_kv_scatter(cache.data_ptr(), ids.data_ptr<int>(), n, LK, NB, page, buf.data_ptr(),
                          block_major ? 1 : 0, cur_stream()), "kv_scatter");
}

void kv_copy(at::Tensor cache, const at::Tensor& src, const at::Tensor& dst) {
  check_dev(cache, "cache"); check_i32(src, "src"); check_i32(dst, "dst");
  TORCH_CHECK(cache.is_contiguous() && cache.dim() == 6 && src.numel() == dst.numel());
  const int LK = (int)(cache.size(0) * cache.size(1));
  const int NB = (int)cache.size(2);
  const int page = (int)(cache.size(3) * cache.size(4) * cache.size(5));
  check_rc(dgi_kv_copy(cache.data_ptr(), src.data_ptr<int>(), dst.data_ptr<int>(), (int)src.numel(),
                       LK, NB, page, cur_stream()), "kv_copy");
}

// token-slot copy inside the paged cache (all layers, K and V); src / dst int32 slots
void kv_slot_copy(at::Tensor cache, const at::Tensor& src, const at::Tensor& dst) {
  check_dev(cache, "cache"); check_i32(src, "src"); check_i32(dst, "dst");
  TORCH_CHECK(cache.is_contiguous() && cache.dim() == 6 && src.numel() == dst.numel());
  TORCH_CHECK(cache.scalar_type() == at::kBFloat16 || cache.scalar_type() == at::kHalf);
  const int n = (int)src.numel();
  if (n == 0) return;
  const int LK = (int)(cache.size(0) * cache.size(1));
  const int NB = (int)cache.size(2), nkv = (int)cache.size(3), bs = (int)cache.size(4), hd = (int)cache.size(5);
  at::Tensor buf = at::empty({(int64_t)n * LK * nkv * hd}, cache.options());
  check_rc(dgi_kv_slot_copy(cache.data_ptr(), src.data_ptr<int>(), dst.data_ptr<int>(), n, LK, NB, nkv, bs, hd,
                            buf.data_ptr(), cur_stream()), "kv_slot_copy");
}

// read `w`'s rows (all, the first `nrows`, or the ids in `rows`) so they sit in the MALL
void mall_prefetch(const at::Tensor& w, const c10::optional<at::Tensor>& rows, at::Tensor sink, int64_t nrows,
                   int64_t blocks) {
  check_dev(w, "w"); check_dev(sink, "sink");
  TORCH_CHECK(w.dim() == 2 && w.stride(1) == 1, "mall_prefetch: w must be a row-major matrix");
  TORCH_CHECK(sink.numel() * sink.element_size() >= 1024, "mall_prefetch: sink needs 1 KB");
  const int* rp = nullptr;
  int n = (int)w.size(0);
  if (rows.has_value()) {
    check_i32(*rows, "rows");
    rp = rows->data_ptr<int>();
    n = (int)rows->numel();
  }
  if (nrows >= 0 && nrows < n) n = (int)nrows;
  const int64_t rb = w.stride(0) * w.element_size();
  TORCH_CHECK(rb < (1LL << 31), "mall_prefetch: row too long");
  check_rc(dgi_mall_prefetch(w.data_ptr(), rp, n, (int)rb, (int)blocks, sink.data_ptr(), cur_stream()),
           "mall_prefetch");
}

void tree_mask(at::Tensor anc, at::Tensor depth, const at::Tensor& parent) {
  check_i32(parent, "parent"); check_i32(depth, "depth");
  TORCH_CHECK(anc.scalar_type() == at::kLong && anc.is_contiguous());
  const int B = (int)parent.size(0), N = (int)parent.size(1);
  TORCH_CHECK(N <= 64 && anc.numel() >= (int64_t)B * 64 && depth.numel() >= (int64_t)B * N);
  check_rc(dgi_tree_mask(parent.data_ptr<int>(), B, N,
                         reinterpret_cast<unsigned long long*>(anc.data_ptr<int64_t>()),
                         depth.data_ptr<int>(), cur_stream()), "tree_mask");
}

void tree_verify(at::Tensor accept_len, at::Tensor path, at::Tensor out_tokens,
                 const at::Tensor& parent, const at::Tensor& draft, const at::Tensor& target,
                 const at::Tensor& anc, const at::Tensor& depth) {
  check_i32(parent, "parent"); check_i32(depth, "depth"); check_i32(accept_len, "accept_len");
  check_i32(path, "path");
  TORCH_CHECK(draft.scalar_type() == at::kLong && target.scalar_type() == at::kLong);
  TORCH_CHECK(out_tokens.scalar_type() == at::kLong && anc.scalar_type() == at::kLong);
  const int B = (int)parent.size(0), N = (int)parent.size(1);
  const int max_path = (int)path.size(1);
  TORCH_CHECK(out_tokens.size(1) == max_path + 1 && draft.numel() >= (int64_t)B * N && target.numel() >= (int64_t)B * N);
  check_rc(dgi_tree_verify(parent.data_ptr<int>(),
                           reinterpret_cast<const long long*>(draft.data_ptr<int64_t>()),
                           reinterpret_cast<const long long*>(target.data_ptr<int64_t>()), B, N,
                           reinterpret_cast<const unsigned long long*>(anc.data_ptr<int64_t>()),
                           depth.data_ptr<int>(), accept_len.data_ptr<int>(), path.data_ptr<int>(),
                           reinterpret_cast<long long*>(out_tokens.data_ptr<int64_t>()), max_path,
                           cur_stream()), "tree_verify");
}

// CUs the MFMA GEMM's persistent launches size their grid for (0 = the device's; a CU-masked
// two-batch-overlap step sets the GEMM stream's share)
void set_gemm_cus(int64_t cus) { dgi_set_gemm_cus(static_cast<int>(cus)); }
int64_t gemm_split_timeouts(bool reset) { return dgi_gemm_split_timeouts(reset ? 1 : 0); }

}  // namespace

TORCH_LIBRARY(dgi, m) {
  m.def("set_gemm_cus(int cus) -> ()", &set_gemm_cus);
  m.def("gemm_split_timeouts(bool reset) -> int", &gemm_split_timeouts);
  m.def("rmsnorm(Tensor(a!) out, Tensor x, Tensor w, float eps) -> ()");
  m.def("fused_add_rmsnorm(Tensor(a!) x, Tensor(b!) residual, Tensor w, float eps) -> ()");
  m.def("rope_cache(Tensor(a!) qkv, Tensor positions, Tensor cos_sin, int nh, int nkv, int hd, "
        "Tensor slot_mapping, Tensor(b!) k_cache, Tensor(c!) v_cache, int mode=0) -> ()");
  m.def("paged_decode(Tensor(a!) out, Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, "
        "Tensor context_lens, Tensor(b!) part_o, Tensor(c!) part_lse, int nh, int nkv, int max_splits, "
        "int part_size, float scale, Tensor(d!)? counters=None) -> ()");
  m.def("paged_prefill(Tensor(a!) out, Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, "
        "Tensor cu_seqlens_q, Tensor context_lens, Tensor tiles, int nh, int nkv, float scale, "
        "Tensor? tree_mask, int tree_n, int tile_rows=128) -> ()");
  m.def("silu_mul(Tensor(a!) out, Tensor gu) -> ()");
  m.def("skinny_gemm(Tensor(a!) out, Tensor x, Tensor w, Tensor? bias, int cfg=0) -> ()");
  m.def("mfma_gemm(Tensor(a!) out, Tensor x, Tensor w, int epi=0) -> ()");
  m.def("mfma_gemm_norm(Tensor(a!) out, Tensor x, Tensor w, int kind, Tensor(b!) ss, float inv_k, float eps, "
        "int phases=0) -> ()");
  m.def("mfma_gemm_norm_rope(Tensor(a!) out, Tensor x, Tensor w, Tensor ss, float inv_k, float eps, "
        "Tensor positions, Tensor cos_sin, Tensor slot_mapping, Tensor(b!) k_cache, Tensor(c!) v_cache, int nh, "
        "int nkv, int phases=0) -> ()");
  m.def("fused_skinny(Tensor(a!) y, Tensor x, Tensor? res, Tensor(b!)? res_out, Tensor? gamma, float eps, "
        "Tensor w, Tensor? bias, int pro, int epi, Tensor? positions, Tensor? cos_sin, Tensor? slots, "
        "Tensor(c!)? k_cache, Tensor(d!)? v_cache, int nh=0, int nkv=0, int cfg=0) -> ()");
  m.def("sample(Tensor(a!) out, Tensor logits, Tensor? temperature, Tensor? seeds, int step, "
        "Tensor? thresh=None) -> ()");
  m.def("topkp_threshold(Tensor(a!) thresh, Tensor logits, Tensor temperature, Tensor top_k, "
        "Tensor top_p) -> ()");
  m.def("topk(Tensor(a!) out_v, Tensor(b!) out_i, Tensor logits, int k) -> ()");
  m.def("topk_logprobs(Tensor(a!) out_v, Tensor(b!) out_i, Tensor logits, int k) -> ()");
  m.def("kv_gather(Tensor(a!) buf, Tensor cache, Tensor ids, bool block_major) -> ()");
  m.def("kv_scatter(Tensor(a!) cache, Tensor ids, Tensor buf, bool block_major) -> ()");
  m.def("kv_copy(Tensor(a!) cache, Tensor src, Tensor dst) -> ()");
  m.def("kv_slot_copy(Tensor(a!) cache, Tensor src, Tensor dst) -> ()");
  m.def("mall_prefetch(Tensor w, Tensor? rows, Tensor(a!) sink, int nrows=-1, int blocks=256) -> ()");
  m.def("tree_mask(Tensor(a!) anc, Tensor(b!) depth, Tensor parent) -> ()");
  m.def("tree_verify(Tensor(a!) accept_len, Tensor(b!) path, Tensor(c!) out_tokens, Tensor parent, "
        "Tensor draft, Tensor target, Tensor anc, Tensor depth) -> ()");
}

TORCH_LIBRARY_IMPL(dgi, CUDA, m) {
  m.impl("rmsnorm", &rmsnorm);
  m.impl("fused_add_rmsnorm", &fused_add_rmsnorm);
  m.impl("rope_cache", &rope_cache);
  m.impl("paged_decode", &paged_decode);
  m.impl("paged_prefill", &paged_prefill);
  m.impl("silu_mul", &silu_mul);
  m.impl("skinny_gemm", &skinny_gemm);
  m.impl("mfma_gemm", &mfma_gemm);
  m.impl("mfma_gemm_norm", &mfma_gemm_norm);
  m.impl("mfma_gemm_norm_rope", &mfma_gemm_norm_rope);
  m.impl("fused_skinny", &fused_skinny);
  m.impl("sample", &sample);
  m.impl("topk", &topk);
  m.impl("topk_logprobs", &topk_logprobs);
  m.impl("topkp_threshold", &topkp_threshold);
  m.impl("kv_gather", &kv_gather);
  m.impl("kv_scatter", &kv_scatter);
  m.impl("kv_copy", &kv_copy);
  m.impl("kv_slot_copy", &kv_slot_copy);
  m.impl("mall_prefetch", &mall_prefetch);
  m.impl("tree_mask", &tree_mask);
  m.impl("tree_verify", &tree_verify);
}
