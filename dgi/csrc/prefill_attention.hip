// dgi/csrc/prefill_attention.hip — varlen causal flash attention over the paged
// KV pool (prefill, chunked prefill, prefix-cache hits, EAGLE tree
// verification).
//
// The reference runs prefill inside HF `generate` / `ModelShard.forward`
// (worker/engines/llm.py:61-69, worker/distributed/model_shard.py:173-228)
// and has no prefix-aware attention.  Here new queries attend over
// [cached prefix | freshly written KV] straight from the block pool.
//
// CDNA4 structure:
//   grid = (q_tiles, n_heads), 256 threads = 4 waves x 32 query rows.
//   K/V tiles of 64 keys are staged through LDS by the whole workgroup:
//     * K image: 256-byte rows, 16-byte chunk XOR-swizzled by (row & 15) so the
//       32-row ds_read_b128 fragment reads are conflict free (guide T2);
//     * V image: chunk XOR (row & 3) << 2 so ds_read_b64_tr_b16 transposed
//       reads (guide T10) are conflict free.
//   Scores are computed swapped, S^T = K Q^T with mfma_f32_32x32x16_bf16, so a
//   lane owns one query: the softmax row reduction is lane-local plus one
//   xor-32 shuffle, and the probabilities are consumed from the accumulator
//   registers as the B operand of O^T += V^T P^T (guide §3 "accumulator tile
//   as the next MFMA's operand").
//   Optional tree mask: for EAGLE verification the last `tree_n` queries of a
//   sequence see the cached prefix plus their ancestors, given as one 64-bit
//   ancestor mask per query (built by tree.hip).
#include "common.h"

using namespace dgi;

namespace {

// Element offset of 16-byte chunk `ch` of LDS row `row`.
// HD=128 (256-B rows): K chunk ^ (row & 15) — 16 consecutive rows at one chunk
// hit 16 distinct slots (ds_read_b128); V chunk ^ ((row & 3) << 2) for the
// transposed reads.  HD=64 (128-B rows, two rows per 64-bank line): row & 1
// already picks the bank half, so K XORs (row >> 1) & 7 and V shifts rows
// 2-3 of each 4-row block by 4 chunks.
template <int HD>
__device__ __forceinline__ int k_off(int row, int ch) {
  if constexpr (HD == 128) return row * 128 + (((ch) ^ (row & 15)) << 3);
  else return row * 64 + (((ch) ^ ((row >> 1) & 7)) << 3);
}
template <int HD>
__device__ __forceinline__ int v_off(int row, int ch) {
  if constexpr (HD == 128) return row * 128 + (((ch) ^ ((row & 3) << 2)) << 3);
  else return row * 64 + (((ch) ^ (((row >> 1) & 1) << 2)) << 3);
}

constexpr int KT = 64;  // keys per tile

// NW waves x 32 query rows per workgroup (one K/V tile staging shared by all of them):
// NW = 4 -> 128-row tiles, 2 workgroups per CU; NW = 8 -> 256-row tiles, 1 per CU
// (same 2 waves per SIMD, half the K/V staging per query row).
// DB = 1: two LDS stages.  Tile i+1 is written into the idle stage right after the one
// barrier of iteration i (its registers were loaded during iteration i-1), tile i+2's
// global loads are issued, then tile i is consumed — one barrier per 64 keys instead of
// two, and a wave's LDS write no longer waits for every other wave before its MFMAs
// (round 5: 24 % MFMA busy with DB = 0, profiles/r5_pmc/).
template <int HD, int NW, int DB>
__global__ __launch_bounds__(NW * 64, NW == 4 ? 2 : 1) void prefill_attn_kernel(
    const uint16_t* __restrict__ q, int q_stride, const uint16_t* __restrict__ k_cache,
    const uint16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ cu_seqlens_q, const int* __restrict__ context_lens,
    const int* __restrict__ tiles, uint16_t* __restrict__ out, int out_stride, int nh, int nkv,
    int bs_log2, float scale_log2, const unsigned long long* __restrict__ tree_mask, int tree_n) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[(DB ? 2 : 1) * 2 * KT * HD];

  const int b = tiles[2 * blockIdx.x];
  const int t0 = tiles[2 * blockIdx.x + 1];  // first query row (within seq) of this tile
  const int head = blockIdx.y;
  const int kvh = head / (nh / nkv);
  const int q0 = cu_seqlens_q[b];
  const int qlen = cu_seqlens_q[b + 1] - q0;
  const int ctx = context_lens[b];
  const int pos_base = ctx - qlen;  // absolute position of query row 0
  const int bs = 1 << bs_log2;
  const int* bt = block_tables + (size_t)b * bt_stride;

  const int tid = threadIdx.x;
  const int w = tid >> 6;
  const int lane = tid & 63;
  const int lr = lane & 31;
  const int hh = lane >> 5;

  const int my_row = t0 + 32 * w + lr;  // query row within the sequence
  const bool row_valid = my_row < qlen;
  const int my_pos = pos_base + my_row;
  const int tree_first = qlen - tree_n;  // rows >= tree_first use the tree mask
  unsigned long long tmask = 0;
  const bool is_tree = tree_mask != nullptr && row_valid && my_row >= tree_first;
  if (is_tree) tmask = tree_mask[(size_t)b * 64 + (my_row - tree_first)];
  const int tree_key0 = pos_base + tree_first;  // key index of tree node 0

  constexpr int NS = HD / 16;   // k-steps of S^T = K Q^T
  constexpr int ND = HD / 32;   // 32-dim blocks of O^T
  constexpr int CH = HD / 8;    // 16-byte chunks per K/V row
  constexpr int NT = NW * 64;        // threads
  constexpr int NP = KT * CH / NT;   // staging passes per tile (one chunk per thread per pass)
  // Q fragments (B operand): lane holds Q[row lr][16 s + 8 hh + j]
  u32x4 qf[NS];
  {
    const uint16_t* qp = q + (size_t)(q0 + (row_valid ? my_row : 0)) * q_stride + head * HD;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      qf[s] = row_valid ? *reinterpret_cast<const u32x4*>(qp + 16 * s + 8 * hh) : u32x4{0, 0, 0, 0};
    // Q lands before any K/V load is issued.  Without this wait the compiler's waitcnt pass
    // merges "Q pending" from the preheader into the loop header and, to reach the older Q
    // loads, emits vmcnt(0) before the first QK^T MFMA of EVERY tile — which also waits for
    // the K/V loads of tile i+2 issued a few instructions earlier: one full HBM round trip
    // per tile and no load/compute overlap at all (round 5 disassembly).
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0), expcnt / lgkmcnt untouched (gfx9 encoding)
  }

  const int last_row = min(t0 + 32 * NW, qlen) - 1;
  const int kv_end = min(ctx, pos_base + last_row + 1);

  float m_run = -1e30f, l_run = 0.f;
  f32x16 o[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;

  const size_t head_stride = (size_t)bs * HD;
  // K/V tile loads are software-pipelined one tile ahead through registers:
  // the global loads of tile i+1 are in flight while tile i is consumed from
  // LDS (1 workgroup per CU at this register budget, so latency must be hidden
  // inside the wave, not by occupancy).
  u32x4 kr[NP], vr[NP];
  auto load_tile = [&](int kb0) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int row = p * (NT / CH) + tid / CH;
      const int ch = tid % CH;
      const int key = min(kb0 + row, kv_end - 1);
      const int blk = bt[key >> bs_log2];
      const size_t base = ((size_t)blk * nkv + kvh) * head_stride + (size_t)(key & (bs - 1)) * HD + ch * 8;
      kr[p] = *reinterpret_cast<const u32x4*>(k_cache + base);
      vr[p] = *reinterpret_cast<const u32x4*>(v_cache + base);
    }
  };
  auto store_tile = [&](uint16_t* kst, uint16_t* vst) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int row = p * (NT / CH) + tid / CH;
      const int ch = tid % CH;
      *reinterpret_cast<u32x4*>(kst + k_off<HD>(row, ch)) = kr[p];
      *reinterpret_cast<u32x4*>(vst + v_off<HD>(row, ch)) = vr[p];
    }
  };
  // Full tiles of 16-token pages (the engine's page size): the rows one wave stages in one
  // pass lie in ONE page (a wave covers 64 / CH consecutive rows, 4 or 8, and passes are
  // whole pages apart), so that page's block id is a wave-uniform scalar load and every
  // lane's offset inside the page is a constant — no per-lane block-table gather and no
  // 64-bit address arithmetic per load (the decode kernel's page16 path, round 4).
  constexpr int RP = NT / CH;                  // tile rows per staging pass (16, 32 or 64)
  static_assert(RP % 16 == 0 && 16 % (64 / CH) == 0, "passes are whole pages");
  const int wsub = __builtin_amdgcn_readfirstlane(w) * (64 / CH);   // first row of this wave in a pass
  const int lane_off = ((wsub & 15) + lane / CH) * HD + (lane % CH) * 8;
  const int wpage = wsub >> 4;
  const bool page16 = bs_log2 == 4;
  // Block ids of a fast tile: wave-uniform scalar loads (s_load), issued at the top of the
  // iteration that issues the tile's K/V loads so their latency overlaps the LDS stores.  (A
  // vector-load prefetch one iteration ahead was tried: vmcnt is in-order, so waiting for it
  // waited for the K/V loads issued after it — the stall the prefetch was meant to remove.)
  int nbt[NP];
  auto fast = [&](int kb0) { return page16 && kb0 + KT <= kv_end; };
  auto fetch_bt = [&](int kb0) {
#pragma unroll
    for (int p = 0; p < NP; ++p) nbt[p] = bt[(kb0 >> 4) + p * (RP / 16) + wpage];
  };
  auto load_tile_fast = [&]() {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const size_t base = ((size_t)nbt[p] * nkv + kvh) * head_stride;
      kr[p] = *reinterpret_cast<const u32x4*>(k_cache + base + lane_off);
      vr[p] = *reinterpret_cast<const u32x4*>(v_cache + base + lane_off);
    }
  };
  auto load_any = [&](int kb0) {
    if (fast(kb0)) {
      fetch_bt(kb0);
      load_tile_fast();
    } else {
      load_tile(kb0);
    }
  };
  if (kv_end > 0) load_any(0);
  if (DB && kv_end > 0) {
    store_tile(lds, lds + KT * HD);             // stage 0 <- tile 0
    if (KT < kv_end) load_any(KT);              // registers <- tile 1
  }
  // last key this wave can see (causal); tiles beyond it are skipped
  const int wave_last_pos = pos_base + min(t0 + 32 * w + 31, qlen - 1);
  // keys <= wave_first_pos are visible to every row of the wave
  const int wave_first_pos = pos_base + t0 + 32 * w;
  const bool wave_tree = tree_mask != nullptr && (t0 + 32 * w + 31 >= tree_first);
  const bool wave_rows = t0 + 32 * w < qlen;
  int it = 0;
  for (int kb0 = 0; kb0 < kv_end; kb0 += KT, ++it) {
    uint16_t* ks;
    uint16_t* vs;
    if (DB) {
      // stage it&1 holds tile it (written last iteration, or before the loop); every wave has
      // finished reading stage (it+1)&1 (tile it-1) once it is past this barrier
      __syncthreads();
      ks = lds + (it & 1) * 2 * KT * HD;
      vs = ks + KT * HD;
      if (kb0 + KT < kv_end) {
        const bool nxt = kb0 + 2 * KT < kv_end;
        const bool nfast = nxt && fast(kb0 + 2 * KT);
        if (nfast) fetch_bt(kb0 + 2 * KT);
        uint16_t* kn = lds + ((it + 1) & 1) * 2 * KT * HD;
        store_tile(kn, kn + KT * HD);           // tile it+1, loaded during the previous iteration
        if (nfast) load_tile_fast();
        else if (nxt) load_tile(kb0 + 2 * KT);
      }
    } else {
      ks = lds;
      vs = lds + KT * HD;
      __syncthreads();  // previous tile fully consumed
      store_tile(ks, vs);
      __syncthreads();
      if (kb0 + KT < kv_end) load_any(kb0 + KT);
    }
    // whole tile above this wave's diagonal, or no valid query row in this wave
    // (it still stages K/V for the others)
    if (kb0 > wave_last_pos || !wave_rows) continue;

    // ---- S^T = K Q^T for two 32-key blocks
    f32x16 sc[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[kb][r] = 0.f;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const u32x4 a = *reinterpret_cast<const u32x4*>(ks + k_off<HD>(32 * kb + lr, 2 * s + hh));
        sc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(a), as_bf16x8(qf[s]), sc[kb], 0, 0, 0);
      }
    }
    // ---- online softmax; lane owns query lr, keys kb0 + 32kb + (r&3) + 8(r>>2) + 4hh.
    // Interior tiles (every key visible to every row of this wave, no tree rows) skip the
    // per-element mask; both kinds then share one exponent path.
    const bool interior = (kb0 + KT <= kv_end) && (kb0 + KT - 1 <= wave_first_pos) && !wave_tree;
    if (!interior) {
      // masked keys -> -inf in raw score units, in place (one select per element, no branches:
      // the tree bit is read with a clamped shift and applied by mask).  -inf, not a large
      // finite value: a lane whose keys are all masked must get max -inf (no rescale) and
      // P = 2^(-inf) = 0, whatever the scale.  Causal-only tiles (the diagonal) skip the
      // 64-bit tree-mask shifts.
      const int lim = row_valid ? min(my_pos, kv_end - 1) : -1;    // last visible key
      const int key0 = kb0 + 4 * hh;
      if (wave_tree) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = key0 + 32 * kb + (r & 3) + 8 * (r >> 2);
            const int dt = key - tree_key0;
            const bool tbit = (tmask >> (dt & 63)) & 1ull;
            const bool ok = (key <= lim) & (!is_tree | (dt < 0) | tbit);
            sc[kb][r] = ok ? sc[kb][r] : -__builtin_inff();
          }
      } else {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            sc[kb][r] = (key0 + 32 * kb + (r & 3) + 8 * (r >> 2) <= lim) ? sc[kb][r] : -__builtin_inff();
      }
    }
    float mx = -1e30f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[kb][r]);
    mx = row_valid ? mx * scale_log2 : -1e30f;
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    // deferred max: rescale O / l only when the running max grows by > 2^8, so
    // most tiles skip the 64 O multiplies (P stays <= 256, safe in f32 / bf16)
    if (__any(mx > m_run + 8.f)) {
      const float m_new = fmaxf(m_run, mx);
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      l_run *= alpha;
#pragma unroll
      for (int d = 0; d < ND; ++d) o[d] *= alpha;
      m_run = m_new;
    }
    // P = 2^(s * scale_log2 - m): packed fp32 (v_pk_fma_f32 / v_pk_add_f32), two scores per
    // VALU issue for the scale and the row sums; raw v_exp_f32 (arguments <= 8; masked scores
    // underflow to 0); four partial row sums instead of one 32-long dependent add chain
    float ps[4];
    {
      const f32x2v s2 = {scale_log2, scale_log2};
      const f32x2v n2 = {-m_run, -m_run};
      f32x2v acc2[2] = {{0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          f32x2v x = {sc[kb][r], sc[kb][r + 1]};
          x = x * s2 + n2;
          x[0] = __builtin_amdgcn_exp2f(x[0]);
          x[1] = __builtin_amdgcn_exp2f(x[1]);
          sc[kb][r] = x[0];
          sc[kb][r + 1] = x[1];
          acc2[(r >> 1) & 1] += x;
        }
      ps[0] = acc2[0][0];
      ps[1] = acc2[0][1];
      ps[2] = acc2[1][0];
      ps[3] = acc2[1][1];
    }
    float psum = (ps[0] + ps[1]) + (ps[2] + ps[3]);
    psum += __shfl_xor(psum, 32, 64);
    l_run += psum;

    // ---- O^T += V^T P^T
    const int g16 = lane >> 4;
    const int idx = lane & 15;
    const int tq = idx >> 2, tp = idx & 3;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        u32x4 pf;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) pf[jj] = pack_bf16x2(sc[kb][8 * s2 + 2 * jj], sc[kb][8 * s2 + 2 * jj + 1]);
#pragma unroll
        for (int d = 0; d < ND; ++d) {
          const int col = 32 * d + 16 * (g16 & 1) + 4 * tp;
          const int r0 = 32 * kb + 16 * s2 + 4 * hh + tq;
          short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_short4*)(vs + v_off<HD>(r0, col >> 3) + (col & 7)));
          short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_short4*)(vs + v_off<HD>(r0 + 8, col >> 3) + (col & 7)));
          u32x4 vf;
          vf[0] = (uint32_t)(uint16_t)lo[0] | ((uint32_t)(uint16_t)lo[1] << 16);
          vf[1] = (uint32_t)(uint16_t)lo[2] | ((uint32_t)(uint16_t)lo[3] << 16);
          vf[2] = (uint32_t)(uint16_t)hi[0] | ((uint32_t)(uint16_t)hi[1] << 16);
          vf[3] = (uint32_t)(uint16_t)hi[2] | ((uint32_t)(uint16_t)hi[3] << 16);
          o[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(vf), as_bf16x8(pf), o[d], 0, 0, 0);
        }
      }
  }

  if (!row_valid) return;
  const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
  uint16_t* op = out + (size_t)(q0 + my_row) * out_stride + head * HD;
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int dim = 32 * d + 8 * rr + 4 * hh;
      uint2 v;
      v.x = pack_bf16x2(o[d][4 * rr] * inv, o[d][4 * rr + 1] * inv);
      v.y = pack_bf16x2(o[d][4 * rr + 2] * inv, o[d][4 * rr + 3] * inv);
      *reinterpret_cast<uint2*>(op + dim) = v;
    }
}


}  // namespace

// tiles: int32 [n_tiles, 2] = (sequence index, first query row of the tile_rows-row tile)
extern "C" int dgi_paged_prefill(const void* q, int q_stride, const void* k_cache,
                                 const void* v_cache, const int* block_tables, int bt_stride,
                                 const int* cu_seqlens_q, const int* context_lens, const int* tiles,
                                 int n_tiles, void* out, int out_stride, int nh, int nkv, int hd,
                                 int block_size, float scale, const unsigned long long* tree_mask,
                                 int tree_n, int tile_rows, hipStream_t s) {
  if (n_tiles == 0) return 0;
  if (hd != 128 && hd != 64) return -5;
  if (nh % nkv) return -2;
  if (tree_n > 64) return -6;
  int bs_log2 = 0;
  while ((1 << bs_log2) < block_size) ++bs_log2;
  if ((1 << bs_log2) != block_size) return -4;
  const float scale_log2 = scale * 1.4426950408889634f;
  const int db = (tile_rows >> 16) & 1;          // bit 16: two LDS stages (prefill_attn_kernel DB)
  tile_rows &= 0xffff;
  if (tile_rows != 128 && tile_rows != 256) return -7;
#define DGI_PREFILL(HDV, NWV, DBV)                                                                     \
  prefill_attn_kernel<HDV, NWV, DBV><<<dim3(n_tiles, nh), NWV * 64, 0, s>>>(                           \
      (const uint16_t*)q, q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables,     \
      bt_stride, cu_seqlens_q, context_lens, tiles, (uint16_t*)out, out_stride, nh, nkv, bs_log2,         \
      scale_log2, tree_mask, tree_n)
  if (hd == 128) {
    if (tile_rows == 256) { if (db) DGI_PREFILL(128, 8, 1); else DGI_PREFILL(128, 8, 0); }
    else { if (db) DGI_PREFILL(128, 4, 1); else DGI_PREFILL(128, 4, 0); }
  } else {
    if (tile_rows == 256) { if (db) DGI_PREFILL(64, 8, 1); else DGI_PREFILL(64, 8, 0); }
    else { if (db) DGI_PREFILL(64, 4, 1); else DGI_PREFILL(64, 4, 0); }
  }
#undef DGI_PREFILL
  DGI_CHECK_LAUNCH();
  return 0;
}
