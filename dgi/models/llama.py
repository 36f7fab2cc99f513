"""Native Llama-family decoder for the MI355X runtime (Llama-3 8B / 70B, Qwen2 / Qwen2.5, GLM-4).

Replaces the HF modules the reference executes (worker/engines/llm.py:22-69,
worker/distributed/model_shard.py:28-246).  Per layer the step runs

    fused_add_rmsnorm (HIP) -> QKV GEMM (hipBLASLt) -> RoPE + paged KV write (HIP)
    -> paged decode / prefill attention (HIP, MFMA) -> O GEMM
    -> fused_add_rmsnorm (HIP) -> gate|up GEMM -> SiLU*mul (HIP) -> down GEMM

with fused QKV and gate|up weights so each layer issues 4 GEMMs.  Qwen2's biased
q/k/v projections ride in the QKV GEMM's bias epilogue (hipBLASLt), so the
family adds no kernel; GLM-4 adds biased QKV and half-dim interleaved RoPE
(``rope_cache`` mode 1 over the first ``rotary_dim`` dims).  A model
object may hold any contiguous layer range (pipeline stage): stage 0 owns the
embedding, the last stage the final norm and LM head, exactly like the
reference's ``ModelShard`` (model_shard.py:28-59).  Between stages a single
hidden tensor travels: the residual stream (h + residual) — the next stage
re-normalises it, which is bit-identical to the fused add it replaces.
"""
from __future__ import annotations

import contextlib
import math
import os
from typing import Optional

import torch
import torch.nn.functional as F

from dgi import ops
from dgi.models.config import ModelConfig
from dgi.runtime.batch import AttnMeta



# DGI_TRIM_LAST_LAYER=0 runs the last layer's o-proj and MLP on every row (A/B switch)
TRIM_LAST_LAYER = os.environ.get("DGI_TRIM_LAST_LAYER", "1") != "0"
# DGI_QKV_PAD=1: the QKV GEMM reuses the MLP's padded rows; DGI_OPROJ_PAD=1: the o-proj
# runs on a zero-padded attention output.  Both off by default: with them the start-up
# table times qkv / o-proj at every row count too, and the 70B bench measured no gain
# (1755 / 1743 vs 1761 / 1750 tok/s, profiles/r2_bench70b_qkvpad_ab.md)
QKV_PAD = os.environ.get("DGI_QKV_PAD", "0") == "1"
OPROJ_PAD = os.environ.get("DGI_OPROJ_PAD", "0") == "1"
# mixed steps: decode-row attention on a side stream beside the prefill-row attention
ATTN_OVERLAP = os.environ.get("DGI_ATTN_OVERLAP", "1") == "1"
# Two-batch overlap (TBO) of large pure-decode steps (``LlamaModel._forward_layers_tbo``): the
# rows are cut in two tile-aligned halves whose decode attention runs on a few CUs of every
# XCD (``DGI_TBO_SIDE`` per XCD) while the other half's GEMM chain runs on the rest.  Two
# plain streams do not overlap (a full-chip GEMM holds every CU: graph-forked GEMM + HBM stream
# 0.713 vs 0.751 ms serial); CU-masked streams do for a plain HBM stream (1.56 vs 1.70 ms
# eagerly), and a captured graph drops the masks, so TBO steps run eagerly.  OFF by default:
# on the 27-layer 70B decode stage at 768 rows it MEASURED 67.0 ms against 41.9 eager / 39.8
# graph-replayed (profiles/r5_pd/README.md) — split-KV decode attention is latency-bound per
# CU (32 CUs ran it 3.1x slower than 256, not 8x) and the half-size GEMMs beside it ran 1.85x
# slower than their share; DGI_TBO=1 turns it on for experiments.
TBO = os.environ.get("DGI_TBO", "0") == "1"
# steps of <= 16 rows that carry prefill tokens (an EAGLE tree verify: N tree nodes per sequence
# under a tree mask) take the fused decode layers too — the qkv / gate_up kernels are per-row
# (norm prologue, RoPE + paged-KV epilogue at each row's own position / slot) and the attention
# dispatch already splits decode and prefill rows; 5 kernels per layer instead of 9
FUSED_SMALL_PREFILL = os.environ.get("DGI_FUSED_SMALL_PREFILL", "1") == "1"
TBO_MIN_ROWS = int(os.environ.get("DGI_TBO_MIN_ROWS", "512"))
# Fused-norm layers (``LlamaModel._forward_layers_folded``): the RMSNorm gains are folded into the
# qkv / gate_up weights once (``fold_norms``), the o-proj and down GEMMs add into the residual
# stream in their epilogue and emit its per-row sums of squares, and the qkv / gate_up GEMMs
# scale their rows by the resulting rstd — no norm kernel and no normalised copy of the stream
# between the four projections (dgi/csrc/mfma_gemm.hip EPI 2-5).  "1" (default): every eligible
# step of >= NORM_FOLD_MIN_ROWS rows of a model the engine routes GEMMs for (a shipped or measured
# routing table: the production shapes) — measured faster on the 512-row decode-role step (77.6 vs
# 78.5 ms) and on the headline's mixed steps (profiles/r6_norm/); "force": every eligible step of
# any model; "table": only where the routing table (timed on one warm weight) prices the all-MFMA
# layer at least as fast as the best mix plus the norm kernels; "0": off.  Smaller steps keep the
# skinny / fused-decode kernels.  (The fused layers round differently from the unfused ones — no
# normalised bf16 copy of the stream — so a model whose steps switch between the two computes
# near-tied greedy tokens batch-dependently; test-size engines without a routing table stay unfused.)
NORM_FOLD = os.environ.get("DGI_NORM_FOLD", "1")
NORM_FOLD_MIN_ROWS = int(os.environ.get("DGI_NORM_FOLD_MIN_ROWS", "256"))
# fused-norm layers: RoPE + the paged-KV write in the qkv GEMM's epilogue (EPI 5) where the geometry
# allows (NeoX rotary over 128-dim heads, q / kv column blocks of 256); "0" keeps rope_cache
NORM_FOLD_ROPE = os.environ.get("DGI_NORM_FOLD_ROPE", "1") != "0"
TBO_SIDE_PER_XCD = int(os.environ.get("DGI_TBO_SIDE", "4"))


def tbo_split(T: int) -> Optional[tuple]:
    """(rows of half A, rows of half B) of a T-row TBO step: B is half of T rounded down to the
    256-row GEMM tile (at least one tile), A the rest; None below ``TBO_MIN_ROWS``."""
    if T < max(512, TBO_MIN_ROWS):
        return None
    b = max(256, (T // 2) // 256 * 256)
    return T - b, b


class TboStreams:
    """The CU-masked stream pair of a device's TBO steps (created once per process)."""

    def __init__(self, device: torch.device, side_per_xcd: int):
        from dgi.utils.streams import cu_masked_stream, xcd_split
        n = torch.cuda.get_device_properties(device).multi_processor_count
        main, side = xcd_split(n, side_per_xcd)
        self.gemm = cu_masked_stream("tbo_gemm", device, main)
        self.attn = cu_masked_stream("tbo_attn", device, side)
        self.gemm_cus = len(main)
        self.events = [torch.cuda.Event() for _ in range(4)]     # q ready / attention done, per half


_TBO_STREAMS: dict = {}

def fold_decision(mode: str, rows: int, fold_impl) -> bool:
    """Whether a GPU step of ``rows`` rows runs the fused-norm layers under ``DGI_NORM_FOLD`` =
    ``mode`` (shape eligibility aside): ``fold_impl`` is the model's routing-table rule (None when
    the engine routes no GEMMs for it, e.g. test-size models)."""
    if mode == "0" or rows < NORM_FOLD_MIN_ROWS:
        return False
    if mode == "force":
        return True
    if fold_impl is None:
        return False
    return mode == "1" or (mode == "table" and bool(fold_impl(rows)))


def _ss_cols(hidden: int) -> int:
    """Columns of the fused-norm row statistics: one partial per 256-column tile of the stream,
    padded to a multiple of 8 (the consumer's vector loads; the pad columns stay zero)."""
    return (hidden // 256 + 7) // 8 * 8


class LlamaLayerWeights:
    __slots__ = ("in_norm", "qkv", "o", "post_norm", "gate_up", "down", "qkv_bias")

    def __init__(self, in_norm, qkv, o, post_norm, gate_up, down, qkv_bias=None):
        self.in_norm, self.qkv, self.o = in_norm, qkv, o
        self.post_norm, self.gate_up, self.down = post_norm, gate_up, down
        self.qkv_bias = qkv_bias   # [qkv_size] for Qwen2, else None (fused into the QKV GEMM epilogue)


def _rand(shape, gen, device, dtype, std):
    t = torch.empty(shape, device=device, dtype=dtype)
    t.normal_(0.0, std, generator=gen)
    return t


class LlamaModel:
    """Layer range [layer_start, layer_end) of a Llama causal LM."""

    def __init__(self, cfg: ModelConfig, device: torch.device | str = "cpu", dtype=torch.bfloat16,
                 layer_start: int = 0, layer_end: Optional[int] = None, has_embed: Optional[bool] = None,
                 has_head: Optional[bool] = None, seed: int = 0, init: str = "random",
                 checkpoint: Optional[str] = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.layer_start = layer_start
        self.layer_end = cfg.num_layers if layer_end is None else layer_end
        self.has_embed = (layer_start == 0) if has_embed is None else has_embed
        self.has_head = (self.layer_end == cfg.num_layers) if has_head is None else has_head
        self.num_local_layers = self.layer_end - self.layer_start
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.kv_cache: Optional[torch.Tensor] = None  # [L_local, 2, NB, nkv, bs, hd]
        self.layers: list[LlamaLayerWeights] = []
        self.embed = self.norm = self.lm_head = None
        # EAGLE-3 feature taps: global layer ids whose output residual stream is kept
        self.capture_layers: tuple = ()
        self.captured: dict = {}
        self.force_fused = False
        # tensor parallelism: in-place sum of partial outputs across the TP group
        # after the row-parallel O and down projections (dgi.parallel.tensor)
        self.reduce = None
        # MLP row padding (dgi.runtime.gemm_pad): T -> rows to run gate_up/down on
        self.mlp_pad = None
        self.mlp_impl = None     # rows -> (gate_up on the MFMA SwiGLU kernel, down on the MFMA kernel)
        self.proj_impl = None    # rows -> (QKV on the MFMA kernel, o-proj on the MFMA kernel)
        self._attn_stream = None
        # called with the global layer id once that layer's KV is in the cache
        # (P/D layer-streamed migration sends finished layers while later ones compute)
        self.layer_hook = None
        self._pad_buf: Optional[torch.Tensor] = None
        self._attn_buf: Optional[torch.Tensor] = None
        self.load_info: Optional[dict] = None
        self.norms_folded = False    # fold_norms ran: in_norm / post_norm are ones, qkv / gate_up carry the gains
        self.fold_impl = None        # rows -> run the fused-norm layers? (dgi.runtime.gemm_pad)
        self._ss_buf: Optional[torch.Tensor] = None
        if checkpoint:
            # real weights: only this rank's layers / TP slices are read (dgi.models.weights)
            from dgi.models.weights import load_checkpoint
            self._init_empty()
            self.load_info = load_checkpoint(self, checkpoint, getattr(self, "tp_rank", 0), getattr(self, "tp", 1))
        elif init == "random":
            self._init_random(seed)
        elif init == "empty":
            self._init_empty()
        self.cos_sin = ops.rope_cos_sin(cfg.rope_dim, cfg.max_position, cfg.rope_theta, cfg.rope_scaling,
                                        device=self.device)
        self.rope_mode = 1 if cfg.rope_interleaved else 0

    # ------------------------------------------------------------------ weights
    def _init_empty(self):
        c, dev, dt = self.cfg, self.device, self.dtype
        H, I = c.hidden_size, c.intermediate_size
        for _ in range(self.num_local_layers):
            self.layers.append(LlamaLayerWeights(
                torch.ones(H, device=dev, dtype=dt), torch.empty(c.qkv_size, H, device=dev, dtype=dt),
                torch.empty(H, c.q_size, device=dev, dtype=dt), torch.ones(H, device=dev, dtype=dt),
                torch.empty(2 * I, H, device=dev, dtype=dt), torch.empty(H, I, device=dev, dtype=dt),
                torch.zeros(c.qkv_size, device=dev, dtype=dt) if c.qkv_bias else None))
        if self.has_embed:
            self.embed = torch.empty(c.vocab_size, H, device=dev, dtype=dt)
        if self.has_head:
            self.norm = torch.ones(H, device=dev, dtype=dt)
            self.lm_head = self.embed if (c.tie_embeddings and self.embed is not None) else \
                torch.empty(c.vocab_size, H, device=dev, dtype=dt)

    def _init_random(self, seed: int):
        """Deterministic per-layer seeds, initialised directly on the device.

        Any rank can re-materialise its own layer range without I/O, and a
        layer's weights do not depend on how the model is sharded (SURVEY
        §5.5), so PP=k outputs equal PP=1 outputs bit for bit."""
        c, dev, dt = self.cfg, self.device, self.dtype
        H, I = c.hidden_size, c.intermediate_size
        std = 0.02
        gen = torch.Generator(device=dev)
        for li in range(self.layer_start, self.layer_end):
            gen.manual_seed(seed * 1000003 + li * 7919 + 1)
            ln1 = 1.0 + 0.1 * _rand((H,), gen, dev, torch.float32, 1.0)
            qkv = _rand((c.qkv_size, H), gen, dev, dt, std)
            o = _rand((H, c.q_size), gen, dev, dt, std / math.sqrt(2 * c.num_layers))
            ln2 = 1.0 + 0.1 * _rand((H,), gen, dev, torch.float32, 1.0)
            gu = _rand((2 * I, H), gen, dev, dt, std)
            down = _rand((H, I), gen, dev, dt, std / math.sqrt(2 * c.num_layers))
            bias = _rand((c.qkv_size,), gen, dev, dt, std) if c.qkv_bias else None
            self.layers.append(LlamaLayerWeights(ln1.to(dt), qkv, o, ln2.to(dt), gu, down, bias))
        if self.has_embed or (self.has_head and c.tie_embeddings):
            gen.manual_seed(seed * 1000003 + 17)
            emb = _rand((c.vocab_size, H), gen, dev, dt, 1.0)
            self.embed = emb if self.has_embed else None
        if self.has_head:
            gen.manual_seed(seed * 1000003 + 23)
            self.norm = (1.0 + 0.1 * _rand((H,), gen, dev, torch.float32, 1.0)).to(dt)
            if c.tie_embeddings:
                self.lm_head = emb
            else:
                self.lm_head = _rand((c.vocab_size, H), gen, dev, dt, std)

    def fold_norms(self) -> None:
        """Fold each layer's RMSNorm gains into the projection that consumes the norm:
        qkv <- qkv * diag(in_norm), gate_up <- gate_up * diag(post_norm) (fp32 product,
        rounded once), and the gains become ones.  Every forward path computes the same
        function afterwards (the unfused norms multiply by ones); the fused-norm layers need
        it.  Idempotent; reloading weights clears the flag."""
        if self.norms_folded:
            return
        with torch.no_grad():
            for L in self.layers:
                for w, g in ((L.qkv, L.in_norm), (L.gate_up, L.post_norm)):
                    gf = g.float()[None]
                    step = max(1, (64 << 20) // (4 * w.shape[1]))      # bounded fp32 temporaries
                    for r0 in range(0, w.shape[0], step):
                        blk = w[r0:r0 + step]
                        blk.copy_((blk.float() * gf).to(w.dtype))
                    g.fill_(1.0)
            if self.layers and self.cfg.hidden_size % 256 == 0:
                # the row statistics of the fused-norm layers, allocated here so a graph capture
                # never allocates it (steps of more rows grow it eagerly)
                self._ss_buf = torch.zeros(16384, _ss_cols(self.cfg.hidden_size), device=self.device,
                                           dtype=torch.float32)
        self.norms_folded = True

    def load_state_dict_hf(self, sd: dict):
        """Load HF Llama tensor names (``model.layers.N.self_attn.q_proj.weight``...)."""
        self.norms_folded = False
        c = self.cfg
        for i, li in enumerate(range(self.layer_start, self.layer_end)):
            p = f"model.layers.{li}."
            L = self.layers[i]
            qkv = torch.cat([sd[p + "self_attn.q_proj.weight"], sd[p + "self_attn.k_proj.weight"],
                             sd[p + "self_attn.v_proj.weight"]], 0)
            L.qkv.copy_(qkv)
            if L.qkv_bias is not None:
                L.qkv_bias.copy_(torch.cat([sd[p + "self_attn.q_proj.bias"], sd[p + "self_attn.k_proj.bias"],
                                            sd[p + "self_attn.v_proj.bias"]], 0))
            L.o.copy_(sd[p + "self_attn.o_proj.weight"])
            if p + "mlp.gate_up_proj.weight" in sd:     # GLM: fused [gate; up]
                L.gate_up.copy_(sd[p + "mlp.gate_up_proj.weight"])
            else:
                L.gate_up.copy_(torch.cat([sd[p + "mlp.gate_proj.weight"], sd[p + "mlp.up_proj.weight"]], 0))
            L.down.copy_(sd[p + "mlp.down_proj.weight"])
            L.in_norm.copy_(sd[p + "input_layernorm.weight"])
            L.post_norm.copy_(sd[p + "post_attention_layernorm.weight"])
        if self.has_embed:
            self.embed.copy_(sd["model.embed_tokens.weight"])
        if self.has_head:
            self.norm.copy_(sd["model.norm.weight"])
            if "lm_head.weight" in sd and self.lm_head is not self.embed:
                self.lm_head.copy_(sd["lm_head.weight"])
        del c

    def tensors(self):
        """(name, tensor) pairs of every weight (lm_head omitted when tied)."""
        for i, L in enumerate(self.layers):
            for k in LlamaLayerWeights.__slots__:
                if getattr(L, k) is not None:
                    yield f"layers.{self.layer_start + i}.{k}", getattr(L, k)
        for k in ("embed", "norm"):
            t = getattr(self, k)
            if t is not None:
                yield k, t
        if self.lm_head is not None and self.lm_head is not self.embed:
            yield "lm_head", self.lm_head

    def copy_from(self, other: "LlamaModel") -> "LlamaModel":
        """Copy weights of the overlapping layer range from another instance
        (any device) — used to compare CPU / GPU / sharded models exactly."""
        src = dict(other.tensors())
        self.norms_folded = other.norms_folded
        for name, t in self.tensors():
            if name in src:
                t.copy_(src[name])
        return self

    def weight_bytes(self) -> int:
        n = 0
        for L in self.layers:
            for t in (L.in_norm, L.qkv, L.o, L.post_norm, L.gate_up, L.down, L.qkv_bias):
                if t is not None:
                    n += t.numel() * t.element_size()
        for t in (self.embed, self.norm):
            if t is not None:
                n += t.numel() * t.element_size()
        if self.lm_head is not None and self.lm_head is not self.embed:
            n += self.lm_head.numel() * self.lm_head.element_size()
        return n

    # ------------------------------------------------------------------ forward
    def attention(self, li: int, qkv: torch.Tensor, meta: AttnMeta, rope: bool = True,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
        c = self.cfg
        kc = self.kv_cache[li, 0]
        vc = self.kv_cache[li, 1]
        if rope:       # else the qkv GEMM epilogue already rotated q/k and wrote the cache
            ops.rope_cache(qkv, meta.positions, self.cos_sin, c.num_heads, c.num_kv_heads, c.head_dim,
                           meta.slot_mapping, kc, vc, self.rope_mode)
        T = qkv.shape[0]
        if out is None:
            out = torch.empty(T, c.q_size, device=qkv.device, dtype=qkv.dtype)
        nd = meta.num_decode
        # mixed step: the decode rows' split-KV attention (HBM-latency bound) runs on a side
        # stream beside the prefill rows' flash attention; joined before the o-proj
        side = None
        if ATTN_OVERLAP and nd > 0 and meta.num_prefill_tokens > 0 and qkv.is_cuda \
                and not torch.cuda.is_current_stream_capturing():
            side = self._attn_stream
            if side is None or side.device != qkv.device:
                from dgi.utils.streams import named_stream
                side = self._attn_stream = named_stream("attn_side", qkv.device)
            main = torch.cuda.current_stream()
            side.wait_stream(main)
        if nd > 0:
            with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
                ops.paged_decode(qkv[:nd], kc, vc, meta.dec_block_tables, meta.dec_context_lens, c.num_heads,
                                 c.num_kv_heads, self.scale, meta.dec_max_splits, meta.dec_part_size,
                                 out=out[:nd], workspace=meta.dec_workspace)
        if meta.num_prefill_tokens > 0:
            ops.paged_prefill(qkv[nd:], kc, vc, meta.pre_block_tables, meta.pre_cu_seqlens, meta.pre_context_lens,
                              c.num_heads, c.num_kv_heads, self.scale, tiles=meta.pre_tiles,
                              tree_mask=meta.tree_mask, tree_n=meta.tree_n, out=out[nd:])
        if side is not None:
            main.wait_stream(side)
        return out

    def _mlp_rows(self, T: int, like: torch.Tensor) -> int:
        """Padded MLP row count for a T-row step, and the o-proj buffer it needs."""
        if self.mlp_pad is None or not like.is_cuda or torch.cuda.is_current_stream_capturing():
            return T
        Mp = self.mlp_pad(T)
        if Mp <= T:
            return T
        buf = self._pad_buf
        if buf is None or buf.shape[0] < Mp or buf.dtype != like.dtype or buf.device != like.device:
            buf = self._pad_buf = torch.empty(max(Mp, 4096), like.shape[1], dtype=like.dtype, device=like.device)
        buf[T:Mp].zero_()       # pad rows: zeros in, ignored out
        if OPROJ_PAD:           # attention output rows past T stay zero for the padded o-proj
            ab = self._attn_buf
            q = self.cfg.q_size
            if ab is None or ab.shape[0] < Mp or ab.dtype != like.dtype or ab.device != like.device:
                ab = self._attn_buf = torch.empty(max(Mp, 4096), q, dtype=like.dtype, device=like.device)
            ab[T:Mp].zero_()
        return Mp

    def _fused_decode(self, h: torch.Tensor, meta: AttnMeta) -> tuple:
        """(fuse qkv, fuse gate_up) for this step; (False, False) = unfused layers."""
        T, H = h.shape[0], self.cfg.hidden_size
        if meta.num_prefill_tokens != 0 and not (FUSED_SMALL_PREFILL and T <= 16):
            return False, False
        if not ((h.is_cuda and h.dtype == torch.bfloat16) or self.force_fused):
            return False, False
        # force_fused: run the fused composition through the reference ops on CPU (tests)
        if self.force_fused:
            return True, True
        return ops.fused_decode_ok(T, H, "qkv"), ops.fused_decode_ok(T, H, "gate_up")

    def _forward_layers_fused(self, h: torch.Tensor, meta: AttnMeta, residual: Optional[torch.Tensor],
                              fuse_qkv: bool = True, fuse_gu: bool = True):
        """Pure-decode layers with few rows: the qkv projection with its RMSNorm
        (+ residual add) prologue and RoPE + paged-KV epilogue in one kernel, and
        gate_up with RMSNorm prologue + SwiGLU epilogue (ops.fused_skinny,
        dgi/csrc/fused_decode.hip) — 5 kernels per layer instead of 9 when both
        are fused.  A fused prologue writes the updated residual to a fresh
        buffer (the old one is still being read by other workgroups); the
        unfused steps update it in place as forward_layers does."""
        c = self.cfg
        eps = c.rms_eps
        T = h.shape[0]
        rope_epi = self.rope_mode == 0 and c.head_dim == 128 and self.cos_sin.shape[1] == 128
        for i, L in enumerate(self.layers):
            kc, vc = self.kv_cache[i, 0], self.kv_cache[i, 1]
            if fuse_qkv:
                qkv = torch.empty(T, L.qkv.shape[0], dtype=h.dtype, device=h.device)
                if residual is None:
                    pro, res_out, new_res = 1, None, h
                else:
                    res_out = torch.empty_like(h)
                    pro, new_res = 2, res_out
                ops.fused_skinny(qkv, h, residual, res_out, L.in_norm, eps, L.qkv, L.qkv_bias, pro,
                                 2 if rope_epi else 0, meta.positions, self.cos_sin, meta.slot_mapping, kc, vc,
                                 c.num_heads, c.num_kv_heads)
                residual = new_res
                attn = self.attention(i, qkv, meta, rope=not rope_epi)
            else:
                if residual is None:
                    residual = h
                    h = ops.rmsnorm(h, L.in_norm, eps)
                else:
                    ops.fused_add_rmsnorm(h, residual, L.in_norm, eps)
                attn = self.attention(i, ops.linear(h, L.qkv, L.qkv_bias), meta)
            h = ops.decode_proj(attn, L.o)
            if self.reduce is not None:
                self.reduce(h)
            if fuse_gu:
                act = torch.empty(T, L.gate_up.shape[0] // 2, dtype=h.dtype, device=h.device)
                res_out = torch.empty_like(h)
                ops.fused_skinny(act, h, residual, res_out, L.post_norm, eps, L.gate_up, None, 2, 1)
                residual = res_out
            else:
                ops.fused_add_rmsnorm(h, residual, L.post_norm, eps)
                act = ops.silu_mul(ops.linear(h, L.gate_up))
            h = ops.linear(act, L.down)
            if self.reduce is not None:
                self.reduce(h)
            if self.capture_layers and (self.layer_start + i) in self.capture_layers:
                self.captured[self.layer_start + i] = h + residual
            if self.layer_hook is not None:
                self.layer_hook(self.layer_start + i)
        return h, residual

    # ------------------------------------------------------------------ fused-norm layers
    def _fold_ok(self, h: torch.Tensor) -> bool:
        if NORM_FOLD == "0" or self.reduce is not None:
            return False
        if not h.is_cuda:           # "force-cpu": the same composition through the reference ops (tests)
            return NORM_FOLD == "force-cpu" and h.shape[0] >= NORM_FOLD_MIN_ROWS and self.layers[0].qkv_bias is None
        if h.dtype != torch.bfloat16:
            return False
        T = h.shape[0]
        if T < NORM_FOLD_MIN_ROWS:
            return False
        L = self.layers[0]
        if L.qkv_bias is not None or self.cfg.hidden_size % 256 or self.cfg.hidden_size > 8192:
            return False
        if torch.cuda.is_current_stream_capturing() and not self.norms_folded:
            return False            # weights are folded eagerly, never inside a capture
        ok = getattr(self, "_fold_shapes_ok", None)
        if ok is None:
            x = h[:1]
            a = torch.empty(1, L.o.shape[1], device=h.device, dtype=h.dtype)
            m = torch.empty(1, L.down.shape[1], device=h.device, dtype=h.dtype)
            ok = self._fold_shapes_ok = (ops.mfma_norm_ok(x, L.qkv) and ops.mfma_norm_ok(a, L.o)
                                         and ops.mfma_norm_ok(x, L.gate_up) and ops.mfma_norm_ok(m, L.down)
                                         and (L.gate_up.shape[0] // 2) % 128 == 0)
        if not ok:
            return False
        return fold_decision(NORM_FOLD, T, self.fold_impl)

    def _forward_layers_folded(self, h: torch.Tensor, meta: AttnMeta, residual: Optional[torch.Tensor],
                               trim_last: Optional[torch.Tensor]):
        """Layers on the fused-norm MFMA GEMMs (see NORM_FOLD).  Per layer::

            qkv  = rstd(ss) * (R @ qkv'^T)        (in_norm folded into qkv')
            attn = attention(qkv)
            R   += attn @ o^T;    ss <- row sums of squares of R
            act  = SwiGLU(rstd(ss) * (R @ gate_up'^T))
            R   += act @ down^T;  ss <- ...

        R is the residual stream (updated in place); returns (R, None), or for ``trim_last``
        the last layer's MLP output of the logits rows and their stream (the unfused contract)."""
        if not self.norms_folded:
            self.fold_norms()
        c = self.cfg
        eps = c.rms_eps
        T, H = h.shape
        R = h if residual is None else h + residual      # forward() hands over a tensor it owns
        nt = _ss_cols(H)
        ss = self._ss_buf
        if ss is None or ss.shape[0] < T or ss.shape[1] != nt or ss.device != h.device:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("fused-norm layers: statistics buffer must exist before capture")
            ss = self._ss_buf = torch.zeros(max(T, 4096), nt, device=h.device, dtype=torch.float32)
        ss = ss[:T]
        ops.row_sumsq(R, ss)
        n = len(self.layers)
        rope_epi = (NORM_FOLD_ROPE and (R.is_cuda or NORM_FOLD == "force-cpu") and self.rope_mode == 0 and c.head_dim == 128
                    and self.cos_sin.shape[1] == 128 and (c.num_heads * 128) % 256 == 0
                    and (c.num_kv_heads * 128) % 256 == 0)
        for i, L in enumerate(self.layers):
            if rope_epi:
                qkv = ops.mfma_gemm_norm_rope(R, L.qkv, ss, eps, meta.positions, self.cos_sin, meta.slot_mapping,
                                              self.kv_cache[i, 0], self.kv_cache[i, 1], c.num_heads, c.num_kv_heads)
                attn = self.attention(i, qkv, meta, rope=False)
            else:
                qkv = ops.mfma_gemm_norm(R, L.qkv, ops.NORM_PLAIN, ss, eps)
                attn = self.attention(i, qkv, meta)
            if trim_last is not None and i == n - 1:
                attn = attn.index_select(0, trim_last)
                Rs = R.index_select(0, trim_last)
                ho = ops.linear(attn, L.o)
                ops.fused_add_rmsnorm(ho, Rs, L.post_norm, eps)
                out = ops.linear(ops.silu_mul(ops.linear(ho, L.gate_up)), L.down)
                if self.layer_hook is not None:
                    self.layer_hook(self.layer_start + i)
                return out, Rs
            ops.mfma_gemm_norm(attn, L.o, ops.NORM_RES, ss, eps, out=R)
            act = ops.mfma_gemm_norm(R, L.gate_up, ops.NORM_SWIGLU, ss, eps)
            ops.mfma_gemm_norm(act, L.down, ops.NORM_RES, ss, eps, out=R)
            if self.capture_layers and (self.layer_start + i) in self.capture_layers:
                self.captured[self.layer_start + i] = R.clone()
            if self.layer_hook is not None:
                self.layer_hook(self.layer_start + i)
        return R, None

    # ------------------------------------------------------------------ two-batch overlap
    def _tbo_ok(self, h: torch.Tensor, meta: AttnMeta, trim_last) -> Optional[tuple]:
        if not (TBO and h.is_cuda and self.layers and meta.num_prefill_tokens == 0 and trim_last is None
                and self.reduce is None and not self.capture_layers and self.layer_hook is None
                and h.dtype == torch.bfloat16 and not torch.cuda.is_current_stream_capturing()):
            return None
        return tbo_split(h.shape[0])

    @staticmethod
    def _rows_meta(meta: AttnMeta, a: int, b: int) -> AttnMeta:
        """Decode metadata of rows [a, b) of a pure-decode step."""
        return AttnMeta(positions=meta.positions[a:b], slot_mapping=meta.slot_mapping[a:b], num_decode=b - a,
                        dec_block_tables=meta.dec_block_tables[a:b], dec_context_lens=meta.dec_context_lens[a:b],
                        dec_max_splits=meta.dec_max_splits, dec_part_size=meta.dec_part_size,
                        dec_workspace=meta.dec_workspace, num_prefill_tokens=0, logits_indices=None)

    def _forward_layers_tbo(self, h: torch.Tensor, meta: AttnMeta, residual: Optional[torch.Tensor], split: tuple):
        """Pure-decode layers as two halves A | B: half X's attention (RoPE + paged KV write +
        split-KV decode attention) runs on the side stream's CUs while the GEMM stream runs
        the other half's o-proj, MLP and next QKV, so the attention (~23 % of a 768-row 70B
        stage step) hides under GEMMs instead of following them.  Per layer, in issue order::

            gemm: pre(A, i+1) | post(B, i) pre(B, i+1) | post(A, i+1) ...
            attn:        attn(A, i+1) ->         attn(B, i+1) -> ...

        pre = (add +) RMSNorm + QKV GEMM; post = o-proj + add + RMSNorm + gate_up (SwiGLU) + down.
        Row-independent, so the outputs equal the one-batch step's up to GEMM blocking."""
        dev = h.device
        st = _TBO_STREAMS.get(dev.index)
        if st is None:
            st = _TBO_STREAMS[dev.index] = TboStreams(dev, TBO_SIDE_PER_XCD)
        G, S = st.gemm, st.attn
        eq = st.events[:2]
        ea = st.events[2:]
        c = self.cfg
        eps = c.rms_eps
        T = h.shape[0]
        na = split[0]
        bounds = ((0, na), (na, T))
        metas = [self._rows_meta(meta, a, b) for a, b in bounds]
        main = torch.cuda.current_stream()
        G.wait_stream(main)
        S.wait_stream(main)
        hs = [h[a:b] for a, b in bounds]
        res = [None if residual is None else residual[a:b] for a, b in bounds]
        rows = [b - a for a, b in bounds]
        impl = [(self.mlp_impl(r) if self.mlp_impl is not None else (False, False)) +
                (self.proj_impl(r) if self.proj_impl is not None else (False, False)) for r in rows]
        qkv = [None, None]
        att = [None, None]
        n = len(self.layers)
        ops.set_gemm_cus(st.gemm_cus)
        try:
            def pre(x, i):
                L = self.layers[i]
                if res[x] is None:
                    res[x] = hs[x]
                    hs[x] = ops.rmsnorm(hs[x], L.in_norm, eps)
                else:
                    ops.fused_add_rmsnorm(hs[x], res[x], L.in_norm, eps)
                q = ops.mfma_gemm(hs[x], L.qkv, 0) if (impl[x][2] and L.qkv_bias is None) else \
                    ops.linear(hs[x], L.qkv, L.qkv_bias)
                o = torch.empty(rows[x], c.q_size, device=dev, dtype=h.dtype)
                q.record_stream(S)
                o.record_stream(S)
                qkv[x], att[x] = q, o
                eq[x].record(G)
                with torch.cuda.stream(S):
                    S.wait_event(eq[x])
                    self.attention(i, q, metas[x], out=o)
                    ea[x].record(S)

            def post(x, i):
                L = self.layers[i]
                G.wait_event(ea[x])
                hh = ops.mfma_gemm(att[x], L.o, 0) if impl[x][3] else ops.linear(att[x], L.o)
                ops.fused_add_rmsnorm(hh, res[x], L.post_norm, eps)
                act = ops.mfma_gemm(hh, L.gate_up, 1) if impl[x][0] else ops.silu_mul(ops.linear(hh, L.gate_up))
                hs[x] = ops.mfma_gemm(act, L.down, 0) if impl[x][1] else ops.linear(act, L.down)

            with torch.cuda.stream(G):
                pre(0, 0)
                pre(1, 0)
                for i in range(n):
                    for x in (0, 1):
                        post(x, i)
                        if i + 1 < n:
                            pre(x, i + 1)
                out_h = torch.cat(hs, 0)
                out_r = torch.cat(res, 0)
        finally:
            ops.set_gemm_cus(0)
        main.wait_stream(G)
        out_h.record_stream(main)
        out_r.record_stream(main)
        return out_h, out_r

    def forward_layers(self, h: torch.Tensor, meta: AttnMeta, residual: Optional[torch.Tensor] = None,
                       trim_last: Optional[torch.Tensor] = None):
        """Run the local layers.  ``trim_last`` (row indices): the last layer's
        output is only needed for those rows (the rows that produce logits), so
        after its attention — which has written every row's K/V — its o-proj and
        MLP run on those rows alone and the returned (h, residual) hold just them."""
        c = self.cfg
        eps = c.rms_eps
        T = h.shape[0]
        if self.layers:
            split = self._tbo_ok(h, meta, trim_last)
            if split is not None:
                return self._forward_layers_tbo(h, meta, residual, split)
            if self._fold_ok(h):
                return self._forward_layers_folded(h, meta, residual, trim_last)
            fq, fg = self._fused_decode(h, meta)
            if fq or fg:
                h, residual = self._forward_layers_fused(h, meta, residual, fq, fg)
                if trim_last is not None:     # same contract as the unfused path: only the logits rows
                    h, residual = h.index_select(0, trim_last), residual.index_select(0, trim_last)
                return h, residual
        Mp = self._mlp_rows(T, h) if self.layers else T
        # hand-written MFMA GEMMs where the start-up table measured them faster (dgi.runtime.gemm_pad)
        mfma_gu, mfma_dn = self.mlp_impl(Mp) if (self.mlp_impl is not None and self.layers) else (False, False)
        mfma_q, mfma_o = self.proj_impl(T) if (self.proj_impl is not None and self.layers and h.is_cuda
                                               and not torch.cuda.is_current_stream_capturing()) else (False, False)
        hfull = None
        for i, L in enumerate(self.layers):
            if residual is None:
                residual = h
                h = ops.rmsnorm(h, L.in_norm, eps)
            else:
                ops.fused_add_rmsnorm(h, residual, L.in_norm, eps)
            if hfull is not None:
                # the previous MLP ran on Mp padded rows (zeros past T): the QKV GEMM
                # reuses them, at the row count the start-up table timed for the layer
                qkv = ops.linear(hfull, L.qkv, L.qkv_bias)[:T]
            elif mfma_q and L.qkv_bias is None:
                qkv = ops.mfma_gemm(h, L.qkv, 0)
            else:
                qkv = ops.linear(h, L.qkv, L.qkv_bias)
            last = trim_last is not None and i == len(self.layers) - 1
            attn_pad = Mp > T and OPROJ_PAD and not last
            attn = self.attention(i, qkv, meta, out=self._attn_buf[:T] if attn_pad else None)
            if last:
                attn = attn.index_select(0, trim_last)
                residual = residual.index_select(0, trim_last)
                h = ops.linear(attn, L.o)
                if self.reduce is not None:
                    self.reduce(h)
                ops.fused_add_rmsnorm(h, residual, L.post_norm, eps)
                h = ops.linear(ops.silu_mul(ops.linear(h, L.gate_up)), L.down)
                if self.reduce is not None:
                    self.reduce(h)
                if self.layer_hook is not None:
                    self.layer_hook(self.layer_start + i)
                break
            if attn_pad:
                # attention wrote the first T rows of a zero-padded buffer: the o-proj runs on
                # all Mp rows (zeros in, zeros out past T) straight into the MLP's input
                torch.matmul(self._attn_buf[:Mp], L.o.t(), out=self._pad_buf[:Mp])
                h = self._pad_buf[:T]
            elif Mp > T:
                # o-proj writes the first T rows of the padded MLP input
                h = ops.mfma_gemm(attn, L.o, 0, out=self._pad_buf[:T]) if mfma_o else \
                    torch.matmul(attn, L.o.t(), out=self._pad_buf[:T])
            else:
                h = ops.mfma_gemm(attn, L.o, 0) if mfma_o else ops.linear(attn, L.o)
            if self.reduce is not None:
                self.reduce(h)
            ops.fused_add_rmsnorm(h, residual, L.post_norm, eps)
            x = self._pad_buf[:Mp] if Mp > T else h
            act = ops.mfma_gemm(x, L.gate_up, 1) if mfma_gu else ops.silu_mul(ops.linear(x, L.gate_up))
            h = ops.mfma_gemm(act, L.down, 0) if mfma_dn else ops.linear(act, L.down)
            if Mp > T:
                hfull = h if QKV_PAD else None
                h = h[:T]
            if self.reduce is not None:
                self.reduce(h)
            if self.capture_layers and (self.layer_start + i) in self.capture_layers:
                self.captured[self.layer_start + i] = h + residual
            if self.layer_hook is not None:
                self.layer_hook(self.layer_start + i)
        return h, residual

    def embed_tokens(self, input_ids: torch.Tensor) -> torch.Tensor:
        return F.embedding(input_ids, self.embed)

    def forward(self, meta: AttnMeta, input_ids: Optional[torch.Tensor] = None,
                hidden: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Stage forward.  Returns logits [n, V] on the last stage, else the
        residual stream [T, H] for the next stage."""
        if self.has_embed:
            h = self.embed_tokens(input_ids)
        else:
            h = hidden
        residual = None
        idx = meta.logits_indices
        # the last layer's o-proj + MLP only for the rows that produce logits (prefill
        # chunks sample one row each): skipped when layers' hidden states are captured
        trim = (idx is not None and self.has_head and self.num_local_layers > 0 and TRIM_LAST_LAYER
                and not self.capture_layers and idx.shape[0] < h.shape[0])
        if self.num_local_layers:
            # a fresh residual tensor: fused_add_rmsnorm updates it in place
            h, residual = self.forward_layers(h.clone() if not self.has_embed else h, meta,
                                              trim_last=idx if trim else None)
        if not self.has_head:
            return h if residual is None else h + residual
        return self.compute_logits(h, residual, None if trim else idx)

    def compute_logits(self, h, residual, idx):
        eps = self.cfg.rms_eps
        if idx is not None:
            h = h.index_select(0, idx)
            residual = residual.index_select(0, idx) if residual is not None else None
        if residual is None:
            hn = ops.rmsnorm(h.contiguous(), self.norm, eps)
        else:
            h = h.contiguous()
            residual = residual.contiguous()
            ops.fused_add_rmsnorm(h, residual, self.norm, eps)
            hn = h
        return ops.linear(hn, self.lm_head)

    def final_hidden(self, h, residual, idx=None):
        """Normalised last hidden states (EAGLE draft features)."""
        eps = self.cfg.rms_eps
        if idx is not None:
            h = h.index_select(0, idx)
            residual = residual.index_select(0, idx)
        h = h.contiguous()
        residual = residual.contiguous().clone()
        ops.fused_add_rmsnorm(h, residual, self.norm, eps)
        return h
