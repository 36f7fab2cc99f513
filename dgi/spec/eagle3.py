"""EAGLE-3 speculative decoding on the native runtime.

Replaces the reference's incomplete library (worker/engines/speculative.py:
``DraftHead :78-125``, ``TreeDraftBuffer :128-245``, ``SpeculativeDecoder
:248-471``) with a working, batched, lossless
implementation whose hot paths run on the hand-written HIP kernels:

* **Draft head** (EAGLE-3): target residual-stream features of a low, a mid
  and a high layer are fused (``fc``: 3H -> H) and combined with the token
  embedding into ONE Llama decoder layer (qkv input 2H) with its own paged
  KV cache (sharing the target's block ids); the target's embedding and LM
  head are shared.
* **Tree drafting**: depth ``D``; each depth keeps the ``W`` best nodes by
  cumulative draft log-prob, each expanded to ``K`` children (``dgi_topk``).
  Draft attention over context + ancestors uses the paged prefill kernel's
  tree-mask mode (``dgi_tree_mask`` ancestor bits).
* **Verify**: one target forward over the ``N = 1 + W*D`` tree nodes of
  every sequence (paged prefill, tree mask, positions = ctx + depth);
  greedy acceptance of the longest matching root path plus the bonus token
  by ``dgi_tree_verify``; accepted KV is compacted in place (slot copy).

* **Sampled requests** (temperature > 0, top-k / top-p) speculate too, with
  *coupled* verification: every tree node gets the target's own sample for
  its output position — the same Gumbel-max draw (request seed, output index)
  non-speculative decoding makes — and a drafted child is accepted iff it
  equals its parent's target sample.  Every emitted token is therefore
  exactly the token plain sampled decoding would emit (lossless, not merely
  equal in distribution), and the acceptance probability at a node is the
  target mass of its drafted children — the most any lossless verifier can
  accept for a fixed candidate set.  Greedy rows are the temperature-0 case.
* **Adaptive depth** (reference ``_adapt_depth``, worker/engines/speculative.py:
  456-463): the active tree depth moves down when the step's acceptance rate
  is under ``min_accept_rate`` and up when it is over ``raise_accept_rate``.
* **Auto-off**: the engine times speculative and plain steps per batch
  bucket; when speculation costs more per generated token than plain
  decoding it switches to plain hipGraph decode steps (which still tap the
  EAGLE-3 features) and re-probes periodically, so it is never slower than
  plain decoding for long.

Output is token-for-token identical to non-speculative decoding (the target
decides every token).
"""
from __future__ import annotations

import dataclasses
import math
import time
from typing import Optional

import numpy as np
import torch
import torch.nn.functional as F

from dgi import ops
from dgi.engine import EngineConfig, LLMEngine, StepOutput
from dgi.kv.block_pool import OutOfBlocks
from dgi.models.config import ModelConfig
from dgi.models.llama import LlamaModel, _rand
from dgi.runtime.batch import AttnMeta
from dgi.sched.request import Request
from dgi.runtime.model_runner import graph_capture


@dataclasses.dataclass
class SpecConfig:
    depth: int = 5            # draft tree depth D (max accepted drafts per step)
    width: int = 3            # frontier nodes kept per depth W (3 x depth 5 + root = 16 nodes: a batch-1
                              # verify fits the fused decode layers, profiles/r5_spec/)
    topk: int = 4             # children per frontier node K (<= 16, dgi_topk)
    feature_layers: Optional[tuple] = None  # default: (2, L//2, L-3)
    graphs: bool = True       # hipGraph-capture the tree verify pass per batch bucket (GPU)
    adaptive_depth: bool = True       # reference SpeculativeConfig.adaptive_depth
    min_accept_rate: float = 0.3      # reference SpeculativeConfig.min_accept_rate: shrink below it
    raise_accept_rate: float = 0.7    # grow above it (reference _adapt_depth)
    auto_off: bool = True             # fall back to plain decode while speculation is slower
    probe_every: int = 48             # plain steps between speculation re-probes
    min_gain: float = 0.07            # speculation stays on only if >= 7 % cheaper per token than plain
                                      # (its per-step host work and async tail are partly outside the timer)

    @property
    def num_nodes(self) -> int:
        return 1 + self.width * self.depth

    def nodes(self, depth: int) -> int:
        return 1 + self.width * depth

    def validate(self) -> None:
        if self.num_nodes > 64:
            raise ValueError("tree of more than 64 nodes (ancestor masks are 64-bit)")
        if not 1 <= self.width <= self.topk <= 16:
            raise ValueError("need 1 <= width <= topk <= 16")


def default_feature_layers(num_layers: int) -> tuple:
    lo = min(2, num_layers - 1)
    return (lo, num_layers // 2, max(num_layers - 3, 0))


class Eagle3Draft:
    """One-layer EAGLE-3 draft decoder sharing the target's embedding / LM head."""

    def __init__(self, target: LlamaModel, num_blocks: int, block_size: int, seed: int = 1234):
        c = target.cfg
        self.target = target
        self.cfg = c
        dev, dt = target.device, target.dtype
        H, I = c.hidden_size, c.intermediate_size
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed)
        std = 0.02
        self.fc = _rand((H, 3 * H), gen, dev, dt, std)
        self.embed_norm = torch.ones(H, device=dev, dtype=dt)
        self.hidden_norm = torch.ones(H, device=dev, dtype=dt)
        self.qkv = _rand((c.qkv_size, 2 * H), gen, dev, dt, std)
        self.o = _rand((H, c.q_size), gen, dev, dt, std / math.sqrt(2))
        self.post_norm = torch.ones(H, device=dev, dtype=dt)
        self.gate_up = _rand((2 * I, H), gen, dev, dt, std)
        self.down = _rand((H, I), gen, dev, dt, std / math.sqrt(2))
        self.norm = torch.ones(H, device=dev, dtype=dt)
        self.kv_cache = torch.zeros(1, 2, num_blocks, c.num_kv_heads, block_size, c.head_dim, device=dev, dtype=dt)
        self.scale = 1.0 / math.sqrt(c.head_dim)
        # draft vocabulary (EAGLE-3 "hot" vocabulary): the draft scores only these token ids, so
        # each draft depth streams a [V', H] head instead of the target's [V, H] one (Llama-3:
        # 128k -> 32k rows, 0.79 of 1.05 GB per depth); None = the whole vocabulary
        self.hot: Optional[torch.Tensor] = None
        self.hot_head: Optional[torch.Tensor] = None
        self.vocab_version = 0      # bumped by set_hot_vocab: captured graphs of older versions are stale

    def set_hot_vocab(self, ids: Optional[torch.Tensor]) -> None:
        """Restrict the draft's proposals to token ids ``ids`` (None: every token).  Graphs
        captured before the call read the old head (or the full-vocabulary path): the engine
        drops them when it sees ``vocab_version`` move."""
        self.vocab_version += 1
        if ids is None:
            self.hot = self.hot_head = None
            return
        self.hot = torch.as_tensor(ids, dtype=torch.long, device=self.target.device).sort().values
        self.hot_head = self.target.lm_head.index_select(0, self.hot).contiguous()

    def to_token(self, idx: torch.Tensor) -> torch.Tensor:
        """Token ids of draft-vocabulary indices (``logprobs`` columns)."""
        return idx.long() if self.hot is None else self.hot[idx.long()]

    # ------------------------------------------------------------------ params (training / checkpoints)
    PARAM_NAMES = ("fc", "embed_norm", "hidden_norm", "qkv", "o", "post_norm", "gate_up", "down", "norm")

    def parameters(self) -> dict:
        return {k: getattr(self, k) for k in self.PARAM_NAMES}

    def load(self, params: dict) -> None:
        for k in self.PARAM_NAMES:
            getattr(self, k).copy_(params[k])

    # ------------------------------------------------------------------ inference (paged KV, HIP kernels)
    def fuse(self, feats: torch.Tensor) -> torch.Tensor:
        return ops.linear(feats, self.fc)

    def forward(self, ids: torch.Tensor, hidden: torch.Tensor, meta: AttnMeta) -> torch.Tensor:
        """Draft hidden states g [T, H] (pre-norm residual stream)."""
        c = self.cfg
        eps = c.rms_eps
        e = ops.rmsnorm(F.embedding(ids, self.target.embed), self.embed_norm, eps)
        hn = ops.rmsnorm(hidden.contiguous(), self.hidden_norm, eps)
        qkv = ops.linear(torch.cat([e, hn], dim=-1), self.qkv)
        kc, vc = self.kv_cache[0, 0], self.kv_cache[0, 1]
        ops.rope_cache(qkv, meta.positions, self.target.cos_sin, c.num_heads, c.num_kv_heads, c.head_dim,
                       meta.slot_mapping, kc, vc, self.target.rope_mode)
        attn = ops.paged_prefill(qkv, kc, vc, meta.pre_block_tables, meta.pre_cu_seqlens, meta.pre_context_lens,
                                 c.num_heads, c.num_kv_heads, self.scale, tiles=meta.pre_tiles,
                                 tree_mask=meta.tree_mask, tree_n=meta.tree_n)
        h = ops.linear(attn, self.o)
        residual = hidden.contiguous().clone()
        ops.fused_add_rmsnorm(h, residual, self.post_norm, eps)   # residual <- h + hidden ; h <- norm
        h = ops.linear(ops.silu_mul(ops.linear(h, self.gate_up)), self.down)
        return h + residual

    def topk(self, g: torch.Tensor, k: int) -> tuple:
        """(log-prob, draft-vocabulary index) of the ``k`` most likely next tokens per row of
        ``g`` — ``ops.topk(self.logprobs(g), k)`` without the fp32 log-prob matrix (one fused
        top-k + logsumexp pass over the bf16 logits, ``ops.topk_logprobs``)."""
        hn = ops.rmsnorm(g.contiguous(), self.norm, self.cfg.rms_eps)
        head = self.hot_head if self.hot_head is not None else self.target.lm_head
        return ops.topk_logprobs(ops.linear(hn, head), k)

    def logprobs(self, g: torch.Tensor) -> torch.Tensor:
        """Log-probabilities over the draft vocabulary (columns index ``hot`` when set)."""
        hn = ops.rmsnorm(g.contiguous(), self.norm, self.cfg.rms_eps)
        head = self.hot_head if self.hot_head is not None else self.target.lm_head
        return torch.log_softmax(ops.linear(hn, head).float(), dim=-1)

    # ------------------------------------------------------------------ training (dense, autograd)
    def train_forward(self, P: dict, ids: torch.Tensor, hidden: torch.Tensor, pos: torch.Tensor) -> torch.Tensor:
        """Dense causal forward over [B, S] for self-distillation (plain torch ops)."""
        c = self.cfg
        eps = c.rms_eps

        def rms(x, w):
            xf = x.float()
            return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype) * w

        B, S = ids.shape
        e = rms(F.embedding(ids, self.target.embed), P["embed_norm"])
        qkv = F.linear(torch.cat([e, rms(hidden, P["hidden_norm"])], -1), P["qkv"])
        nh, nkv, hd = c.num_heads, c.num_kv_heads, c.head_dim
        q, k, v = qkv.split([nh * hd, nkv * hd, nkv * hd], -1)
        cs = self.target.cos_sin[pos.long()].reshape(B * S, -1).float()   # [B*S, rd] (cos | sin halves)

        def rot(x, n):   # differentiable RoPE, same pairing / partial dims as the target's kernel
            y = ops._rope(x.reshape(B * S, n, hd).float(), cs, self.target.rope_mode)
            return y.view(B, S, n, hd).to(qkv.dtype)
        q, k = rot(q, nh), rot(k, nkv)
        v = v.view(B, S, nkv, hd)
        rep = nh // nkv
        k = k.repeat_interleave(rep, 2)
        v = v.repeat_interleave(rep, 2)
        a = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=True)
        h = F.linear(a.transpose(1, 2).reshape(B, S, nh * hd), P["o"]) + hidden
        m = F.linear(rms(h, P["post_norm"]), P["gate_up"])
        g_, u_ = m.chunk(2, -1)
        return F.linear(F.silu(g_) * u_, P["down"]) + h

    def train_logits(self, P: dict, g: torch.Tensor) -> torch.Tensor:
        xf = g.float()
        hn = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.cfg.rms_eps)).to(g.dtype) * P["norm"]
        return F.linear(hn, self.target.lm_head)


class _SpecState:
    __slots__ = ("draft_len", "feat_start", "_feat", "chunks", "n_chunked")

    def __init__(self, draft_len: int):
        self.draft_len = draft_len      # positions [0, draft_len) have draft KV
        self.feat_start = 0             # position of feat[0]
        self._feat: Optional[torch.Tensor] = None   # fused target features [m, H]
        self.chunks: list = []          # appended rows not yet concatenated (plain decode steps)
        self.n_chunked = 0

    @property
    def feat(self) -> Optional[torch.Tensor]:
        if self.chunks:                 # one concatenation per spec step, not one per plain step
            parts = ([self._feat] if self._feat is not None else []) + self.chunks
            self._feat = torch.cat(parts)
            self.chunks, self.n_chunked = [], 0
        return self._feat

    @feat.setter
    def feat(self, v: Optional[torch.Tensor]) -> None:
        self._feat, self.chunks, self.n_chunked = v, [], 0

    def rows(self) -> int:
        return (0 if self._feat is None else self._feat.shape[0]) + self.n_chunked


def _varlen_meta(runner, positions, slots, block_rows, cu, ctx, device, tree_mask=None, tree_n=0,
                 logits_idx=None) -> AttnMeta:
    """Prefill-style metadata from host arrays (one H2D copy)."""
    nb = len(ctx)
    maxw = runner.max_blocks
    bt = np.zeros((nb, maxw), np.int32)
    for i, blk in enumerate(block_rows):
        bt[i, : len(blk)] = blk
    tiles = [(j, t0) for j in range(nb) for t0 in range(0, int(cu[j + 1] - cu[j]), ops.PREFILL_TILE)]
    tiles_np = np.asarray(tiles, np.int32).reshape(-1, 2)
    parts = [np.asarray(positions, np.int32), np.asarray(slots, np.int32), bt.ravel(), np.asarray(cu, np.int32),
             np.asarray(ctx, np.int32), tiles_np.ravel()]
    flat = np.concatenate(parts)
    dev = runner.to_device(flat)
    o = 0
    views = []
    for p in parts:
        views.append(dev[o: o + p.size])
        o += p.size
    d_pos, d_slots, d_bt, d_cu, d_ctx, d_tiles = views
    return AttnMeta(positions=d_pos, slot_mapping=d_slots, num_decode=0, num_prefill_tokens=int(cu[-1]),
                    pre_block_tables=d_bt.view(nb, maxw), pre_cu_seqlens=d_cu, pre_context_lens=d_ctx,
                    pre_tiles=d_tiles.view(-1, 2), tree_mask=tree_mask, tree_n=tree_n, logits_indices=logits_idx)


def kv_slot_copy(kv: torch.Tensor, src: torch.Tensor, dst: torch.Tensor, block_size: int) -> None:
    """Copy token slots (all layers, K and V) inside a paged cache [L, 2, NB, nkv, bs, hd]:
    every source is read before any destination is written (a compaction chain's source can
    be another move's destination).  GPU: two HIP kernels (kv_ops.hip: gather, scatter)."""
    if ops._native(kv) and kv.dtype in (torch.bfloat16, torch.float16):
        torch.ops.dgi.kv_slot_copy(kv, src.to(torch.int32).contiguous(), dst.to(torch.int32).contiguous())
        return
    L, two, NB, nkv, bs, hd = kv.shape
    c = kv.view(L * two, NB, nkv, bs, hd)
    src, dst = src.long(), dst.long()
    vals = c[:, src // bs, :, src % bs]          # [n, L*2, nkv, hd] (advanced dims first)
    c[:, dst // bs, :, dst % bs] = vals


VERIFY_BUCKETS = (1, 2, 4, 8, 16, 32, 64, 128)


class _VerifyGraph:
    """hipGraph of the tree-verify pass for ``Rb`` sequences of ``N`` tree nodes.

    Static inputs: one int32 metadata buffer (positions, slots, block tables,
    context lengths; cu_seqlens and tiles are fixed by Rb and N), draft
    tokens and tree parents.  The graph runs the ancestor masks, the target
    forward with EAGLE-3 feature capture (tree-masked paged prefill
    attention), argmax and ``tree_verify``.  Rows past the live batch are
    padding that reads/writes only the reserved scratch page 0."""

    def __init__(self, eng: "SpecEngine", Rb: int, depth: int):
        sp, run = eng.spec, eng.runner
        N, dev = sp.nodes(depth), eng.device
        self.eng = eng
        self.depth = depth
        self.Rb, self.N, self.maxw = Rb, N, run.max_blocks
        T = Rb * N
        # per-node sampling parameters of the coupled verification (temperature 0 = argmax)
        self.temps = torch.zeros(T, dtype=torch.float32, device=dev)
        self.seeds = torch.zeros(T, dtype=torch.long, device=dev)
        self.topk = torch.zeros(T, dtype=torch.long, device=dev)
        self.topp = torch.ones(T, dtype=torch.float32, device=dev)
        self.n_dyn = 2 * T + Rb * self.maxw + Rb            # positions, slots, block tables, ctx
        self.host = torch.zeros(self.n_dyn, dtype=torch.int32).pin_memory()
        self.dyn = torch.zeros(self.n_dyn, dtype=torch.int32, device=dev)
        self.cu = torch.arange(0, T + 1, N, dtype=torch.int32, device=dev)
        self.tiles = torch.stack([torch.arange(Rb, dtype=torch.int32), torch.zeros(Rb, dtype=torch.int32)],
                                 1).contiguous().to(dev)
        self.tok = torch.zeros(Rb, N, dtype=torch.long, device=dev)
        par = torch.full((Rb, N), -1, dtype=torch.int32)
        par[:, 1:] = 0
        self.par = par.to(dev)
        o = 0
        self.d_pos = self.dyn[o:o + T]
        o += T
        self.d_slots = self.dyn[o:o + T]
        o += T
        self.d_bt = self.dyn[o:o + Rb * self.maxw].view(Rb, self.maxw)
        o += Rb * self.maxw
        self.d_ctx = self.dyn[o:o + Rb]
        self._fill_padding(0)
        self.dyn.copy_(self.host)
        self.graph = None
        self._capture()

    def _fill_padding(self, R: int) -> None:
        """Rows >= R: a valid dummy tree on scratch page 0 (position 0.., context N)."""
        T, N, Rb, maxw = self.Rb * self.N, self.N, self.Rb, self.maxw
        h = self.host.numpy()
        if R >= Rb:
            return
        h[R * N:T] = np.tile(np.arange(N, dtype=np.int32), Rb - R)                               # positions
        h[T + R * N:2 * T] = np.arange(N, dtype=np.int32)[None].repeat(Rb - R, 0).ravel() % \
            self.eng.pool.block_size                                                              # slots in page 0
        bt0 = 2 * T
        h[bt0 + R * maxw:bt0 + Rb * maxw] = 0
        h[bt0 + Rb * maxw + R:bt0 + Rb * maxw + Rb] = N

    def _body(self):
        eng = self.eng
        anc, depth = ops.tree_mask(self.par)
        meta = AttnMeta(positions=self.d_pos, slot_mapping=self.d_slots, num_decode=0,
                        num_prefill_tokens=self.Rb * self.N, pre_block_tables=self.d_bt, pre_cu_seqlens=self.cu,
                        pre_context_lens=self.d_ctx, pre_tiles=self.tiles, tree_mask=anc, tree_n=self.N)
        logits, feats = eng._forward_capture(meta, self.tok.view(-1))
        tgt = ops.sample(logits, self.temps, self.seeds, 0, top_k=self.topk, top_p=self.topp).view(self.Rb, self.N)
        acc, path, toks = ops.tree_verify(self.par, self.tok, tgt, anc, depth, self.depth + 1)
        return acc, path, toks, feats

    @torch.inference_mode()
    def _capture(self) -> None:
        eng = self.eng
        eng.model.kv_cache = eng.pool.kv
        from dgi.utils.streams import named_stream
        s = named_stream("capture", eng.device)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._body()                                   # warm-up (lazy inits outside capture)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize(eng.device)
        self.graph = torch.cuda.CUDAGraph()
        with graph_capture(self.graph, pool=eng._graph_pool):
            self.out = self._body()

    def run(self, R: int, tok: torch.Tensor, par: torch.Tensor, pos, slots, brows, ctx, samp):
        T, N, maxw = self.Rb * self.N, self.N, self.maxw
        temps, seeds, topk, topp = samp
        n = R * N
        self.temps[:n].copy_(temps, non_blocking=True)
        self.seeds[:n].copy_(seeds, non_blocking=True)
        self.topk[:n].copy_(topk, non_blocking=True)
        self.topp[:n].copy_(topp, non_blocking=True)
        if n < T:
            self.temps[n:].zero_()
        h = self.host.numpy()
        h[:R * N] = pos
        h[T:T + R * N] = slots
        bt0 = 2 * T
        h[bt0:bt0 + R * maxw] = 0
        for i, blk in enumerate(brows):
            h[bt0 + i * maxw: bt0 + i * maxw + len(blk)] = blk
        h[bt0 + self.Rb * maxw: bt0 + self.Rb * maxw + R] = ctx
        self._fill_padding(R)
        self.dyn.copy_(self.host, non_blocking=True)
        self.tok[:R].copy_(tok)
        self.par[:R].copy_(par)
        if R < self.Rb:
            self.tok[R:].zero_()
        self.graph.replay()
        acc, path, toks, feats = self.out
        return acc[:R], path[:R], toks[:R], feats[:R * N]


def _draft_tree(dr: "Eagle3Draft", g_root, last, lv, d_bt, W: int, D: int, K: int, N: int):
    """Tree drafting on device (root top-k, then depths 2..D), all metadata precomputed in
    ``lv`` (per depth: offset, m, positions, slots, ctx, cu, tiles): the body of the draft
    and whole-step graphs.  Returns (tokens, parents) [Rb, N]."""
    Rb, H = g_root.shape
    dev = g_root.device
    v1, t1 = dr.topk(g_root, K)
    t1 = dr.to_token(t1)
    tok = torch.zeros(Rb, N, dtype=torch.long, device=dev)
    par = torch.full((Rb, N), -1, dtype=torch.int32, device=dev)
    score = torch.zeros(Rb, N, dtype=torch.float32, device=dev)
    G = torch.zeros(Rb, N, H, dtype=g_root.dtype, device=dev)
    tok[:, 0] = last
    G[:, 0] = g_root
    tok[:, 1:W + 1] = t1[:, :W].long()
    par[:, 1:W + 1] = 0
    score[:, 1:W + 1] = v1[:, :W].float()
    for d, (_, m, pos, slots, ctx, cu, tiles) in zip(range(2, D + 1), lv):
        cpar = par[:, 1:m + 1] - 1
        cpar = torch.where(cpar < 0, torch.full_like(cpar, -1), cpar)
        anc, _ = ops.tree_mask(cpar.contiguous())
        cm = AttnMeta(positions=pos, slot_mapping=slots, num_decode=0, num_prefill_tokens=Rb * m,
                      pre_block_tables=d_bt, pre_cu_seqlens=cu, pre_context_lens=ctx, pre_tiles=tiles,
                      tree_mask=anc, tree_n=m)
        pidx = par[:, 1:m + 1].long()
        hin = torch.gather(G, 1, pidx[:, :, None].expand(Rb, m, H)).reshape(Rb * m, H)
        gc = dr.forward(tok[:, 1:m + 1].reshape(-1), hin, cm).view(Rb, m, H)
        G[:, 1:m + 1] = gc
        fr = torch.arange(m - W + 1, m + 1, device=dev)
        vf, tf = dr.topk(gc[:, m - W:].reshape(Rb * W, H), K)
        tf = dr.to_token(tf)
        cand = (score[:, fr][:, :, None] + vf.view(Rb, W, K).float()).view(Rb, W * K)
        best, bi = torch.topk(cand, W, dim=1)
        base = 1 + W * (d - 1)
        tok[:, base: base + W] = torch.gather(tf.view(Rb, W * K).long(), 1, bi)
        par[:, base: base + W] = fr[bi // K].int()
        score[:, base: base + W] = best
    return tok, par


class _DraftGraph:
    """hipGraph of tree drafting (root top-k, then depths 2..D) for ``Rb`` sequences.

    The per-depth metadata depends only on each sequence's length and block
    table, never on what the draft proposes, so all depths' positions, KV
    slots and context lengths are built on the host in one buffer and copied
    once; the graph then runs every depth (ancestor masks, draft layer over
    the chunk of tree nodes, top-k expansion, beam selection) without a host
    round trip.  Inputs: root hidden states and last tokens; outputs: tree
    tokens and parents.  Padding rows use the scratch page 0."""

    def __init__(self, eng: "SpecEngine", Rb: int, depth: int):
        sp, run = eng.spec, eng.runner
        self.eng, self.Rb, self.maxw = eng, Rb, run.max_blocks
        self.W, self.D, self.K, self.N = sp.width, depth, sp.topk, sp.nodes(depth)
        dev = eng.device
        H = eng.model_cfg.hidden_size
        self.ms = [self.W * (d - 1) for d in range(2, self.D + 1)]
        self.depth_np = np.concatenate([[0]] + [[d] * self.W for d in range(1, self.D + 1)]).astype(np.int64)
        n_dyn = Rb * self.maxw + sum(2 * Rb * m + Rb for m in self.ms)
        self.host = torch.zeros(n_dyn, dtype=torch.int32).pin_memory()
        self.dyn = torch.zeros(n_dyn, dtype=torch.int32, device=dev)
        o = 0
        self.d_bt = self.dyn[o:o + Rb * self.maxw].view(Rb, self.maxw)
        o += Rb * self.maxw
        self.lv = []                     # per depth: (offset, m, pos, slots, ctx, cu, tiles)
        tiles = torch.stack([torch.arange(Rb, dtype=torch.int32), torch.zeros(Rb, dtype=torch.int32)],
                            1).contiguous().to(dev)
        for m in self.ms:
            pos = self.dyn[o:o + Rb * m]
            slots = self.dyn[o + Rb * m:o + 2 * Rb * m]
            ctx = self.dyn[o + 2 * Rb * m:o + 2 * Rb * m + Rb]
            cu = torch.arange(0, Rb * m + 1, m, dtype=torch.int32, device=dev)
            self.lv.append((o, m, pos, slots, ctx, cu, tiles))
            o += 2 * Rb * m + Rb
        self.g_root = torch.zeros(Rb, H, dtype=eng.cfg.dtype, device=dev)
        self.last = torch.zeros(Rb, dtype=torch.long, device=dev)
        self._fill(np.ones(Rb, np.int64), [[0]] * Rb)
        self.dyn.copy_(self.host)
        self._capture()

    def _fill(self, n_vec, brows) -> None:
        """Host metadata of every depth for sequences of length ``n_vec``."""
        Rb, maxw, bs = self.Rb, self.maxw, self.eng.pool.block_size
        h = self.host.numpy()
        h[:Rb * maxw] = 0
        for i, blk in enumerate(brows):
            h[i * maxw: i * maxw + len(blk)] = blk
        for o, m, *_ in self.lv:
            ps = np.empty((Rb, m), np.int64)
            sl = np.empty((Rb, m), np.int64)
            for i in range(Rb):
                n = int(n_vec[i]) if i < len(n_vec) else 1
                blk = np.asarray(brows[i] if i < len(brows) else [0], np.int64)
                ps[i] = n - 1 + self.depth_np[1:m + 1]
                s_ = n + np.arange(m)
                sl[i] = blk[np.minimum(s_ // bs, len(blk) - 1)] * bs + s_ % bs
                if i >= len(brows):
                    sl[i] = np.arange(m) % bs             # padding: scratch page 0
            h[o:o + Rb * m] = ps.ravel()
            h[o + Rb * m:o + 2 * Rb * m] = sl.ravel()
            h[o + 2 * Rb * m:o + 2 * Rb * m + Rb] = [int(n_vec[i]) + m if i < len(n_vec) else 1 + m
                                                     for i in range(Rb)]

    def _body(self):
        return _draft_tree(self.eng.draft, self.g_root, self.last, self.lv, self.d_bt, self.W, self.D, self.K, self.N)

    @torch.inference_mode()
    def _capture(self) -> None:
        eng = self.eng
        from dgi.utils.streams import named_stream
        s = named_stream("capture", eng.device)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._body()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize(eng.device)
        self.graph = torch.cuda.CUDAGraph()
        with graph_capture(self.graph, pool=eng._graph_pool):
            self.out = self._body()

    def run(self, R: int, g_root: torch.Tensor, last: list, n_vec, brows):
        self._fill(n_vec, brows)
        self.dyn.copy_(self.host, non_blocking=True)
        self.g_root[:R].copy_(g_root)
        self.last[:R].copy_(torch.as_tensor(last, dtype=torch.long).pin_memory(), non_blocking=True)
        self.graph.replay()
        tok, par = self.out
        return tok[:R], par[:R]


class _StepGraph:
    """hipGraph of a WHOLE speculative step for ``Rb`` sequences at tree depth ``D`` (SURVEY §3.6,
    VERDICT r5 #5; the reference loop it replaces: worker/engines/speculative.py:305-365):

        draft catch-up over the last step's accepted tokens (D + 1 rows per sequence, the
        rows past each sequence's count are padding on the scratch page)
        -> tree drafting (root top-k, depths 2..D)
        -> target verify over the N tree nodes (tree-masked attention, EAGLE-3 feature tap,
           coupled sampling) -> ``tree_verify`` (accept length, path, tokens)
        -> KV compaction of the accepted path (slot moves computed on device from the path
           and the block table; rejected moves copy scratch-page slots onto themselves)
        -> the accepted nodes' features, gathered for the next catch-up.

    One int32 metadata buffer (block tables + the catch-up, per-depth and verify positions /
    slots / context lengths, all derivable from each sequence's length) goes up per step and
    only the accept lengths and tokens come back: one host round trip per step, no eager
    launches.  Padding rows of a partial bucket live on the scratch page 0."""

    def __init__(self, eng: "SpecEngine", Rb: int, depth: int):
        sp, run = eng.spec, eng.runner
        self.eng, self.Rb, self.D = eng, Rb, depth
        self.W, self.K, self.N = sp.width, sp.topk, sp.nodes(depth)
        self.C = depth + 1
        self.maxw = run.max_blocks
        dev = eng.device
        H = eng.model_cfg.hidden_size
        W, D, N, C = self.W, self.D, self.N, self.C
        self.ms = [W * (d - 1) for d in range(2, D + 1)]
        self.depth_np = np.concatenate([[0]] + [[d] * W for d in range(1, D + 1)]).astype(np.int64)
        # int32 metadata: bt | catch-up pos, slots, ctx, last index | per depth pos, slots, ctx | verify pos, slots, ctx
        n_dyn = Rb * self.maxw + (2 * Rb * C + 2 * Rb) + sum(2 * Rb * m + Rb for m in self.ms) + (2 * Rb * N + Rb)
        self.host = torch.zeros(n_dyn, dtype=torch.int32).pin_memory()
        self.dyn = torch.zeros(n_dyn, dtype=torch.int32, device=dev)
        o = 0

        def take(n):
            nonlocal o
            v = self.dyn[o:o + n]
            o += n
            return v
        self.o_bt = o
        self.d_bt = take(Rb * self.maxw).view(Rb, self.maxw)
        self.o_c = o
        self.c_pos, self.c_slots, self.c_ctx, self.c_last = take(Rb * C), take(Rb * C), take(Rb), take(Rb)
        ar = torch.arange(Rb, dtype=torch.int32)
        self.c_cu = torch.arange(0, Rb * C + 1, C, dtype=torch.int32, device=dev)
        self.c_tiles = torch.stack([ar, torch.zeros(Rb, dtype=torch.int32)], 1).contiguous().to(dev)
        tiles = self.c_tiles
        self.lv = []
        for m in self.ms:
            off = o
            pos, slots, ctx = take(Rb * m), take(Rb * m), take(Rb)
            cu = torch.arange(0, Rb * m + 1, m, dtype=torch.int32, device=dev)
            self.lv.append((off, m, pos, slots, ctx, cu, tiles))
        self.o_v = o
        self.v_pos, self.v_slots, self.v_ctx = take(Rb * N), take(Rb * N), take(Rb)
        self.v_cu = torch.arange(0, Rb * N + 1, N, dtype=torch.int32, device=dev)
        # other static inputs
        self.c_ids = torch.zeros(Rb, C, dtype=torch.long, device=dev)
        self.c_feat = torch.zeros(Rb, C, H, dtype=eng.cfg.dtype, device=dev)
        self.temps = torch.zeros(Rb * N, dtype=torch.float32, device=dev)
        self.seeds = torch.zeros(Rb * N, dtype=torch.long, device=dev)
        self.topk = torch.zeros(Rb * N, dtype=torch.long, device=dev)
        self.topp = torch.ones(Rb * N, dtype=torch.float32, device=dev)
        self.greedy = True               # the sampling buffers hold temperature 0 everywhere
        self._fill([], [], [], [])
        self.dyn.copy_(self.host)
        self.graph = None
        self._capture()

    # ---------------------------------------------------------------- metadata
    def _fill(self, n_vec, p0_vec, brows, nv_vec) -> None:
        """Host metadata of sequences with committed length n, first catch-up position p0 and
        nv valid catch-up rows; rows past the live batch are padding on page 0."""
        Rb, C, N, maxw = self.Rb, self.C, self.N, self.maxw
        bs = self.eng.pool.block_size
        R = len(n_vec)
        h = self.host.numpy()
        bt = h[self.o_bt:self.o_bt + Rb * maxw].reshape(Rb, maxw)
        bt[:] = 0
        for i, blk in enumerate(brows):
            bt[i, :len(blk)] = blk

        live = np.arange(R)[:, None]
        n_l = np.asarray(n_vec[:R], dtype=np.int64)[:, None]

        def slots(P):                                      # slots of live rows' positions P [R, k]
            return bt[live, P // bs].astype(np.int64) * bs + P % bs
        # catch-up: rows p0 .. p0 + C - 1 (valid: the first nv), context p0 + C; padding rows
        # (past nv, or past the live batch) write scratch slots on page 0
        o = self.o_c
        cpos = h[o:o + Rb * C].reshape(Rb, C)
        cslot = h[o + Rb * C:o + 2 * Rb * C].reshape(Rb, C)
        cctx = h[o + 2 * Rb * C:o + 2 * Rb * C + Rb]
        clast = h[o + 2 * Rb * C + Rb:o + 2 * Rb * C + 2 * Rb]
        kk = np.arange(C)
        p0 = np.zeros(Rb, dtype=np.int64)
        nv = np.ones(Rb, dtype=np.int64)
        p0[:R] = np.asarray(p0_vec[:R], dtype=np.int64)
        nv[:R] = np.asarray(nv_vec[:R], dtype=np.int64)
        cpos[:] = p0[:, None] + kk
        cslot[:] = kk % bs
        if R:
            cslot[:R] = np.where(kk < nv[:R, None], slots(cpos[:R].astype(np.int64)), kk % bs)
        cctx[:] = p0 + C
        clast[:] = nv - 1
        # draft depths 2..D: chunk nodes at positions n - 1 + depth, slots n .. n + m - 1
        for off, m, *_ in self.lv:
            dp = h[off:off + Rb * m].reshape(Rb, m)
            dsl = h[off + Rb * m:off + 2 * Rb * m].reshape(Rb, m)
            dctx = h[off + 2 * Rb * m:off + 2 * Rb * m + Rb]
            n = np.ones(Rb, dtype=np.int64)
            n[:R] = n_l[:, 0]
            dp[:] = n[:, None] - 1 + self.depth_np[1:m + 1]
            dsl[:] = np.arange(m) % bs
            if R:
                dsl[:R] = slots(n_l + np.arange(m))
            dctx[:] = n + m
        # verify: node k at position n - 1 + depth(k), slot n - 1 + k, context n - 1 + N
        o = self.o_v
        vp = h[o:o + Rb * N].reshape(Rb, N)
        vsl = h[o + Rb * N:o + 2 * Rb * N].reshape(Rb, N)
        vctx = h[o + 2 * Rb * N:o + 2 * Rb * N + Rb]
        vp[:] = np.arange(N)
        vsl[:] = np.arange(N) % bs
        vctx[:] = N
        if R:
            vp[:R] = n_l - 1 + self.depth_np
            vsl[:R] = slots(n_l - 1 + np.arange(N))
            vctx[:R] = n_l[:, 0] - 1 + N

    # ---------------------------------------------------------------- the step
    def _body(self):
        eng, dr = self.eng, self.eng.draft
        Rb, C, D, N, W = self.Rb, self.C, self.D, self.N, self.W
        H = self.c_feat.shape[2]
        bs = eng.pool.block_size
        # 1) draft catch-up
        cm = AttnMeta(positions=self.c_pos, slot_mapping=self.c_slots, num_decode=0, num_prefill_tokens=Rb * C,
                      pre_block_tables=self.d_bt, pre_cu_seqlens=self.c_cu, pre_context_lens=self.c_ctx,
                      pre_tiles=self.c_tiles)
        g = dr.forward(self.c_ids.view(-1), self.c_feat.view(Rb * C, H), cm).view(Rb, C, H)
        li = self.c_last.long()
        g_root = torch.gather(g, 1, li[:, None, None].expand(Rb, 1, H)).squeeze(1)
        last = torch.gather(self.c_ids, 1, li[:, None]).squeeze(1)
        # 2) tree drafting
        tok, par = _draft_tree(dr, g_root, last, self.lv, self.d_bt, W, D, self.K, N)
        # 3) verify
        anc, depth = ops.tree_mask(par)
        tiles = self.c_tiles
        vm = AttnMeta(positions=self.v_pos, slot_mapping=self.v_slots, num_decode=0, num_prefill_tokens=Rb * N,
                      pre_block_tables=self.d_bt, pre_cu_seqlens=self.v_cu, pre_context_lens=self.v_ctx,
                      pre_tiles=tiles, tree_mask=anc, tree_n=N)
        logits, feats = eng._forward_capture(vm, tok.view(-1))
        tgt = ops.sample(logits, self.temps, self.seeds, 0, top_k=self.topk, top_p=self.topp).view(Rb, N)
        acc, path, toks = ops.tree_verify(par, tok, tgt, anc, depth, D + 1)
        # 4) compaction: accepted node path[k] (k = 1..acc) moves to position base + k
        base = self.v_pos.view(Rb, N)[:, :1].long()                  # n - 1 (node 0's position)
        kk = torch.arange(1, D + 1, device=tok.device)
        ps = base + path[:, 1:D + 1].long()
        pd = base + kk[None]
        bt = self.d_bt.long()
        slot = lambda p: torch.gather(bt, 1, (p // bs).clamp(0, bt.shape[1] - 1)) * bs + p % bs  # noqa: E731
        src, dst = slot(ps), slot(pd)
        move = (kk[None] <= acc[:, None].long()) & (src != dst)
        scratch = (kk % bs)[None].expand(Rb, D)
        src = torch.where(move, src, scratch)
        dst = torch.where(move, dst, scratch)
        kv_slot_copy(eng.model.kv_cache, src.reshape(-1), dst.reshape(-1), bs)
        # 5) the accepted nodes' features (positions n - 1 .. n - 1 + acc) for the next catch-up
        fidx = path[:, :D + 1].long().clamp(min=0)
        fkeep = torch.gather(feats.view(Rb, N, H), 1, fidx[:, :, None].expand(Rb, D + 1, H))
        return acc, toks, fkeep

    @torch.inference_mode()
    def _capture(self) -> None:
        eng = self.eng
        eng.model.kv_cache = eng.pool.kv
        from dgi.utils.streams import named_stream
        s = named_stream("capture", eng.device)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._body()                                   # warm-up (lazy inits outside capture)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize(eng.device)
        self.graph = torch.cuda.CUDAGraph()
        with graph_capture(self.graph, pool=eng._graph_pool):
            self.out = self._body()

    def run(self, n_vec, p0_vec, brows, nv_vec, ids, feats, samp) -> tuple:
        """Replay for R live sequences: ``ids`` [R][<= C] catch-up tokens, ``feats`` R feature
        tensors [nv, H], ``samp`` (temps, seeds, top-k, top-p) host arrays [R, N] or None (all
        greedy).  Returns device (acc [R], tokens [R, D + 1], kept features [R, D + 1, H])."""
        R, C, N = len(n_vec), self.C, self.N
        self._fill(n_vec, p0_vec, brows, nv_vec)
        self.dyn.copy_(self.host, non_blocking=True)
        ids_h = np.zeros((self.Rb, C), np.int64)
        for i, t in enumerate(ids):
            ids_h[i, :len(t)] = t
        self.c_ids.copy_(torch.from_numpy(ids_h).pin_memory(), non_blocking=True)
        for i, f in enumerate(feats):
            self.c_feat[i, :f.shape[0]].copy_(f)
        if samp is None:
            if not self.greedy:
                self.temps.zero_()
                self.greedy = True
        else:
            n = R * N
            for buf, x in zip((self.temps, self.seeds, self.topk, self.topp), samp):
                buf[:n].copy_(torch.from_numpy(np.ascontiguousarray(x).ravel()).pin_memory(), non_blocking=True)
            self.temps[n:].zero_()
            self.greedy = False
        self.graph.replay()
        acc, toks, fkeep = self.out
        return acc[:R], toks[:R], fkeep[:R]


def _token_range(r, a: int, b: int) -> list:
    """``r.all_tokens()[a:b]`` without building the whole prompt + output list (a catch-up
    window is a few tokens at the end of a possibly long context)."""
    P = len(r.prompt)
    if a >= P:
        return r.output[a - P:b - P]
    return r.prompt[a:b] + (r.output[:b - P] if b > P else [])


class SpecEngine(LLMEngine):
    """``LLMEngine`` with EAGLE-3 tree speculation (greedy and sampled requests)."""

    def __init__(self, cfg: EngineConfig, spec: Optional[SpecConfig] = None, model_cfg: Optional[ModelConfig] = None,
                 model=None, draft: Optional[Eagle3Draft] = None):
        super().__init__(cfg, model_cfg, model)
        self.spec = spec or SpecConfig()
        self.spec.validate()
        L = self.model_cfg.num_layers
        self.feature_layers = tuple(self.spec.feature_layers or default_feature_layers(L))
        self.draft = draft or Eagle3Draft(self.model, self.pool.num_blocks, self.pool.block_size)
        self.spec_stats = {"spec_steps": 0, "spec_rows": 0, "accepted": 0, "spec_tokens": 0, "draft_s": 0.0,
                           "verify_s": 0.0, "plain_steps": 0, "switches_off": 0, "depth_changes": 0}
        # measurement aid: rid -> known greedy continuation; the depth-d node of
        # the first chain is replaced by it (kept with probability oracle_accept)
        self.oracle: Optional[dict] = None
        self.oracle_accept = 1.0
        self._oracle_rng = np.random.default_rng(0)
        self._vgraphs: dict = {}
        self._dgraphs: dict = {}
        self._sgraphs: dict = {}    # (bucket, depth) -> _StepGraph (whole speculative step)
        self.whole_step = True      # speculative steps as one captured graph where eligible
        self._graphs_vocab = self.draft.vocab_version
        self._graph_pool = torch.cuda.graph_pool_handle() if self.device.type == "cuda" else None
        # plain decode steps replay the engine's hipGraphs with the EAGLE-3 feature tap on
        if self.runner.graphs is not None:
            self.runner.graphs.features = (self.feature_layers, self.draft.fuse)
        # adaptive depth + auto-off controller
        self.cur_depth = self.spec.depth
        self.spec_on = True
        self._mode_steps = 0
        self._probe = False
        self._cost: dict = {}       # (mode, bucket) -> seconds per generated token (spec: EMA, plain: recent min)
        self._plain_win: dict = {}  # (plain, bucket) -> last 16 plain cost samples
        # step-time accounting by mode (seconds, steps): plain steps right after a speculative
        # step vs after a plain one, and speculative steps
        self.step_times = {"after_spec": [0.0, 0], "after_plain": [0.0, 0], "spec": [0.0, 0]}
        self._last_mode = None
        self._acc_ema: Optional[float] = None   # smoothed acceptance rate driving depth changes
        self._acc_n = 0                          # steps behind it (at the current depth)
        self._period = [0.0, 0, 0]               # clean spec samples this period: seconds, tokens, steps
        self._period_acc = [0, 0]                # accepted drafts, rows speculated this period
        self._backoff = 1                        # probe interval multiplier
        self._probed = False                     # the current speculation period is a re-probe
        self._captured = False      # this step captured a hipGraph (its time is not a cost sample)
        self.force_plain = False    # measurement aid: plain decode steps only (feature tap still on)

    def _bucket(self, R: int) -> int:
        return next((b for b in VERIFY_BUCKETS if b >= R), VERIFY_BUCKETS[-1])

    def _check_graph_vocab(self) -> None:
        """Drop the draft / verify graphs captured against an older draft vocabulary (they hold
        pointers to the replaced ``hot`` / ``hot_head`` tensors)."""
        if self._graphs_vocab != self.draft.vocab_version:
            self._dgraphs.clear()
            self._vgraphs.clear()
            self._sgraphs.clear()
            self._graphs_vocab = self.draft.vocab_version

    def _draft_graph(self, R: int) -> Optional[_DraftGraph]:
        if not (self.spec.graphs and self.device.type == "cuda" and self.cur_depth >= 2):
            return None
        self._check_graph_vocab()
        Rb = next((b for b in VERIFY_BUCKETS if b >= R), None)
        if Rb is None:
            return None
        g = self._dgraphs.get((Rb, self.cur_depth))
        if g is None:
            g = self._dgraphs[(Rb, self.cur_depth)] = _DraftGraph(self, Rb, self.cur_depth)
            self._captured = True
        return g

    def _verify_graph(self, R: int) -> Optional[_VerifyGraph]:
        if not (self.spec.graphs and self.device.type == "cuda"):
            return None
        self._check_graph_vocab()
        Rb = next((b for b in VERIFY_BUCKETS if b >= R), None)
        if Rb is None:
            return None
        g = self._vgraphs.get((Rb, self.cur_depth))
        if g is None:
            g = self._vgraphs[(Rb, self.cur_depth)] = _VerifyGraph(self, Rb, self.cur_depth)
            self._captured = True
        return g

    def _step_graph(self, R: int) -> Optional[_StepGraph]:
        if not (self.whole_step and self.spec.graphs and self.device.type == "cuda" and self.cur_depth >= 2
                and not self.oracle):
            return None
        self._check_graph_vocab()
        Rb = next((b for b in VERIFY_BUCKETS if b >= R), None)
        if Rb is None:
            return None
        g = self._sgraphs.get((Rb, self.cur_depth))
        if g is None:
            g = self._sgraphs[(Rb, self.cur_depth)] = _StepGraph(self, Rb, self.cur_depth)
            self._captured = True
        return g

    def warmup_spec(self, batches=(1,), depths=None) -> int:
        """Capture the draft / verify hipGraphs of every (batch bucket, depth) the
        adaptive controller can reach, so no capture lands in a serving step (a
        capture inside a timed step also corrupts the auto-off cost estimate)."""
        if not (self.spec.graphs and self.device.type == "cuda"):
            return 0
        keep, n = self.cur_depth, 0
        try:
            for R in batches:
                for d in (depths or range(1, self.spec.depth + 1)):
                    self.cur_depth = d
                    n += int(self._verify_graph(R) is not None) + int(self._draft_graph(R) is not None)
                    n += int(self._step_graph(R) is not None)
        finally:
            self.cur_depth = keep
            self._captured = False
        return n

    def reset_controller(self, keep_plain_costs: bool = False) -> None:
        """Back to full depth, speculation on, no acceptance history.  Plain-decode
        cost per bucket is a property of the hardware, not of the workload:
        ``keep_plain_costs`` keeps it so a new workload needs no plain probe."""
        self.cur_depth, self.spec_on = self.spec.depth, True
        self._mode_steps, self._probe, self._probed, self._backoff = 0, False, False, 1
        self._period = [0.0, 0, 0]
        self._period_acc = [0, 0]
        self._cost = {k: v for k, v in self._cost.items() if keep_plain_costs and k[0] == "plain"}
        if not keep_plain_costs:
            self._plain_win = {}
        self._acc_ema, self._acc_n = None, 0

    # ------------------------------------------------------------------ helpers
    def _eligible(self, r: Request) -> bool:
        return not r.in_prefill and not r.busy

    def _state(self, r: Request) -> _SpecState:
        if r.spec_state is None:
            r.spec_state = _SpecState(r.num_cached)
        return r.spec_state

    def _forward_capture(self, meta: AttnMeta, ids: torch.Tensor, fuse: bool = True):
        """Target forward that also returns the EAGLE-3 features of every row
        (fused [T, H], or the raw low|mid|high concatenation [T, 3H])."""
        m = self.model
        m.capture_layers, m.captured = self.feature_layers, {}
        try:
            logits = m.forward(meta, input_ids=ids)
            raw = torch.cat([m.captured[li] for li in self.feature_layers], dim=-1)
        finally:
            m.capture_layers, m.captured = (), {}
        return logits, (self.draft.fuse(raw) if fuse else raw)

    def _append_feats(self, r: Request, start: int, feats: torch.Tensor) -> None:
        """Record target features of positions [start, start + len(feats)).  ``feats``
        must not alias a buffer that is rewritten later (callers clone once per step)."""
        st = self._state(r)
        if st.rows() == 0 or st.feat_start + st.rows() != start:
            st.feat, st.feat_start = feats, start
        else:
            st.chunks.append(feats)
            st.n_chunked += feats.shape[0]

    # ------------------------------------------------------------------ controller
    def _record(self, mode: str, R: int, seconds: float, tokens: int) -> None:
        if tokens <= 0:
            return
        key = (mode, self._bucket(R))
        c = seconds / tokens
        if mode == "plain":
            # plain decode cost at a bucket is a hardware property: keep the fastest of the
            # recent samples (a one-off stall — a lazily captured graph, a pipeline tail — must
            # not make speculation look cheaper than it is)
            win = self._plain_win.setdefault(key, [])
            win.append(c)
            del win[:-16]
            self._cost[key] = min(win)
        else:
            old = self._cost.get(key)
            self._cost[key] = c if old is None else 0.7 * old + 0.3 * c
        if mode == "spec":           # this speculation period's own cost (acceptance changes between probes)
            self._period[0] += seconds
            self._period[1] += tokens
            self._period[2] += 1

    def _adapt_depth(self, accept_rate: float) -> None:
        """Reference thresholds (worker/engines/speculative.py:456-463), applied to
        an EMA of the per-step rate (the reference reacts to single steps, which
        makes the depth — and with graphs, the captured graph — flip-flop); the
        EMA restarts at every depth change since the rate depends on the depth."""
        if not self.spec.adaptive_depth:
            return
        e = accept_rate if self._acc_ema is None else 0.6 * self._acc_ema + 0.4 * accept_rate
        self._acc_ema = e
        self._acc_n += 1
        if self._acc_n < 2:
            return
        d = self.cur_depth
        if e < self.spec.min_accept_rate:
            d = max(1, d - 1)
        elif e > self.spec.raise_accept_rate:
            d = min(self.spec.depth, d + 1)
        if d != self.cur_depth:
            self.cur_depth = d
            self._acc_ema, self._acc_n = None, 0
            self.spec_stats["depth_changes"] += 1

    def _control(self, R: int) -> None:
        """Auto-off: compare this speculation period's measured cost per generated
        token with plain decoding's at the same batch bucket.  Two clean samples
        decide; a first period without a plain reference probes 3 plain steps.
        Slower than plain: first step the tree one level shallower (adaptive
        depth), and only at depth 1 fall back to plain decoding.
        Probes that keep losing back off exponentially (probe_every x 1, 2, 4, 8
        plain steps), a winning probe resets the interval."""
        if not self.spec.auto_off or R == 0:
            return
        self._mode_steps += 1
        cp = self._cost.get(("plain", self._bucket(R)))
        if self.spec_on:
            secs, toks, n = self._period
            if n < 2:
                return               # fewer than 2 clean samples (graph-capture steps are not samples)
            if cp is None:
                self.spec_on, self._mode_steps, self._probe = False, 0, True
            elif secs / toks > cp * (1.0 - self.spec.min_gain) and self.spec.adaptive_depth and self.cur_depth > 1:
                # slower than plain at this depth: a shallower tree costs less per step and
                # wastes fewer rejected nodes — try it before giving up on speculation; jump
                # straight to one level past the accepted length this period measured
                acc_len = self._period_acc[0] / max(1, self._period_acc[1])
                self.cur_depth = max(1, min(self.cur_depth - 1, int(math.ceil(acc_len)) + 1))
                self._acc_ema, self._acc_n = None, 0
                self.spec_stats["depth_changes"] += 1
            elif secs / toks > cp * (1.0 - self.spec.min_gain):
                self.spec_on, self._mode_steps, self._probe = False, 0, False
                self.spec_stats["switches_off"] += 1
                if self._probed:
                    self._backoff = min(8, self._backoff * 2)
            else:
                self._backoff = 1
                self._period = [0.0, 0, 0]     # keep speculating; judge the next window afresh
                self._period_acc = [0, 0]
                return
            self._period = [0.0, 0, 0]
            self._period_acc = [0, 0]
        else:
            wait = 3 if self._probe else self.spec.probe_every * self._backoff
            if self._mode_steps >= wait:
                self._probed = not self._probe
                self.spec_on, self._mode_steps, self._probe = True, 0, False

    # ------------------------------------------------------------------ step
    def step(self) -> list:
        t0 = time.perf_counter()
        self.model.kv_cache = self.pool.kv
        outs: list[StepOutput] = []
        spec_reqs = [r for r in self.scheduler.running if self._eligible(r)] \
            if self.spec_on and not self.force_plain else []
        for r in spec_reqs:
            r.busy = True            # keep them out of the normal batch
        try:
            sb = self.scheduler.schedule()
        finally:
            for r in spec_reqs:
                r.busy = False
        if not sb.empty:
            o = self._normal_step(sb)
            outs += o
            if not sb.prefill and not spec_reqs:
                # cost samples are whole steps (scheduling and host work included) in both
                # modes, so neither mode's per-step overhead falls outside its timer
                dt = time.perf_counter() - t0
                self._record("plain", len(sb.decode), dt, len(o))
                k = "after_spec" if self._last_mode == "spec" else "after_plain"
                self.step_times[k][0] += dt
                self.step_times[k][1] += 1
                self._last_mode = "plain"
                self.spec_stats["plain_steps"] += 1
                self._control(len(sb.decode))
        live = [r for r in spec_reqs if r in self.scheduler.running and self._eligible(r)]
        if live:
            self._captured = False
            o = self._spec_step(live)
            outs += o
            if sb.empty and not self._captured:
                dt = time.perf_counter() - t0
                self._record("spec", len(live), dt, len(o))
                self.step_times["spec"][0] += dt
                self.step_times["spec"][1] += 1
            self._last_mode = "spec"
            self._control(len(live))
        self.stats["step_time"] += time.perf_counter() - t0
        return outs

    @torch.inference_mode()
    def _normal_step(self, sb) -> list:
        run = self.runner
        run.step_id += 1
        g = run.graphs
        if g is not None and not sb.prefill and sb.decode and len(sb.decode) <= g.max_bucket:
            # plain decode: hipGraph replay with the feature tap
            pos = [r.num_computed for r in sb.decode]
            toks = g.run(sb)
            feats = g.last_features(len(sb.decode)).clone()     # one copy per step; rows are views of it
            for i, r in enumerate(sb.decode):
                self._append_feats(r, pos[i], feats[i: i + 1])
            return self._apply(sb, list(sb.decode), toks)
        flat, hdr, sampled = run.build_host(sb)
        ids, meta, samp = run.meta_from_device(run.to_device(flat), hdr)
        logits, feats = self._forward_capture(meta, ids)
        nd = len(sb.decode)
        for i, r in enumerate(sb.decode):
            self._append_feats(r, r.num_computed, feats[i: i + 1])
        row = nd
        for c in sb.prefill:
            self._append_feats(c.req, c.start, feats[row: row + c.length])
            row += c.length
        if not sampled:
            return self._apply(sb, [], [])
        return self._apply(sb, sampled, samp.sample(logits).tolist())

    def _node_sampling(self, reqs: list, depth_np: np.ndarray):
        """Per tree node (row-major [R, N]) temperature / seed / top-k / top-p of the
        coupled verification: node of depth d samples output index len(output) + d
        with the seed plain decoding uses for that index."""
        R, N = len(reqs), len(depth_np)
        temps = np.empty((R, N), np.float32)
        seeds = np.empty((R, N), np.int64)
        topk = np.zeros((R, N), np.int64)
        topp = np.ones((R, N), np.float32)
        for i, r in enumerate(reqs):
            p = r.params
            temps[i] = p.temperature
            seeds[i] = (r.seed * 1000003 + len(r.output) + depth_np) & 0x7FFFFFFF
            if p.needs_filter:
                topk[i] = max(0, p.top_k)
                topp[i] = p.top_p
        out = [torch.from_numpy(x.ravel()) for x in (temps, seeds, topk, topp)]
        if self.device.type == "cuda":
            out = [x.pin_memory().to(self.device, non_blocking=True) for x in out]
        return out

    @torch.inference_mode()
    def _spec_step(self, reqs: list) -> list:
        sp = self.spec
        D = self.cur_depth
        W, K, N = sp.width, sp.topk, sp.nodes(D)
        bs = self.pool.block_size
        dev = self.device
        run = self.runner
        run.gate_rows(reqs)           # host KV tier restores (swap-ins, prefix pages) land first
        sched = self.scheduler
        # ---- blocks for the tree slots [n-1, n-1+N)
        ok = []
        for r in reqs:
            try:
                sched._grow(r, r.total_len - 1 + N)
                ok.append(r)
            except OutOfBlocks:
                pass
        reqs = ok
        if not reqs:
            return []
        R = len(reqs)
        outs = self._whole_step(reqs)
        if outs is not None:
            return outs
        td = time.perf_counter()
        # ---- 1) draft catch-up over committed positions [draft_len, n-1]
        pos, slots, cu, ctx, ids, feat_rows, brows = [], [], [0], [], [], [], []
        H = self.model_cfg.hidden_size
        for r in reqs:
            st = self._state(r)
            n = r.total_len
            toks = r.all_tokens()
            p0 = min(st.draft_len, n - 1)
            blk = np.asarray(r.blocks, np.int64)
            ps = np.arange(p0, n)
            pos.append(ps)
            slots.append(blk[ps // bs] * bs + ps % bs)
            ids.extend(toks[p0:n])
            cu.append(cu[-1] + len(ps))
            ctx.append(n)
            brows.append(r.blocks)
            feat_rows.append(self._feature_rows(st, p0 - 1, n - 1, H))
        meta = _varlen_meta(run, np.concatenate(pos), np.concatenate(slots), brows, cu, ctx, dev)
        d_ids = torch.tensor(ids, dtype=torch.long).pin_memory().to(dev, non_blocking=True) \
            if dev.type == "cuda" else torch.tensor(ids, dtype=torch.long)
        g = self.draft.forward(d_ids, torch.cat(feat_rows), meta)
        last = torch.tensor(cu[1:], device=dev) - 1
        g_root = g.index_select(0, last)                         # [R, H]
        for r in reqs:
            r.spec_state.draft_len = r.total_len
        # ---- 2) tree drafting
        n_vec = np.asarray([r.total_len for r in reqs], np.int64)
        depth_np = np.concatenate([[0]] + [[d] * W for d in range(1, D + 1)]).astype(np.int64)
        dg = self._draft_graph(R)
        if dg is not None:
            tok, par = dg.run(R, g_root, [r.all_tokens()[-1] for r in reqs], n_vec, brows)
        else:
            tok, par = self._draft_tree_eager(reqs, g_root, n_vec, depth_np, brows, D)
        if self.oracle:
            self._apply_oracle(reqs, tok, par, n_vec, D)
        self.spec_stats["draft_s"] += time.perf_counter() - td
        tv = time.perf_counter()
        # ---- 3) target verify over all N tree nodes (coupled sampling, greedy = temperature 0)
        samp = self._node_sampling(reqs, depth_np)
        vpos, vslots, vctx, vcu = [], [], [], [0]
        for i, r in enumerate(reqs):
            n = int(n_vec[i])
            blk = np.asarray(r.blocks, np.int64)
            vpos.append(n - 1 + depth_np)
            sl = n - 1 + np.arange(N)
            vslots.append(blk[sl // bs] * bs + sl % bs)
            vctx.append(n - 1 + N)
            vcu.append(vcu[-1] + N)
        vpos, vslots = np.concatenate(vpos), np.concatenate(vslots)
        vg = self._verify_graph(R)
        if vg is not None:
            acc, path, toks, feats = vg.run(R, tok, par, vpos, vslots, brows, vctx, samp)
        else:
            anc, depth = ops.tree_mask(par)
            vm = _varlen_meta(run, vpos, vslots, brows, vcu, vctx, dev, tree_mask=anc, tree_n=N)
            logits, feats = self._forward_capture(vm, tok.view(-1))
            tgt = ops.sample(logits, samp[0], samp[1], 0, top_k=samp[2], top_p=samp[3]).view(R, N)
            acc, path, toks = ops.tree_verify(par, tok, tgt, anc, depth, D + 1)
        if dev.type == "cuda":
            # one wait for the three verify outputs (three .cpu() calls were three round trips)
            hs = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in (acc, path, toks)]
            for h_, t in zip(hs, (acc, path, toks)):
                h_.copy_(t, non_blocking=True)
            torch.cuda.current_stream(dev).synchronize()
            acc_h, path_h, toks_h = hs[0].tolist(), hs[1].numpy(), hs[2].numpy()
        else:
            acc_h = acc.cpu().tolist()
            path_h = path.cpu().numpy()
            toks_h = toks.cpu().numpy()
        # ---- 4) compact accepted KV, keep their features, commit tokens
        src, dst = [], []
        fsel = []
        for i, r in enumerate(reqs):
            n = int(n_vec[i])
            a = acc_h[i]
            blk = np.asarray(r.blocks, np.int64)
            for k in range(1, a + 1):
                s_, d_ = n - 1 + int(path_h[i, k]), n - 1 + k
                if s_ != d_:
                    src.append(int(blk[s_ // bs] * bs + s_ % bs))
                    dst.append(int(blk[d_ // bs] * bs + d_ % bs))
            fsel.extend((i * N + path_h[i, : a + 1]).tolist())
        if src:
            kv_slot_copy(self.model.kv_cache, torch.tensor(src, device=dev), torch.tensor(dst, device=dev), bs)
        fkeep = feats.index_select(0, torch.tensor(fsel, device=dev))
        self.spec_stats["verify_s"] += time.perf_counter() - tv
        outs = []
        now = time.perf_counter()
        st_all = self.stats
        st_all["steps"] += 1
        o = 0
        for i, r in enumerate(reqs):
            n = int(n_vec[i])
            a = acc_h[i]
            st = r.spec_state
            st.feat, st.feat_start = fkeep[o: o + a + 1], n - 1
            o += a + 1
            r.num_computed = n + a
            st_all["decode_tokens"] += a + 1
            self.spec_stats["accepted"] += a
            for k in range(a + 1):
                t = int(toks_h[i, k])
                r.output.append(t)
                r.token_times.append(now)
                st_all["generated"] += 1
                self.spec_stats["spec_tokens"] += 1
                reason = self._check_stop(r, t)
                if reason is not None:
                    self.scheduler.finish(r, reason)
                    st_all["finished"] += 1
                    self.requests.pop(r.rid, None)
                outs.append(StepOutput(r.rid, t, reason is not None, reason, r))
                if reason is not None:
                    break
        self.spec_stats["spec_steps"] += 1
        self.spec_stats["spec_rows"] += R
        self._period_acc[0] += sum(acc_h)
        self._period_acc[1] += R
        self._adapt_depth(sum(acc_h) / (R * D))
        return outs

    def _whole_step(self, reqs: list) -> Optional[list]:
        """The speculative step as one captured graph (``_StepGraph``) when every sequence's
        draft catch-up fits its D + 1 rows and its features are at hand (the steady state of a
        speculating batch); None: the staged path runs it."""
        D = self.cur_depth
        C = D + 1
        if D < 2:
            return None
        rows = []
        for r in reqs:
            st = self._state(r)
            n = r.total_len
            p0 = min(st.draft_len, n - 1)
            nv = n - p0
            f = st.feat
            if p0 < 1 or nv > C or f is None or st.feat_start > p0 - 1 or p0 - 1 + nv > st.feat_start + f.shape[0]:
                return None
            rows.append((r, st, n, p0, nv, f[p0 - 1 - st.feat_start: p0 - 1 - st.feat_start + nv]))
        sg = self._step_graph(len(reqs))
        if sg is None:
            return None
        t0 = time.perf_counter()
        samp = None
        if any(r.params.temperature > 0 for r in reqs):
            samp = self._node_sampling_host(reqs, sg.depth_np)
        acc, toks, fkeep = sg.run([x[2] for x in rows], [x[3] for x in rows], [r.blocks for r in reqs],
                                  [x[4] for x in rows], [_token_range(r, x[3], x[2]) for x, r in zip(rows, reqs)],
                                  [x[5] for x in rows], samp)
        hs = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in (acc, toks)]
        for h_, t in zip(hs, (acc, toks)):
            h_.copy_(t, non_blocking=True)
        fk = fkeep.clone()                       # the graph's output buffer is rewritten next replay
        torch.cuda.current_stream(self.device).synchronize()
        acc_h, toks_h = hs[0].tolist(), hs[1].numpy()
        self.spec_stats["verify_s"] += time.perf_counter() - t0
        self.spec_stats["whole_steps"] = self.spec_stats.get("whole_steps", 0) + 1
        outs = []
        now = time.perf_counter()
        st_all = self.stats
        st_all["steps"] += 1
        for i, (r, st, n, p0, nv, _f) in enumerate(rows):
            a = acc_h[i]
            st.draft_len = n
            st.feat, st.feat_start = fk[i, :a + 1], n - 1
            r.num_computed = n + a
            st_all["decode_tokens"] += a + 1
            self.spec_stats["accepted"] += a
            for k in range(a + 1):
                t = int(toks_h[i, k])
                r.output.append(t)
                r.token_times.append(now)
                st_all["generated"] += 1
                self.spec_stats["spec_tokens"] += 1
                reason = self._check_stop(r, t)
                if reason is not None:
                    self.scheduler.finish(r, reason)
                    st_all["finished"] += 1
                    self.requests.pop(r.rid, None)
                outs.append(StepOutput(r.rid, t, reason is not None, reason, r))
                if reason is not None:
                    break
        R = len(rows)
        self.spec_stats["spec_steps"] += 1
        self.spec_stats["spec_rows"] += R
        self._period_acc[0] += sum(acc_h)
        self._period_acc[1] += R
        self._adapt_depth(sum(acc_h) / (R * D))
        return outs

    def _node_sampling_host(self, reqs: list, depth_np: np.ndarray) -> tuple:
        """``_node_sampling`` as host arrays [R, N] (the whole-step graph copies them into its
        static buffers)."""
        R, N = len(reqs), len(depth_np)
        temps = np.empty((R, N), np.float32)
        seeds = np.empty((R, N), np.int64)
        topk = np.zeros((R, N), np.int64)
        topp = np.ones((R, N), np.float32)
        for i, r in enumerate(reqs):
            p = r.params
            temps[i] = p.temperature
            seeds[i] = (r.seed * 1000003 + len(r.output) + depth_np) & 0x7FFFFFFF
            if p.needs_filter:
                topk[i] = max(0, p.top_k)
                topp[i] = p.top_p
        return temps, seeds, topk, topp

    def _feature_rows(self, st: _SpecState, q0: int, q1: int, H: int) -> torch.Tensor:
        """Fused target features of positions [q0, q1) (zeros where unknown)."""
        n = q1 - q0
        f = st.feat
        if f is not None and st.feat_start <= q0 and q1 <= st.feat_start + f.shape[0]:
            return f[q0 - st.feat_start: q1 - st.feat_start]
        out = torch.zeros(n, H, dtype=self.cfg.dtype, device=self.device)
        if f is not None:
            lo, hi = max(q0, st.feat_start), min(q1, st.feat_start + f.shape[0])
            if lo < hi:
                out[lo - q0: hi - q0] = f[lo - st.feat_start: hi - st.feat_start]
        return out

    def _draft_tree_eager(self, reqs, g_root, n_vec, depth_np, brows, D):
        """Tree drafting, one host-built metadata copy per depth (CPU / no graphs)."""
        W, K, N = self.spec.width, self.spec.topk, self.spec.nodes(D)
        R, H = g_root.shape
        dev, run, bs = self.device, self.runner, self.pool.block_size
        g = g_root
        v1, t1 = self.draft.topk(g_root, K)                      # log-probs over the draft vocabulary
        t1 = self.draft.to_token(t1)
        tok = torch.zeros(R, N, dtype=torch.long, device=dev)
        par = torch.full((R, N), -1, dtype=torch.int32, device=dev)
        score = torch.zeros(R, N, dtype=torch.float32, device=dev)
        G = torch.zeros(R, N, H, dtype=g.dtype, device=dev)
        tok[:, 0] = torch.tensor([r.all_tokens()[-1] for r in reqs], device=dev)
        G[:, 0] = g_root
        tok[:, 1:W + 1] = t1[:, :W].long()
        par[:, 1:W + 1] = 0
        score[:, 1:W + 1] = v1[:, :W].float()
        for d in range(2, D + 1):
            m = W * (d - 1)                                       # nodes 1..m (depths 1..d-1)
            cpar = par[:, 1:m + 1] - 1                            # chunk-local parents (root -> -1)
            cpar = torch.where(cpar < 0, torch.full_like(cpar, -1), cpar)
            anc, _ = ops.tree_mask(cpar.contiguous())
            cpos, cslots, cctx, ccu = [], [], [], [0]
            for i, r in enumerate(reqs):
                n = int(n_vec[i])
                blk = np.asarray(r.blocks, np.int64)
                ps = n - 1 + depth_np[1:m + 1]
                sl = n + np.arange(m)
                cpos.extend(ps.tolist())
                cslots.extend((blk[sl // bs] * bs + sl % bs).tolist())
                cctx.append(n + m)
                ccu.append(ccu[-1] + m)
            cm = _varlen_meta(run, cpos, cslots, brows, ccu, cctx, dev, tree_mask=anc, tree_n=m)
            pidx = par[:, 1:m + 1].long()                          # parents of chunk nodes
            hin = torch.gather(G, 1, pidx[:, :, None].expand(R, m, H)).reshape(R * m, H)
            gc = self.draft.forward(tok[:, 1:m + 1].reshape(-1), hin, cm).view(R, m, H)
            G[:, 1:m + 1] = gc
            fr = torch.arange(m - W + 1, m + 1, device=dev)        # frontier = depth d-1 nodes
            vf, tf = self.draft.topk(gc[:, m - W:].reshape(R * W, H), K)   # [R*W, K]
            tf = self.draft.to_token(tf)
            cand = (score[:, fr][:, :, None] + vf.view(R, W, K).float()).view(R, W * K)
            best, bi = torch.topk(cand, W, dim=1)
            base = 1 + W * (d - 1)
            tok[:, base: base + W] = torch.gather(tf.view(R, W * K).long(), 1, bi)
            par[:, base: base + W] = fr[bi // K].int()
            score[:, base: base + W] = best
        return tok, par

    def _apply_oracle(self, reqs, tok, par, n_vec, D) -> None:
        W = self.spec.width
        V = self.model_cfg.vocab_size
        rows = np.zeros((len(reqs), D), np.int64)
        for i, r in enumerate(reqs):
            fut = self.oracle.get(r.rid, [])
            base = int(n_vec[i]) - len(r.prompt)        # output index of the depth-1 token
            for d in range(D):
                t = fut[base + d] if base + d < len(fut) else 0
                if self._oracle_rng.random() >= self.oracle_accept:
                    t = int(self._oracle_rng.integers(0, V))
                rows[i, d] = t
        chain = torch.from_numpy(rows).to(tok.device)
        for d in range(1, D + 1):
            node = 1 + W * (d - 1)                        # first node of depth d
            tok[:, node] = chain[:, d - 1]
            par[:, node] = 0 if d == 1 else 1 + W * (d - 2)

    def acceptance(self) -> dict:
        s = self.spec_stats
        rows = max(1, s["spec_rows"])
        return {"mean_accepted": s["accepted"] / rows, "tokens_per_step": s["spec_tokens"] / rows,
                "current_depth": self.cur_depth, "spec_on": self.spec_on,
                # the controller's per-bucket cost estimates (ms per generated token)
                "cost_ms_per_token": {f"{m}@{b}": round(v * 1000, 4) for (m, b), v in sorted(self._cost.items())},
                **s}


# ---------------------------------------------------------------------------
# self-distillation of the draft head (EAGLE-style, with training-time unroll)
# ---------------------------------------------------------------------------

def collect_features(engine: SpecEngine, seqs: torch.Tensor) -> tuple:
    """Teacher-forced target pass over token sequences [B, S] -> (raw features [B,S,3H], target argmax [B,S])."""
    run = engine.runner
    B, S = seqs.shape
    dev = engine.device
    pool = engine.pool
    bs = pool.block_size
    need = (S + bs - 1) // bs
    feats, tgts = [], []
    for b in range(B):
        blocks = pool.allocate(need)
        try:
            ps = np.arange(S)
            blk = np.asarray(blocks, np.int64)
            meta = _varlen_meta(run, ps.tolist(), (blk[ps // bs] * bs + ps % bs).tolist(), [blocks], [0, S], [S],
                                dev)
            with torch.inference_mode():
                logits, f = engine._forward_capture(meta, seqs[b].to(dev), fuse=False)
            feats.append(f.clone())
            tgts.append(logits.argmax(-1))
        finally:
            pool.free(blocks)
    return torch.stack(feats), torch.stack(tgts)


def generate_corpus(engine: LLMEngine, num_seqs: int, prompt_len: int, gen_len: int, seed: int = 0) -> torch.Tensor:
    """Random prompts continued greedily by the target -> token sequences [num_seqs, prompt_len + gen_len]."""
    from dgi.sched.request import SamplingParams
    g = torch.Generator().manual_seed(seed)
    V = engine.model_cfg.vocab_size
    lo = min(1000, V // 4)
    prompts = [torch.randint(lo, V, (prompt_len,), generator=g).tolist() for _ in range(num_seqs)]
    reqs = [engine.add_request(p, SamplingParams(max_tokens=gen_len, temperature=0.0, ignore_eos=True))
            for p in prompts]
    while engine.has_unfinished():
        LLMEngine.step(engine)
    return torch.tensor([r.prompt + r.output[:gen_len] for r in reqs], dtype=torch.long)


def hot_vocab_from_targets(tgts: torch.Tensor, vocab: int, size: int) -> torch.Tensor:
    """The ``size`` token ids the target chose most often (ties: lower id first) — EAGLE-3's
    draft vocabulary.  Every chosen token is kept when fewer than ``size`` distinct ones occur."""
    counts = torch.bincount(tgts.reshape(-1).long().cpu(), minlength=vocab).float()
    # tie-break towards lower ids deterministically: subtract a tiny id-proportional amount
    order = torch.argsort(counts - torch.arange(vocab, dtype=torch.float32) / (2.0 * vocab), descending=True)
    return order[:min(size, vocab)].sort().values


AUTO_VOCAB_SIZES = (8192, 16384, 32768, 65536)
AUTO_VOCAB_COVERAGE = 0.99


def auto_draft_vocab(tgts: torch.Tensor, vocab: int, coverage: float = AUTO_VOCAB_COVERAGE,
                     sizes: tuple = AUTO_VOCAB_SIZES) -> int:
    """Smallest draft vocabulary (of ``sizes``) whose most frequent target tokens cover
    ``coverage`` of the training corpus's target choices; 0 (the whole vocabulary) when none
    does.  A draft scoring 32k of Llama-3's 128k tokens streams a quarter of the LM head per
    draft depth (6 x 180 us per batch-1 spec step with the full head, profiles/r5_spec/); on a
    target whose choices spread over the vocabulary the hot set would cap acceptance instead
    (48 % coverage at 32k on the random-init bench target), so the full head stays."""
    counts = torch.bincount(tgts.reshape(-1).long().cpu(), minlength=vocab).float()
    total = float(counts.sum())
    if total <= 0:
        return 0
    csum = torch.cumsum(counts.sort(descending=True).values, 0)
    for n in sizes:
        if n < vocab and float(csum[n - 1]) / total >= coverage:
            return int(n)
    return 0


def train_draft(engine: SpecEngine, steps: int = 200, batch: int = 8, prompt_len: int = 64, gen_len: int = 192,
                unroll: int = 3, lr: float = 1e-3, num_seqs: int = 64, random_seqs: int = 0, seed: int = 0,
                log=None, draft_vocab: int = 0) -> dict:
    """Self-distil the draft head on the target's own greedy continuations.

    A teacher-forced target pass gives the raw low|mid|high features f_p and
    the target's next-token choice at every position.  Draft row p sees
    (x_p, f_{p-1}) and must predict the target token after x_p; unroll step
    k > 1 feeds the draft its own previous hidden instead of f (EAGLE-3
    "training-time test"), matching how deeper tree levels are drafted.
    ``random_seqs`` adds teacher-forced uniformly random token sequences so
    the draft sees the whole vocabulary, not only the tokens the target's
    own continuations happen to visit."""
    dr = engine.draft
    dev = engine.device
    g = torch.Generator().manual_seed(seed + 1)
    V = engine.model_cfg.vocab_size
    seqs = generate_corpus(engine, num_seqs, prompt_len, gen_len, seed)
    if random_seqs:
        lo = min(1000, V // 4)
        rnd = torch.randint(lo, V, (random_seqs, seqs.shape[1]), generator=torch.Generator().manual_seed(seed + 7))
        seqs = torch.cat([seqs, rnd])
    feats, tgts = collect_features(engine, seqs)
    P = {k: v.detach().clone().float().requires_grad_(True) for k, v in dr.parameters().items()}
    opt = torch.optim.AdamW(list(P.values()), lr=lr, weight_decay=0.0)
    S = seqs.shape[1]
    pos0 = torch.arange(S, device=dev)[None]
    hist = []
    for it in range(steps):
        idx = torch.randint(0, seqs.shape[0], (batch,), generator=g)
        ids_k = seqs[idx].to(dev)
        tg_k = tgts[idx.to(dev)]
        Pb = {k: v.to(engine.cfg.dtype) for k, v in P.items()}
        f = F.linear(feats[idx.to(dev)], Pb["fc"])
        hid_k = torch.cat([torch.zeros_like(f[:, :1]), f[:, :-1]], 1)
        pos_k = pos0.expand(batch, -1)
        loss = 0.0
        for k in range(unroll):
            gk = dr.train_forward(Pb, ids_k, hid_k, pos_k)
            lg = dr.train_logits(Pb, gk).float()
            loss = loss + F.cross_entropy(lg.reshape(-1, V), tg_k.reshape(-1)) / unroll
            if ids_k.shape[1] <= 1:
                break
            ids_k, hid_k, pos_k, tg_k = ids_k[:, 1:], gk[:, :-1], pos_k[:, 1:], tg_k[:, 1:]
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        hist.append(float(loss.detach()))
        if log and (it % 50 == 0 or it == steps - 1):
            log(f"draft step {it} loss {hist[-1]:.4f}")
    with torch.no_grad():
        dr.load({k: v.detach() for k, v in P.items()})
    hot = None
    if draft_vocab < 0:
        draft_vocab = auto_draft_vocab(tgts, V)
    if 0 < draft_vocab < V:
        hot_ids = hot_vocab_from_targets(tgts, V, draft_vocab)
        dr.set_hot_vocab(hot_ids)
        covered = float(torch.isin(tgts.reshape(-1).cpu(), hot_ids).float().mean())
        hot = {"size": int(hot_ids.numel()), "target_tokens_covered": round(covered, 4)}
    return {"loss_first": hist[0] if hist else None, "loss_last": hist[-1] if hist else None, "steps": steps,
            "tokens": int(seqs.numel()), "draft_vocab": hot}


@torch.inference_mode()
def greedy_gap(engine: LLMEngine, prompt: list, output: list) -> float:
    """Largest (max logit - chosen logit) over the generated tokens under a
    teacher-forced target pass: 0 for an exact greedy trajectory, small
    positive values only at bf16 near-ties (different kernels may order such
    ties differently)."""
    seq = list(prompt) + list(output)
    S = len(seq) - 1
    pool, run, bs = engine.pool, engine.runner, engine.pool.block_size
    blocks = pool.allocate((S + bs - 1) // bs)
    try:
        ps = np.arange(S)
        blk = np.asarray(blocks, np.int64)
        meta = _varlen_meta(run, ps.tolist(), (blk[ps // bs] * bs + ps % bs).tolist(), [blocks], [0, S], [S],
                            engine.device)
        ids = torch.tensor(seq[:S], dtype=torch.long, device=engine.device)
        logits = engine.model.forward(meta, input_ids=ids).float()
    finally:
        pool.free(blocks)
    rows = logits[len(prompt) - 1:]
    chosen = torch.tensor(output, device=rows.device)
    gap = rows.max(-1).values - rows.gather(1, chosen[:, None])[:, 0]
    return float(gap.max())
