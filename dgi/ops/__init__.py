"""Kernel entry points: HIP (gfx950) on GPU tensors, pure-torch references on CPU.

Every op has two implementations:

* ``torch.ops.dgi.<op>`` from ``dgi/_C.so`` (hand-written CDNA4 HIP kernels,
  see ``dgi/csrc``) — used whenever the tensors live on the GPU.  If the
  extension is missing on a GPU box the op raises: there is no silent
  eager fallback on the device path.
* ``*_ref`` — a plain PyTorch (fp32 accumulate) version of the same math,
  used for CPU execution (the CPU test-suite, OPT-125m config #1) and as the
  numerics oracle of the kernel tests.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import numpy as np
import torch

_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C.so")
_loaded = False
_load_error: Optional[str] = None


def load_native(required: bool = False) -> bool:
    """Load ``dgi/_C.so`` once. ``required`` raises if it cannot be loaded."""
    global _loaded, _load_error
    if _loaded:
        return True
    if os.path.exists(_LIB):
        try:
            torch.ops.load_library(_LIB)
            _loaded = True
            return True
        except Exception as e:  # pragma: no cover - depends on the box
            _load_error = repr(e)
    else:
        _load_error = f"{_LIB} not built (run `python -m dgi.build`)"
    if required:
        raise RuntimeError(f"dgi native kernels unavailable: {_load_error}")
    return False


_WARNED: set = set()


def _warn_once(key: str, msg: str) -> None:
    if key not in _WARNED:
        _WARNED.add(key)
        import warnings
        warnings.warn(msg, RuntimeWarning, stacklevel=3)


def _call(name: str, *args) -> None:
    """Invoke a dgi HIP op; under DGI_DEBUG_SYNC=1 synchronize and name it on a fault."""
    getattr(torch.ops.dgi, name)(*args)
    if _DEBUG_SYNC:
        from dgi.utils.debug import after_op
        after_op(name, *args)


_DEBUG_SYNC = os.environ.get("DGI_DEBUG_SYNC", "0") == "1"


def native_available() -> bool:
    return load_native(False)


def _native(t: torch.Tensor) -> bool:
    if t.is_cuda:
        load_native(required=True)
        return True
    return False


# ----------------------------------------------------------------------------
# RMSNorm
# ----------------------------------------------------------------------------

def rmsnorm_ref(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    return (xf * torch.rsqrt(var + eps) * w.float()).to(x.dtype)


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if _native(x):
        out = torch.empty_like(x) if out is None else out
        _call("rmsnorm", out, x, w, eps)
        return out
    r = rmsnorm_ref(x, w, eps)
    if out is not None:
        out.copy_(r)
        return out
    return r


def fused_add_rmsnorm_ref(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float) -> None:
    s = (x.float() + residual.float()).to(residual.dtype)
    residual.copy_(s)
    x.copy_(rmsnorm_ref(s, w, eps))


def fused_add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float) -> None:
    """residual <- x + residual; x <- rmsnorm(residual) * w (in place)."""
    if _native(x):
        _call("fused_add_rmsnorm", x, residual, w, eps)
    else:
        fused_add_rmsnorm_ref(x, residual, w, eps)


# ----------------------------------------------------------------------------
# RoPE + paged cache write
# ----------------------------------------------------------------------------

def rope_cos_sin(head_dim: int, max_pos: int, theta: float, scaling: Optional[dict] = None,
                 device=None) -> torch.Tensor:
    """[max_pos, head_dim] fp32 table: first half cos, second half sin.

    Supports Llama-3.1 style ``rope_scaling`` (``rope_type == "llama3"``).
    """
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lo = scaling.get("low_freq_factor", 1.0)
        hi = scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (1 - smooth) * inv / factor + smooth * inv
        is_mid = (wl <= lo_wl) & (wl >= hi_wl)
        inv = torch.where(is_mid, mid, scaled)
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], dim=-1).float().to(device)


def _rotate(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    h = x.shape[-1] // 2
    x1, x2 = x[..., :h], x[..., h:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)


def _rotate_interleaved(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    x1, x2 = x[..., 0::2], x[..., 1::2]
    return torch.stack([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).flatten(-2)


def _rope(x: torch.Tensor, cs: torch.Tensor, mode: int) -> torch.Tensor:
    """Rotate the first rd = cs.shape[-1] dims of x (fp32); the rest pass through."""
    rd = cs.shape[-1]
    cos, sin = cs[:, None, : rd // 2], cs[:, None, rd // 2:]
    rot = _rotate(x[..., :rd], cos, sin) if mode == 0 else _rotate_interleaved(x[..., :rd], cos, sin)
    return rot if rd == x.shape[-1] else torch.cat([rot, x[..., rd:]], dim=-1)


def rope_cache_ref(qkv, positions, cos_sin, nh, nkv, hd, slot_mapping, k_cache, v_cache, mode: int = 0) -> None:
    T = qkv.shape[0]
    if T == 0:
        return
    bs = k_cache.shape[2]
    cs = cos_sin[positions.long()]
    q = qkv[:, : nh * hd].float().view(T, nh, hd)
    k = qkv[:, nh * hd:(nh + nkv) * hd].float().view(T, nkv, hd)
    v = qkv[:, (nh + nkv) * hd:(nh + 2 * nkv) * hd].view(T, nkv, hd)
    qr = _rope(q, cs, mode).to(qkv.dtype)
    kr = _rope(k, cs, mode).to(qkv.dtype)
    qkv[:, : nh * hd] = qr.reshape(T, nh * hd)
    slots = slot_mapping.long()
    ok = slots >= 0
    if ok.any():
        s = slots[ok]
        blk, off = s // bs, s % bs
        k_cache[blk, :, off] = kr[ok]
        v_cache[blk, :, off] = v[ok]


def rope_cache(qkv, positions, cos_sin, nh, nkv, hd, slot_mapping, k_cache, v_cache, mode: int = 0) -> None:
    """Rotate q in place inside the fused qkv rows, write rotated k and v into the paged cache.

    ``cos_sin`` is [max_pos, rd] (rd <= hd rotary dims); ``mode`` 0 = NeoX
    pairing (Llama, Qwen2), 1 = interleaved pairs (GLM-4, GPT-J)."""
    if _native(qkv):
        _call("rope_cache", qkv, positions, cos_sin, nh, nkv, hd, slot_mapping, k_cache, v_cache, mode)
    else:
        rope_cache_ref(qkv, positions, cos_sin, nh, nkv, hd, slot_mapping, k_cache, v_cache, mode)


# ----------------------------------------------------------------------------
# Attention
# ----------------------------------------------------------------------------

def _gather_kv(k_cache, v_cache, bt_row, ctx):
    bs = k_cache.shape[2]
    nblk = (ctx + bs - 1) // bs
    ids = bt_row[:nblk].long()
    k = k_cache[ids].permute(0, 2, 1, 3).reshape(nblk * bs, k_cache.shape[1], -1)[:ctx]
    v = v_cache[ids].permute(0, 2, 1, 3).reshape(nblk * bs, v_cache.shape[1], -1)[:ctx]
    return k, v


def paged_decode_ref(q, k_cache, v_cache, block_tables, context_lens, nh, nkv, scale) -> torch.Tensor:
    hd = k_cache.shape[-1]
    B = q.shape[0]
    out = torch.empty(B, nh * hd, dtype=q.dtype, device=q.device)
    G = nh // nkv
    for b in range(B):
        ctx = int(context_lens[b])
        k, v = _gather_kv(k_cache, v_cache, block_tables[b], ctx)
        qb = q[b, : nh * hd].float().view(nkv, G, hd)
        s = torch.einsum("hgd,thd->hgt", qb, k.float()) * scale
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("hgt,thd->hgd", p, v.float())
        out[b] = o.reshape(nh * hd).to(q.dtype)
    return out


def decode_split_plan(batch: int, max_ctx: int, nkv: int, num_cus: int = 256) -> tuple[int, int]:
    """(max_splits, part_size) for the split-KV decode kernel.

    Aim for >= 4 workgroups per CU; part_size is a multiple of 128 tokens
    (4 waves x 32-token tiles)."""
    want = max(1, (4 * num_cus + batch * nkv - 1) // max(1, batch * nkv))
    max_parts = max(1, (max_ctx + 127) // 128)
    splits = min(want, max_parts)
    part = ((max_ctx + splits - 1) // splits + 127) // 128 * 128
    part = max(part, 128)
    splits = (max_ctx + part - 1) // part
    return max(1, splits), part


def paged_decode(q, k_cache, v_cache, block_tables, context_lens, nh, nkv, scale,
                 max_splits: int = 1, part_size: int = 1 << 30, out=None, workspace=None) -> torch.Tensor:
    """Single-token attention for each row of ``q`` over its paged context.

    ``part_size > 0``: fixed parts; ``max_splits``/``part_size`` must cover the
    longest context (``decode_split_plan``).  ``part_size <= 0``: device-side
    plan per sequence — up to ``max_splits`` parts of at least ``-part_size``
    tokens (what captured graphs use).  With ``max_splits > 1`` a workspace
    ``(part_o[B*nh*splits*hd], part_lse[B*nh*splits][, counters[B*nkv] int32 zeros])``
    is used; with counters the last workgroup of each (sequence, kv-head)
    combines the splits (no reduce kernel).
    """
    if _native(q):
        hd = k_cache.shape[-1]
        B = q.shape[0]
        if out is None:
            out = torch.empty(B, nh * hd, dtype=q.dtype, device=q.device)
        cnt = None
        if max_splits > 1:
            if workspace is None:
                workspace = (torch.empty(B * nh * max_splits * hd, dtype=torch.float32, device=q.device),
                             torch.empty(B * nh * max_splits, dtype=torch.float32, device=q.device),
                             torch.zeros(B * nkv, dtype=torch.int32, device=q.device))
            po, pl = workspace[0], workspace[1]
            cnt = workspace[2] if len(workspace) > 2 else None
        else:
            po = pl = torch.empty(0, dtype=torch.float32, device=q.device)
            if part_size > 0:
                part_size = max(128, ((part_size if part_size < (1 << 30) else 1 << 20) + 127) // 128 * 128)
        _call("paged_decode", out, q, k_cache, v_cache, block_tables, context_lens, po, pl,
              nh, nkv, max_splits, part_size, scale, cnt)
        return out
    r = paged_decode_ref(q, k_cache, v_cache, block_tables, context_lens, nh, nkv, scale)
    if out is not None:
        out.copy_(r)
        return out
    return r


def paged_prefill_ref(q, k_cache, v_cache, block_tables, cu_seqlens_q, context_lens, nh, nkv, scale,
                      tree_mask=None, tree_n: int = 0) -> torch.Tensor:
    hd = k_cache.shape[-1]
    T = q.shape[0]
    out = torch.zeros(T, nh * hd, dtype=q.dtype, device=q.device)
    G = nh // nkv
    cu = cu_seqlens_q.tolist()
    for b in range(len(cu) - 1):
        q0, q1 = cu[b], cu[b + 1]
        ql = q1 - q0
        if ql == 0:
            continue
        ctx = int(context_lens[b])
        k, v = _gather_kv(k_cache, v_cache, block_tables[b], ctx)
        qb = q[q0:q1, : nh * hd].float().view(ql, nkv, G, hd)
        s = torch.einsum("qhgd,thd->hgqt", qb, k.float()) * scale
        qpos = torch.arange(ctx - ql, ctx, device=q.device)
        kpos = torch.arange(ctx, device=q.device)
        allow = kpos[None, :] <= qpos[:, None]
        if tree_mask is not None and tree_n > 0:
            tf = ql - tree_n
            key0 = ctx - ql + tf
            bits = tree_mask[b, :tree_n].cpu().tolist()
            for i in range(tree_n):
                m = bits[i] & ((1 << 64) - 1)
                for a in range(tree_n):
                    if key0 + a < ctx and not ((m >> a) & 1):
                        allow[tf + i, key0 + a] = False
        s = s.masked_fill(~allow[None, None], float("-inf"))
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("hgqt,thd->qhgd", p, v.float())
        out[q0:q1] = o.reshape(ql, nh * hd).to(q.dtype)
    return out


# query rows per prefill-attention workgroup: 128 (4 waves) or 256 (8 waves sharing
# each staged K/V tile).  Every producer of ``tiles`` (model runner, EAGLE verify /
# draft metadata, ops.paged_prefill) cuts sequences at this size.
PREFILL_TILE = int(os.environ.get("DGI_PREFILL_TILE", "128"))
# two LDS stages in the prefill attention kernel (one barrier per K/V tile); 0 = the round-4 loop
PREFILL_DB = int(os.environ.get("DGI_PREFILL_DB", "1"))


def order_prefill_tiles(cu_seqlens_q, context_lens=None, tile: int = 0) -> np.ndarray:
    """int32 [n_tiles, 2] (sequence, first query row) of a prefill-attention launch, the
    heaviest tiles first.  A causal tile's work is the keys it reads, kv_end = context -
    qlen + t0 + tile, so in (sequence, row) order the longest workgroups of the last heads
    are dispatched last and run alone at the end of the grid; longest-first ordering lets
    the short ones fill in behind them (the grid is (tiles, heads): every head walks the
    same order).  Ties keep (sequence, row) order."""
    tile = tile or PREFILL_TILE
    cu = np.asarray(cu_seqlens_q, np.int64)
    nb = len(cu) - 1
    ql = cu[1:] - cu[:-1]
    ctx = ql if context_lens is None else np.asarray(context_lens, np.int64)[:nb]
    seq, t0, work = [], [], []
    for b in range(nb):
        starts = np.arange(0, int(ql[b]), tile, dtype=np.int64)
        seq.append(np.full(len(starts), b, np.int64))
        t0.append(starts)
        work.append(np.minimum(int(ctx[b]), int(ctx[b]) - int(ql[b]) + starts + tile))
    if not seq:
        return np.zeros((0, 2), np.int32)
    seq, t0, work = np.concatenate(seq), np.concatenate(t0), np.concatenate(work)
    order = np.argsort(-work, kind="stable")
    return np.stack([seq[order], t0[order]], 1).astype(np.int32)


def prefill_tiles(cu_seqlens_q: list[int], tile: int = 0, context_lens=None) -> list[tuple[int, int]]:
    return [tuple(t) for t in order_prefill_tiles(cu_seqlens_q, context_lens, tile).tolist()]


def paged_prefill(q, k_cache, v_cache, block_tables, cu_seqlens_q, context_lens, nh, nkv, scale,
                  tiles=None, tree_mask=None, tree_n: int = 0, out=None) -> torch.Tensor:
    """Causal varlen attention of packed queries over the paged KV (prefix + new)."""
    if _native(q) and k_cache.shape[-1] not in (64, 128):
        _warn_once("paged_prefill", f"head_dim {k_cache.shape[-1]}: the MFMA prefill kernel is built for 64 / 128; "
                                    "using the PyTorch reference")
    elif _native(q):
        hd = k_cache.shape[-1]
        if out is None:
            out = torch.empty(q.shape[0], nh * hd, dtype=q.dtype, device=q.device)
        if tiles is None:
            tl = prefill_tiles(cu_seqlens_q.tolist(), context_lens=context_lens.tolist())
            tiles = torch.tensor(tl if tl else [[0, 0]], dtype=torch.int32, device=q.device)[: len(tl)]
        _call("paged_prefill", out, q, k_cache, v_cache, block_tables, cu_seqlens_q, context_lens,
              tiles, nh, nkv, scale, tree_mask, tree_n,
              PREFILL_TILE | ((PREFILL_DB & 1) << 16))
        return out
    r = paged_prefill_ref(q, k_cache, v_cache, block_tables, cu_seqlens_q, context_lens, nh, nkv, scale,
                          tree_mask, tree_n)
    if out is not None:
        out.copy_(r)
        return out
    return r


# ----------------------------------------------------------------------------
# MLP activation
# ----------------------------------------------------------------------------

# ----------------------------------------------------------------------------
# Linear: weight-streaming MFMA kernel for decode-sized M, hipBLASLt otherwise
# ----------------------------------------------------------------------------

# Where the skinny kernel beats hipBLASLt (profiles/r1_skinny_gemm.md, weights
# streamed cold from HBM): K <= 4096 projections of 8B-class models at M <= 8
# (1.3-2.1x on qkv / o / gate_up), and square 4096x4096 (o-proj) up to M = 16
# (at M = 32 the end-to-end decode step was no faster).
# Larger K, the 128k-vocab head and every 70B shape stream at 4.5-5.7 TB/s in
# hipBLASLt already.  DGI_SKINNY_MAX_M=0 disables the kernel.
SKINNY_MAX_M = int(os.environ.get("DGI_SKINNY_MAX_M", "32"))


def _use_skinny(M: int, N: int, K: int) -> bool:
    if M > SKINNY_MAX_M or K % 1024 or N % 16 or K > 4096 or N > 32768:
        return False
    # wide projections (8B gate_up, N = 28672) stay ahead of hipBLASLt up to M = 16
    # with the 16-wave config (profiles/r2_decode8b_fused.md, plain GEMM table)
    return M <= 8 or (N <= 4096 and M <= 16) or (N >= 16384 and M <= 16)


SKINNY_CFG = int(os.environ.get("DGI_SKINNY_CFG", "0"))    # > 0 forces a skinny_gemm launch config (sweeps)


def _skinny_cfg(M: int, N: int) -> int:
    if SKINNY_CFG > 0:
        return SKINNY_CFG
    return 5 if (M > 8 and N >= 16384) else 0


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
           out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x @ w.T (+ bias) for a 2-D activation; [N, K] weights as stored."""
    if x.dim() != 2:
        return torch.nn.functional.linear(x, w, bias)
    M, K = x.shape
    N = w.shape[0]
    if (x.is_cuda and _use_skinny(M, N, K) and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and x.stride(1) == 1 and x.stride(0) % 8 == 0 and w.is_contiguous()):
        load_native(required=True)
        if out is None:
            out = torch.empty(M, N, dtype=x.dtype, device=x.device)
        _call("skinny_gemm", out, x, w, bias, _skinny_cfg(M, N))
        return out
    r = torch.nn.functional.linear(x, w, bias)
    if out is not None:
        out.copy_(r)
        return out
    return r


# Fused decode GEMM (fused_decode.hip): RMSNorm prologue + SwiGLU / RoPE+KV epilogue.
# Where it pays (profiles/r2_decode8b_fused.md, hipGraph-timed, weights cold):
# the qkv projection at M <= 8 (15 vs 18 us at M = 1 on 8B); gate_up on the persistent
# one-ring workgroups (cfg 12-16: X staged once per CU, one weight stream per CU) at every
# M <= 16 (55.5 vs 62.4 us unfused at M = 16, profiles/r3_decode/persistent_gemv.md).
# K <= 4096 (8B-class) like _use_skinny.
# DGI_FUSED_DECODE=0 disables, =force uses it for every M <= 16 and K.
FUSED_DECODE = os.environ.get("DGI_FUSED_DECODE", "1")
FUSED_MAX_M = {"qkv": 8, "gate_up": 16}
# launch config per projection and row count (fused_decode.hip cfg = waves, K-steps per load
# group, tiles per workgroup, load ring depth: 6 = 8x1 one-tile ring 4, 7 = 8x1 two-tile ring 4,
# 8 = 4x2 one-tile ring 4, 10 = 8x2 one-tile, 11 = 4x1 one-tile ring 8; persistent one-ring
# workgroups 12 = 8x1 ring 8, 16 = 16x1 ring 4; balanced quarter-pair workgroups 24 = 16x1 ring 4).  Fastest per M on the 8B shapes, weights cold,
# hipGraph-timed (profiles/r3_decode_gemm/README.md, profiles/r3_decode/persistent_gemv.md): qkv
# 16.6 -> 15.0 us at M = 1 against round 2's fixed config 4; gate_up + SwiGLU 48.6 -> 43.0 us at
# M = 1, 56.2 -> 45.5 at M = 4, 66.1 -> 48.2 at M = 8 (cfg 16; 16 waves do not fit M = 16's LDS).
# qkv + RoPE/KV at M <= 8: balanced quarter-pair workgroups, 16 waves (cfg 24: 384 pair tiles
# = 768 quarters, 3 per CU instead of 1.5 whole tiles): 14.96 -> 13.16 us at M = 1, 18.52 -> 17.40
# at M = 4, 21.37 -> 20.23 at M = 8 (profiles/r3_decode/quarter_gemv.md).
FUSED_M_CFG = {"qkv": ((8, 24), (16, 7)), "gate_up": ((8, 16), (16, 12))}
FUSED_KIND_CFG = {"qkv": int(os.environ.get("DGI_FUSED_QKV_CFG", "-1")),
                  "gate_up": int(os.environ.get("DGI_FUSED_GU_CFG", "-1"))}


def fused_cfg(kind: str, M: int) -> int:
    if FUSED_CFG >= 0:
        return FUSED_CFG
    if FUSED_KIND_CFG[kind] >= 0:
        return FUSED_KIND_CFG[kind]
    for m, c in FUSED_M_CFG[kind]:
        if M <= m:
            return c
    return FUSED_M_CFG[kind][-1][1]


def fused_decode_ok(M: int, K: int, kind: str = "qkv") -> bool:
    if FUSED_DECODE == "0" or not 0 < M <= 16 or K % 1024 or M * (K + 8) * 2 > 136 * 1024:
        return False
    if FUSED_DECODE == "force":
        return True
    return K <= 4096 and M <= min(SKINNY_MAX_M, FUSED_MAX_M.get(kind, 0))


def fused_skinny_ref(y, x, res, res_out, gamma, eps, w, bias, pro, epi, positions=None, cos_sin=None,
                     slots=None, k_cache=None, v_cache=None, nh=0, nkv=0):
    """Unfused composition of the same ops (CPU reference / test oracle)."""
    if pro == 2:
        s_ = (x.float() + res.float()).to(x.dtype)
        res_out.copy_(s_)
        xin = s_
    else:
        xin = x
    xn = rmsnorm_ref(xin, gamma, eps) if pro else xin
    out = torch.nn.functional.linear(xn.float(), w.float(), None if bias is None else bias.float()).to(x.dtype)
    if epi == 1:
        out = silu_mul_ref(out)
    elif epi == 2:
        rope_cache_ref(out, positions[: out.shape[0]], cos_sin, nh, nkv, 128, slots[: out.shape[0]], k_cache,
                       v_cache, 0)
    y.copy_(out)
    return y


FUSED_CFG = int(os.environ.get("DGI_FUSED_CFG", "-1"))      # >= 0 overrides FUSED_KIND_CFG


def fused_skinny(y, x, res, res_out, gamma, eps, w, bias, pro: int, epi: int, positions=None, cos_sin=None,
                 slots=None, k_cache=None, v_cache=None, nh: int = 0, nkv: int = 0, cfg: Optional[int] = None):
    """y = epi(rmsnorm_pro(x [+ res]) @ w.T + bias); pro 2 also writes res_out = x + res.

    epi 0 stores [M, N]; epi 1 is SwiGLU over w = [gate; up] (y is [M, I]);
    epi 2 applies NeoX RoPE to the q/k heads of a fused qkv output and writes k/v
    into the paged cache at ``slots`` (head_dim 128, full rotary)."""
    if _native(x):
        if cfg is None:
            cfg = fused_cfg("gate_up" if epi == 1 else "qkv", x.shape[0])
        _call("fused_skinny", y, x, res, res_out, gamma, eps, w, bias, pro, epi, positions, cos_sin, slots,
              k_cache, v_cache, nh, nkv, cfg)
        return y
    return fused_skinny_ref(y, x, res, res_out, gamma, eps, w, bias, pro, epi, positions, cos_sin, slots,
                            k_cache, v_cache, nh, nkv)


# batch-1 decode o-proj (no prologue / epilogue) through the persistent fused GEMV config 16:
# 8.35 vs 8.80 us for the skinny kernel on Llama-3-8B (profiles/r4_decode/plain_proj_fused_configs.json);
# at M >= 2 the skinny kernel is as fast or faster.  DGI_OPROJ_FUSED=0: always ops.linear
OPROJ_FUSED = os.environ.get("DGI_OPROJ_FUSED", "1") == "1"


def decode_proj(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """A decode step's plain projection (o-proj): the persistent fused GEMV at one row,
    ``linear`` otherwise."""
    M, K = x.shape
    if (OPROJ_FUSED and M == 1 and _native(x) and x.dtype == torch.bfloat16 and x.is_contiguous()
            and w.dtype == torch.bfloat16 and w.is_contiguous() and w.shape[1] == K
            and fused_decode_ok(M, K, "qkv") and w.shape[0] % 16 == 0):
        y = torch.empty(M, w.shape[0], dtype=x.dtype, device=x.device)
        _call("fused_skinny", y, x, None, None, None, 0.0, w, None, 0, 0, None, None, None, None, None, 0, 0, 16)
        return y
    return linear(x, w)


_PREFETCH_SINKS: dict = {}


def mall_prefetch(w: torch.Tensor, rows: Optional[torch.Tensor] = None, nrows: int = -1, blocks: int = 256) -> None:
    """Read ``w``'s rows (all, the first ``nrows``, or the int32 ids ``rows``) so that a later
    kernel finds them in the memory-side cache (dgi/csrc/prefetch.hip).  Nothing is written;
    a no-op off the native path."""
    if not _native(w):
        return
    sink = _PREFETCH_SINKS.get(w.device)
    if sink is None:
        sink = _PREFETCH_SINKS[w.device] = torch.zeros(256, dtype=torch.int32, device=w.device)
    _call("mall_prefetch", w, rows, sink, nrows, blocks)


def silu_mul_ref(gu: torch.Tensor) -> torch.Tensor:
    I = gu.shape[-1] // 2
    g = gu[..., :I].float()
    return (torch.nn.functional.silu(g) * gu[..., I:].float()).to(gu.dtype)


def silu_mul(gu: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if _native(gu):
        if out is None:
            out = torch.empty(*gu.shape[:-1], gu.shape[-1] // 2, dtype=gu.dtype, device=gu.device)
        _call("silu_mul", out, gu)
        return out
    r = silu_mul_ref(gu)
    if out is not None:
        out.copy_(r)
        return out
    return r


def mfma_gemm_ref(x: torch.Tensor, w: torch.Tensor, epi: int = 0) -> torch.Tensor:
    """fp32 reference of ``mfma_gemm``: x @ w.T, or SwiGLU over w = [gate; up]."""
    y = x.float() @ w.float().t()
    if epi == 1:
        I = w.shape[0] // 2
        y = torch.nn.functional.silu(y[:, :I]) * y[:, I:]
    return y.to(x.dtype)


def mfma_gemm_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Shapes/layouts the LDS-tiled MFMA GEMM kernel takes (dgi/csrc/mfma_gemm.hip)."""
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 2
            and x.stride(1) == 1 and x.stride(0) % 8 == 0 and w.is_contiguous() and w.shape[0] % 256 == 0
            and x.shape[1] % 64 == 0 and x.data_ptr() % 16 == 0 and x.shape[0] * x.stride(0) < (1 << 31))


MFMA_SCHED = int(os.environ.get("DGI_MFMA_SCHED", "3"))


def set_gemm_cus(cus: int) -> None:
    """CUs the MFMA GEMM's persistent / split-K launches size their grid for (0 = all of the
    device's): GEMMs issued on a CU-masked stream (two-batch overlap) set its CU count."""
    if native_available():
        torch.ops.dgi.set_gemm_cus(int(cus))


def gemm_split_timeouts(reset: bool = False) -> int:
    """Split-K waits of the MFMA GEMM on the current device that ran out since the last reset
    (the last piece of a tile waits, bounded, for the other pieces' slabs; a timeout means a wrong
    tile).  0 in a healthy process; synchronizes the device.  DGI_DEBUG_SYNC=1 checks it after
    every GEMM."""
    if not native_available() or not torch.cuda.is_available():
        return 0
    return int(torch.ops.dgi.gemm_split_timeouts(bool(reset)))


def mfma_gemm(x: torch.Tensor, w: torch.Tensor, epi: int = 0, out: Optional[torch.Tensor] = None,
              sched: Optional[int] = None, streamk: int = 0, prio: int = 0, phases: int = 0,
              overlap: bool = True) -> torch.Tensor:
    """Hand-written LDS-tiled MFMA GEMM (256x256 tiles, global_load_lds
    staging, XCD-aware tile order): ``epi`` 0 -> x @ w.T; 1 -> the fused
    SwiGLU of the MLP, silu(x @ gate.T) * (x @ up.T) with w = [gate; up],
    written once (no [M, 2I] intermediate and no separate silu_mul pass).
    ``sched`` 3 is the ping-pong schedule; its ``streamk`` (split-K of the
    last partial wave) policy: 0 auto, 1 off, 2 whenever it applies;
    ``phases`` per K tile: 0 auto (2 up to M = 2560, else 4), 2 or 4;
    ``prio``: s_setprio variant (benchmarking); ``overlap`` False: no
    cross-tile prologue / epilogue overlap (A/B)."""
    M = x.shape[0]
    N = w.shape[0] // 2 if epi == 1 else w.shape[0]
    if mfma_gemm_ok(x, w):
        load_native(required=True)
        if out is None:
            out = torch.empty(M, N, dtype=x.dtype, device=x.device)
        _call("mfma_gemm", out, x, w, epi | ((MFMA_SCHED if sched is None else sched) << 4) | (streamk << 8)
              | (prio << 10) | ((1 if phases == 2 else 0) << 12) | ((1 if phases == 4 else 0) << 13)
              | ((0 if overlap else 1) << 14))
        return out
    r = mfma_gemm_ref(x, w, epi)
    if out is not None:
        out.copy_(r)
        return out
    return r


NORM_RES, NORM_PLAIN, NORM_SWIGLU = 2, 3, 4


def mfma_gemm_norm_ref(x: torch.Tensor, w: torch.Tensor, kind: int, ss: torch.Tensor, eps: float,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 reference of ``mfma_gemm_norm`` (same contract, any device)."""
    y = x.float() @ w.float().t()
    M = x.shape[0]
    if kind == NORM_RES:
        new = (out.float() + y).to(out.dtype)
        out.copy_(new)
        nf = new.float()
        ss[:M, : w.shape[0] // 256].copy_((nf * nf).view(M, -1, 256).sum(-1))
        return out
    rstd = torch.rsqrt(ss[:M].sum(-1, keepdim=True) / x.shape[1] + eps)
    y = y * rstd
    if kind == NORM_SWIGLU:
        I = w.shape[0] // 2
        y = torch.nn.functional.silu(y[:, :I]) * y[:, I:]
    r = y.to(x.dtype)
    if out is None:
        return r
    out.copy_(r)
    return out


def mfma_gemm_norm(x: torch.Tensor, w: torch.Tensor, kind: int, ss: torch.Tensor, eps: float,
                   out: Optional[torch.Tensor] = None, phases: int = 0) -> torch.Tensor:
    """The ping-pong MFMA GEMM with a fused RMSNorm epilogue (dgi/csrc/mfma_gemm.hip, EPI 2-4).

    ``kind`` 2 (NORM_RES): ``out`` is the residual stream, updated in place to out + x @ w.T,
    and ``ss[m, j]`` receives the sum of squares of the new row m over columns 256 j .. 256 j + 255
    (``ss`` has at least N / 256 columns; the consumers read a multiple of 8 <= 32, extra
    columns zero): the statistics of the next RMSNorm, with no norm kernel.
    ``kind`` 3 / 4 (NORM_PLAIN / NORM_SWIGLU): x is the un-normalised residual stream and
    ``w`` carries the norm's gain (``LlamaModel.fold_norms``); each output row is scaled by
    rsqrt(sum(ss[m]) / K + eps) — then SwiGLU for kind 4 — which equals
    (rmsnorm(x) * gamma) @ w.T up to rounding."""
    M = x.shape[0]
    N = w.shape[0] // 2 if kind == NORM_SWIGLU else w.shape[0]
    if kind == NORM_RES and out is None:
        raise ValueError("mfma_gemm_norm: kind 2 updates the residual `out` in place")
    if _native(x):
        if out is None:
            out = torch.empty(M, N, dtype=x.dtype, device=x.device)
        _call("mfma_gemm_norm", out, x, w, kind, ss, 1.0 / x.shape[1], eps, phases)
        return out
    return mfma_gemm_norm_ref(x, w, kind, ss, eps, out)


def mfma_gemm_norm_rope_ref(x, w, ss, eps, positions, cos_sin, slots, k_cache, v_cache, nh, nkv,
                            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 reference of ``mfma_gemm_norm_rope``: the normalised qkv (bf16), then RoPE + paged KV
    write (``rope_cache_ref``, NeoX, head dim 128)."""
    y = mfma_gemm_norm_ref(x, w, NORM_PLAIN, ss, eps)
    rope_cache_ref(y, positions[: x.shape[0]], cos_sin, nh, nkv, 128, slots[: x.shape[0]], k_cache, v_cache, 0)
    if out is None:
        return y
    out.copy_(y)
    return out


def mfma_gemm_norm_rope(x, w, ss, eps, positions, cos_sin, slots, k_cache, v_cache, nh: int, nkv: int,
                        out: Optional[torch.Tensor] = None, phases: int = 0) -> torch.Tensor:
    """The normalised qkv projection with RoPE and the paged-KV write in its epilogue
    (mfma_gemm.hip EPI 5): returns y whose q columns are rotated (its k / v columns are NOT
    written — they go to ``k_cache`` / ``v_cache`` at ``slots``, which attention reads), i.e.
    ``mfma_gemm_norm(x, w, NORM_PLAIN, ss)`` followed by ``rope_cache`` in one kernel.  Llama
    geometry: head dim 128, full NeoX rotary, cos_sin [max_pos, 128]."""
    if _native(x):
        if out is None:
            out = torch.empty(x.shape[0], w.shape[0], dtype=x.dtype, device=x.device)
        _call("mfma_gemm_norm_rope", out, x, w, ss, 1.0 / x.shape[1], eps, positions, cos_sin, slots, k_cache,
              v_cache, nh, nkv, phases)
        return out
    return mfma_gemm_norm_rope_ref(x, w, ss, eps, positions, cos_sin, slots, k_cache, v_cache, nh, nkv, out)


def mfma_norm_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Shapes the fused-norm GEMM takes (K % 128 and >= 256 on top of ``mfma_gemm_ok``; a
    normalising consumer also needs its K — the stream width — <= 8192: 32 row partials)."""
    return mfma_gemm_ok(x, w) and x.shape[1] % 128 == 0 and x.shape[1] >= 256


def row_sumsq(x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out[:, 0] = sum of squares of each row of x (fp32), the other columns zero: the
    statistics the fused-norm GEMM reads for a stream no residual epilogue produced (the
    first layer's input)."""
    out.zero_()
    xf = x.float()
    out[: x.shape[0], 0] = (xf * xf).sum(-1)
    return out


# ----------------------------------------------------------------------------
# Sampling
# ----------------------------------------------------------------------------

def topkp_threshold(logits: torch.Tensor, temperature: torch.Tensor, top_k: torch.Tensor,
                    top_p: torch.Tensor) -> torch.Tensor:
    """Per-row logit cut for top-k / top-p: keep ``logits >= thresh`` (fp32 [B]).

    HF / vLLM order (temperature, then top-k, then nucleus over the top-k
    survivors, renormalised): element v is kept iff ``#{u > v} < top_k`` and
    ``sum_{u > v} exp(u / T) <= top_p * Z_k`` where ``Z_k`` is the softmax mass of
    the top-k set.  Ties at the cut are kept.  Rows that are greedy (T <= 1e-5)
    or unfiltered (top_k <= 0 and top_p >= 1) get -inf.  Native path: one HIP
    kernel (sampler.hip, interval searches with register-resident counters; no
    sort)."""
    B, V = logits.shape
    if _native(logits):
        th = torch.empty(B, dtype=torch.float32, device=logits.device)
        _call("topkp_threshold", th, logits, temperature.float().contiguous(), top_k.long().contiguous(),
                                      top_p.float().contiguous())
        return th
    lf = logits.float()
    s, _ = lf.sort(dim=-1, descending=True)
    t = temperature.float().clamp(min=1e-5)[:, None]
    fin = torch.isfinite(s)
    e = torch.where(fin, torch.exp((s - s[:, :1]) / t), torch.zeros_like(s))
    cum_excl = e.cumsum(-1) - e
    asc = s.flip(-1).contiguous()
    cnt_gt = V - torch.searchsorted(asc, s, right=True)              # #{u > v}
    mass_gt = cum_excl.gather(-1, cnt_gt.clamp(max=V - 1))           # sum over u > v
    k = torch.where(top_k > 0, top_k.long().clamp(max=V), torch.full_like(top_k.long(), V))
    in_k = (cnt_gt < k[:, None]) & fin
    z_k = torch.where(in_k, e, torch.zeros_like(e)).sum(-1, keepdim=True)   # mass of the top-k survivors
    ok = in_k & (mass_gt <= top_p.float()[:, None] * z_k)
    last = ok.sum(-1) - 1                                            # kept prefix of the sorted row
    th = s.gather(-1, last.clamp(min=0)[:, None]).squeeze(-1)
    keep_all = ok.sum(-1) == fin.sum(-1)                             # every finite logit survives
    off = (temperature <= 1e-5) | ((top_k <= 0) & (top_p >= 1.0)) | keep_all
    return torch.where(off.to(th.device), torch.full_like(th, float("-inf")), th)


def apply_top_k_top_p(logits: torch.Tensor, top_k: torch.Tensor, top_p: torch.Tensor,
                      temperature: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Mask (to -inf) the logits outside the top-k / top-p set (see ``topkp_threshold``)."""
    if temperature is None:
        temperature = torch.ones(logits.shape[0], device=logits.device)
    th = topkp_threshold(logits, temperature, top_k, top_p)
    lf = logits.float()
    return lf.masked_fill(lf < th[:, None], float("-inf"))


_M32 = 0xFFFFFFFF


def _hash32(x: torch.Tensor) -> torch.Tensor:
    """sampler.hip ``hash32`` on int64 tensors holding uint32 values (products
    wrap mod 2^64, so the low 32 bits are exact)."""
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def gumbel_uniform(seeds: Optional[torch.Tensor], step: int, V: int, B: int) -> torch.Tensor:
    """The per-(row, vocab id) uniforms the HIP sampler draws: a counter-based
    hash of (row seed, step, token id), so a row's draw depends on its own seed
    only (never on the batch it shares) and CPU and GPU pick the same tokens."""
    sd = seeds.long().cpu() if seeds is not None else torch.zeros(B, dtype=torch.long)
    row = ((sd * 2654435761) & _M32) ^ ((step * 40503) & _M32)
    ids = _hash32((torch.arange(V, dtype=torch.long) + 0x9E3779B9) & _M32)
    h = _hash32(row[:, None] ^ ids[None, :])
    return ((h >> 8).float() + 0.5) * (1.0 / 16777216.0)


def sample(logits: torch.Tensor, temperature: Optional[torch.Tensor] = None,
           seeds: Optional[torch.Tensor] = None, step: int = 0, out: Optional[torch.Tensor] = None,
           top_k: Optional[torch.Tensor] = None, top_p: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Greedy (temperature 0) or Gumbel-max sampling per row; returns int64 token ids.

    With ``top_k`` / ``top_p`` the draw is restricted to ``topkp_threshold``'s set
    (on GPU: a threshold kernel + the threshold-aware sampler, no sort and no
    masked copy of the logits)."""
    B = logits.shape[0]
    filt = top_k is not None and top_p is not None and temperature is not None
    if _native(logits):
        if out is None:
            out = torch.empty(B, dtype=torch.long, device=logits.device)
        th = topkp_threshold(logits, temperature, top_k, top_p) if filt else None
        _call("sample", out, logits, temperature, seeds, step, th)
        return out
    if filt:
        logits = apply_top_k_top_p(logits, top_k, top_p, temperature)
    lf = logits.float()
    if temperature is None or bool((temperature <= 1e-5).all()):
        r = lf.argmax(-1)
    else:
        t = temperature.float().clamp(min=1e-5)
        noisy = lf / t[:, None] - torch.log(-torch.log(gumbel_uniform(seeds, step, lf.shape[1], B)))
        r = torch.where(temperature <= 1e-5, lf.argmax(-1), noisy.argmax(-1))
    if out is not None:
        out.copy_(r)
        return out
    return r


def topk_logprobs(logits: torch.Tensor, k: int):
    """Top-k (k <= 16) of ``log_softmax(logits.float())`` per row: fp32 log-probs and int64
    indices, descending (ties: lower index first).  Native path (k <= 8): two HIP kernels
    straight from bf16 logits (sampler.hip: chunked top-k + logsumexp, then a per-row merge)."""
    if _native(logits) and logits.dtype == torch.bfloat16 and logits.stride(-1) == 1 \
            and logits.stride(0) % 8 == 0 and k <= 8:
        B = logits.shape[0]
        v = torch.empty(B, k, dtype=torch.float32, device=logits.device)
        i = torch.empty(B, k, dtype=torch.long, device=logits.device)
        _call("topk_logprobs", v, i, logits, k)
        return v, i
    return topk(torch.log_softmax(logits.float(), dim=-1), k)


def topk(logits: torch.Tensor, k: int):
    """Top-k (k <= 16) values (fp32) and indices (int64), descending."""
    if _native(logits):
        B = logits.shape[0]
        v = torch.empty(B, k, dtype=torch.float32, device=logits.device)
        i = torch.empty(B, k, dtype=torch.long, device=logits.device)
        _call("topk", v, i, logits, k)
        return v, i
    v, i = logits.float().topk(k, dim=-1)
    return v, i


# ----------------------------------------------------------------------------
# KV block movement
# ----------------------------------------------------------------------------

def kv_gather(cache: torch.Tensor, ids: torch.Tensor, out: Optional[torch.Tensor] = None,
              block_major: bool = False) -> torch.Tensor:
    """cache [L,2,NB,...] -> [L,2,n,...] pages of ``ids`` (``block_major``: [n,L,2,...], every
    layer of one page contiguous — the host KV tier's slot layout)."""
    if _native(cache):
        if out is None:
            shape = ((ids.numel(), cache.shape[0], cache.shape[1]) if block_major else
                     (cache.shape[0], cache.shape[1], ids.numel())) + tuple(cache.shape[3:])
            out = torch.empty(shape, dtype=cache.dtype, device=cache.device)
        _call("kv_gather", out, cache, ids, bool(block_major))
        return out
    r = cache[:, :, ids.long()]
    if block_major:
        r = r.permute(2, 0, 1, 3, 4, 5).contiguous()
    if out is not None:
        out.copy_(r.view(out.shape))
        return out
    return r


def kv_scatter(cache: torch.Tensor, ids: torch.Tensor, buf: torch.Tensor, block_major: bool = False) -> None:
    if _native(cache):
        _call("kv_scatter", cache, ids, buf, bool(block_major))
    elif block_major:
        cache[:, :, ids.long()] = buf.reshape(ids.numel(), cache.shape[0], cache.shape[1],
                                              *cache.shape[3:]).permute(1, 2, 0, 3, 4, 5)
    else:
        cache[:, :, ids.long()] = buf.view(cache.shape[0], cache.shape[1], ids.numel(), *cache.shape[3:])


def kv_copy(cache: torch.Tensor, src: torch.Tensor, dst: torch.Tensor) -> None:
    """Copy pages src[i] -> dst[i] for every layer (src/dst sets must be disjoint)."""
    if _native(cache):
        _call("kv_copy", cache, src, dst)
    else:
        cache[:, :, dst.long()] = cache[:, :, src.long()]


# ----------------------------------------------------------------------------
# EAGLE tree
# ----------------------------------------------------------------------------

def tree_mask_ref(parent: torch.Tensor):
    B, N = parent.shape
    anc = torch.zeros(B, 64, dtype=torch.long)
    depth = torch.zeros(B, N, dtype=torch.int32)
    par = parent.cpu().tolist()
    for b in range(B):
        for n in range(N):
            m = 1 << n
            d = 0
            p = par[b][n]
            while p >= 0:
                m |= 1 << p
                p = par[b][p]
                d += 1
            if m >= 1 << 63:
                m -= 1 << 64
            anc[b, n] = m
            depth[b, n] = d
    return anc.to(parent.device), depth.to(parent.device)


def tree_mask(parent: torch.Tensor):
    """Ancestor-or-self bitmask [B,64] (int64 bit patterns) and depth [B,N]."""
    if _native(parent):
        B, N = parent.shape
        anc = torch.zeros(B, 64, dtype=torch.long, device=parent.device)
        depth = torch.empty(B, N, dtype=torch.int32, device=parent.device)
        _call("tree_mask", anc, depth, parent)
        return anc, depth
    return tree_mask_ref(parent)


def tree_verify_ref(parent, draft, target, anc, depth, max_path: int):
    B, N = parent.shape
    acc = torch.zeros(B, dtype=torch.int32)
    path = torch.zeros(B, max_path, dtype=torch.int32)
    toks = torch.zeros(B, max_path + 1, dtype=torch.long)
    par, dr, tg = parent.cpu().tolist(), draft.cpu().tolist(), target.cpu().tolist()
    dp = depth.cpu().tolist()
    for b in range(B):
        ok = [False] * N
        for n in range(N):
            if n == 0:
                ok[n] = True
            else:
                ok[n] = ok[par[b][n]] and dr[b][n] == tg[b][par[b][n]]
        best, bd = 0, 0
        for n in range(N):
            if ok[n] and dp[b][n] > bd:
                best, bd = n, dp[b][n]
        acc[b] = bd
        node = best
        for k in range(bd, -1, -1):
            if k < max_path:
                path[b, k] = node
                if k > 0:
                    toks[b, k - 1] = dr[b][node]
            node = par[b][node] if node > 0 else 0
        if bd < max_path + 1:
            toks[b, bd] = tg[b][best]
    dev = parent.device
    return acc.to(dev), path.to(dev), toks.to(dev)


def tree_verify(parent, draft, target, anc, depth, max_path: int):
    """Greedy tree acceptance: (accept_len[B], path[B,max_path], tokens[B,max_path+1])."""
    if _native(parent):
        B = parent.shape[0]
        acc = torch.empty(B, dtype=torch.int32, device=parent.device)
        path = torch.zeros(B, max_path, dtype=torch.int32, device=parent.device)
        toks = torch.zeros(B, max_path + 1, dtype=torch.long, device=parent.device)
        _call("tree_verify", acc, path, toks, parent, draft, target, anc, depth)
        return acc, path, toks
    return tree_verify_ref(parent, draft, target, anc, depth, max_path)
