"""Model runner: ScheduledBatch -> device metadata -> forward -> sampled tokens.

* All int32 step metadata (token ids, positions, slot mapping, block tables,
  context lengths, cu_seqlens, attention tiles) is packed into ONE pinned host
  buffer and moved with a single async H2D copy per step.
* Pure-decode steps replay a hipGraph captured per batch-size bucket
  (``GraphRunner``): the 80-layer Llama-3-70B decode step is ~900 kernel
  launches, which the graph turns into one replay with no host work per
  kernel (SURVEY §7.1 "fixed-shape decode in hipGraphs").
* Mixed prefill+decode steps run eagerly (their GEMMs dominate).
"""
from __future__ import annotations

import contextlib
import dataclasses
import gc
import itertools
import os
import time
from typing import Optional

import numpy as np
import torch

from dgi import ops
from dgi.runtime.batch import AttnMeta
from dgi.sched.scheduler import ScheduledBatch

DEFAULT_BUCKETS = (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192, 224, 256, 320, 384, 448, 512)


@dataclasses.dataclass
class SamplingMeta:
    """Per-row sampling parameters of one step, as device views of the step buffer."""
    temps: torch.Tensor
    seeds: torch.Tensor
    top_k: Optional[torch.Tensor] = None     # None: no row of this step is filtered
    top_p: Optional[torch.Tensor] = None

    def sample(self, logits: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        return ops.sample(logits, self.temps, self.seeds, 0, out=out, top_k=self.top_k, top_p=self.top_p)


@dataclasses.dataclass
class StepResult:
    tokens: list          # sampled token per logits row (decode rows first, then sampled chunks)
    rows: list            # Request per sampled row
    hidden: Optional[torch.Tensor] = None


@contextlib.contextmanager
def graph_capture(g, pool=None):
    """``torch.cuda.graph`` with Python's cyclic GC held off while the stream is
    capturing: a collection that frees an object owning device memory or a graph
    from an earlier engine during capture aborts the process (seen in the GPU
    suite when one engine's graphs were collected while the next engine captured)."""
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(g, pool=pool):
            yield
    finally:
        if was:
            gc.enable()


def decode_rows(reqs: list, bs: int, bt_out: np.ndarray, ahead: int = 0):
    """Per-row decode metadata of ``reqs``, vectorised (the per-request Python work is
    one attribute read per field): returns (input token, position, KV slot, context
    length) int32 arrays and fills ``bt_out[:n]`` (zeroed by the caller) with the
    block tables.  ``ahead``: tokens each row has in flight that are not applied yet
    (decode lookahead: positions move on by that many; the input token then comes
    from the device, the returned ids are placeholders)."""
    n = len(reqs)
    pos = np.fromiter((r.num_computed + ahead for r in reqs), np.int32, n)
    ids = np.fromiter((r.output[-1] if r.output else r.prompt[-1] for r in reqs), np.int32, n)
    lens = np.fromiter((len(r.blocks) for r in reqs), np.int64, n)
    tot = int(lens.sum())
    flatb = np.fromiter(itertools.chain.from_iterable(r.blocks for r in reqs), np.int32, tot)
    starts = np.cumsum(lens) - lens
    rows = np.repeat(np.arange(n), lens)
    cols = np.arange(tot) - np.repeat(starts, lens)
    bt_out[rows, cols] = flatb
    slots = bt_out[np.arange(n), pos // bs] * bs + pos % bs
    return ids, pos, slots.astype(np.int32), pos + 1


def sampling_rows(sampled: list, ahead=0):
    """(temperature bits, seed, top-k, top-p bits, any filtered) of the sampled rows; ``ahead``
    (tokens of each row still in flight) is one number or one per row."""
    n = len(sampled)
    nf = [r.params.needs_filter for r in sampled]
    temps = np.fromiter((r.params.temperature for r in sampled), np.float32, n).view(np.int32)
    if isinstance(ahead, int):
        seeds = np.fromiter((r.sample_seed(ahead) for r in sampled), np.int64, n).astype(np.int32)
    else:
        seeds = np.fromiter((r.sample_seed(a) for r, a in zip(sampled, ahead)), np.int64, n).astype(np.int32)
    topk = np.fromiter((max(0, r.params.top_k) if f else 0 for r, f in zip(sampled, nf)), np.int32, n)
    topp = np.fromiter((r.params.top_p if f else 1.0 for r, f in zip(sampled, nf)), np.float32, n).view(np.int32)
    return temps, seeds, topk, topp, any(nf)


class ModelRunner:
    def __init__(self, model, pool, max_num_seqs: int = 256, max_model_len: int = 8192,
                 max_num_batched_tokens: int = 8192, use_graphs: bool = True,
                 graph_buckets=DEFAULT_BUCKETS, decode_part_size: int = 256, num_cus: int = 256):
        self.model = model
        self.pool = pool
        self.device = pool.device
        self.bs = pool.block_size
        self.max_num_seqs = max_num_seqs
        self.max_model_len = max_model_len
        self.max_blocks = (max_model_len + self.bs - 1) // self.bs
        self.max_tokens = max_num_batched_tokens
        self.num_cus = num_cus
        self.step_id = 0
        model.kv_cache = pool.kv
        self.is_cuda = self.device.type == "cuda"
        # decode split-KV plan used by graphs (fixed) and workspaces
        self.graph_part = decode_part_size
        self.graph_splits = (max_model_len + decode_part_size - 1) // decode_part_size
        self.ws_splits = (max_model_len + 127) // 128
        nh, hd = model.cfg.num_heads, model.cfg.head_dim
        maxb = max(max_num_seqs, max(graph_buckets) if graph_buckets else 1)
        self.dec_ws = None
        if self.is_cuda:
            # partial O / log-sum-exp per split + one ticket counter per (sequence, kv-head) for the
            # in-kernel split reduce (write-through partials, one acquire on the last arriver; round 3's
            # form fenced every workgroup, which wrote back L2 and cost more than a reduce kernel).
            # Opt-in (DGI_DECODE_FUSED_REDUCE=1): 8B TPOT ties the reduce kernel at batch 1-4 and
            # loses 0.09-0.23 ms at batch 16-64, where the last arriver's serial combine is the
            # tail of the launch (profiles/r4_decode/README.md)
            self.dec_ws = (torch.empty(maxb * nh * self.ws_splits * hd, dtype=torch.float32, device=self.device),
                           torch.empty(maxb * nh * self.ws_splits, dtype=torch.float32, device=self.device))
            if os.environ.get("DGI_DECODE_FUSED_REDUCE", "0") == "1":
                self.dec_ws += (torch.zeros(maxb * model.cfg.num_kv_heads, dtype=torch.int32, device=self.device),)
        # called while the host waits for a step's sampled tokens (P/D ranks keep
        # their KV handshakes moving instead of blocking in a stream synchronize)
        self.wait_hook = None
        # pinned host KV tier of the engine (restores run on its copy stream; every forward gates
        # on the last one, ``gate``)
        self.host_tier = None
        self._spans = []
        self.span_total_ms = 0.0
        self.graphs = None
        if use_graphs and self.is_cuda and model.has_head:
            self.graphs = GraphRunner(self, [b for b in graph_buckets if b <= max_num_seqs])

    # ------------------------------------------------------------------ metadata
    # header layout (int64): the host-side shape of one step, shipped along
    # the pipeline so every stage rebuilds the same AttnMeta
    H_LEN, H_T, H_NDP, H_NPRE, H_NB, H_MAXW, H_SPLITS, H_PART, H_NTILES, H_NLOG, H_STEP, H_FILT = range(1, 13)
    HEADER_SIZE = 16

    def prebuild_decode(self, reqs: list, ahead: int = 1) -> dict:
        """Per-row decode metadata of ``reqs`` for the step AFTER the one in flight (positions
        ``ahead`` further on; the input tokens are filled in when that step's tokens are
        back): what ``build_host(..., dec_pre=...)`` takes for the first rows of its batch.
        The pipeline driver builds it while it waits for the tokens (``PipelineEngine``)."""
        n = len(reqs)
        bt = np.zeros((n, self.max_blocks), np.int32)
        _ids, pos, slots, ctx = decode_rows(reqs, self.bs, bt, ahead)
        temps, seeds, topk, topp, filt = sampling_rows(reqs, ahead)
        return {"rows": list(reqs), "pos": pos, "slots": slots, "ctx": ctx, "bt": bt,
                "samp": (temps, seeds, topk, topp), "filt": filt}

    @staticmethod
    def subset_prebuilt(pre: dict, keep: np.ndarray) -> dict:
        """The rows of a ``prebuild_decode`` result where ``keep`` is True."""
        idx = np.flatnonzero(keep)
        samp = tuple(a[idx] for a in pre["samp"])
        return {"rows": [pre["rows"][i] for i in idx], "pos": pre["pos"][idx], "slots": pre["slots"][idx],
                "ctx": pre["ctx"][idx], "bt": pre["bt"][idx], "samp": samp,
                "filt": bool((samp[2] > 0).any() or (samp[3].view(np.float32) < 1.0).any())}

    def build_host(self, sb: ScheduledBatch, pad_decode_to: int = 0, dec_pre: Optional[dict] = None,
                   pre_ids: Optional[np.ndarray] = None, seed_ahead=None):
        """Pack one step's metadata into a flat int32 array + int64 header.  ``dec_pre``
        (``prebuild_decode``) holds the first decode rows' metadata, built ahead; their input
        tokens are ``pre_ids``.  ``seed_ahead``: per sampled row, tokens still in flight (a
        step scheduled before the previous step's tokens are applied)."""
        bs = self.bs
        nd = len(sb.decode)
        ndp = max(nd, pad_decode_to)
        chunks = sb.prefill
        npre = sum(c.length for c in chunks)
        T = ndp + npre
        ids = np.zeros(T, np.int32)
        pos = np.zeros(T, np.int32)
        slots = np.zeros(T, np.int32)
        maxw = self.max_blocks
        dec_bt = np.zeros((ndp, maxw), np.int32)
        dec_ctx = np.ones(ndp, np.int32)
        k = len(dec_pre["rows"]) if dec_pre is not None else 0
        if k:
            ids[:k] = pre_ids
            pos[:k], slots[:k], dec_ctx[:k] = dec_pre["pos"], dec_pre["slots"], dec_pre["ctx"]
            dec_bt[:k] = dec_pre["bt"]
        if nd > k:
            ids[k:nd], pos[k:nd], slots[k:nd], dec_ctx[k:nd] = decode_rows(sb.decode[k:], bs, dec_bt[k:nd])
        # padded decode rows write into reserved block 0 and read it back
        nb = len(chunks)
        pre_bt = np.zeros((nb, maxw), np.int32)
        cu = np.zeros(nb + 1, np.int32)
        pctx = np.zeros(nb, np.int32)
        logit_rows = list(range(nd))
        row = ndp
        sampled = list(sb.decode)
        for j, c in enumerate(chunks):
            r = c.req
            toks = r.all_tokens()
            ids[row: row + c.length] = toks[c.start: c.start + c.length]
            p = np.arange(c.start, c.start + c.length, dtype=np.int32)
            pos[row: row + c.length] = p
            blk = np.asarray(r.blocks, np.int32)
            slots[row: row + c.length] = blk[p // bs] * bs + p % bs
            pre_bt[j, : len(r.blocks)] = blk
            cu[j + 1] = cu[j] + c.length
            pctx[j] = c.start + c.length
            if c.sample:
                logit_rows.append(row + c.length - 1)
                sampled.append(r)
            row += c.length
        tiles_np = ops.order_prefill_tiles(cu[: nb + 1], pctx[:nb])
        nlog = len(logit_rows)
        lidx = np.asarray(logit_rows, np.int32)
        # top-k / top-p ride in the same flat buffer (one H2D copy; pipeline stages get them too)
        if k:
            rest = sampling_rows(sampled[k:])
            temps, seeds, topk, topp = (np.concatenate([a, b]) for a, b in zip(dec_pre["samp"], rest[:4]))
            filt = dec_pre["filt"] or rest[4]
        else:
            temps, seeds, topk, topp, filt = sampling_rows(sampled, 0 if seed_ahead is None else seed_ahead)
        parts = [ids, pos, slots, dec_bt.ravel(), dec_ctx, pre_bt.ravel(), cu, pctx, tiles_np.ravel(), lidx,
                 temps, seeds, topk, topp]
        flat = np.concatenate(parts)
        max_ctx = int(dec_ctx.max()) if ndp else 1
        if self.is_cuda and ndp:
            splits, part = ops.decode_split_plan(ndp, max_ctx, self.model.cfg.num_kv_heads, self.num_cus)
        else:
            splits, part = 1, 1 << 20
        hdr = np.zeros(self.HEADER_SIZE, np.int64)
        hdr[[self.H_LEN, self.H_T, self.H_NDP, self.H_NPRE, self.H_NB, self.H_MAXW, self.H_SPLITS, self.H_PART,
             self.H_NTILES, self.H_NLOG, self.H_STEP, self.H_FILT]] = [flat.size, T, ndp, npre, nb, maxw, splits,
                                                                      part, len(tiles_np), nlog, self.step_id, int(filt)]
        return flat, hdr, sampled

    def meta_from_device(self, dev: torch.Tensor, hdr):
        """Views of the device copy of ``flat`` -> (input ids, AttnMeta, SamplingMeta)."""
        h = [int(x) for x in hdr]
        T, ndp, npre, nb, maxw = h[self.H_T], h[self.H_NDP], h[self.H_NPRE], h[self.H_NB], h[self.H_MAXW]
        ntiles, nlog = h[self.H_NTILES], h[self.H_NLOG]
        sizes = [T, T, T, ndp * maxw, ndp, nb * maxw, nb + 1, nb, ntiles * 2, nlog, nlog, nlog, nlog, nlog]
        views = []
        o = 0
        for sz in sizes:
            views.append(dev[o: o + sz])
            o += sz
        (d_ids, d_pos, d_slots, d_dbt, d_dctx, d_pbt, d_cu, d_pctx, d_tiles, d_lidx, d_temps, d_seeds,
         d_topk, d_topp) = views
        meta = AttnMeta(
            positions=d_pos, slot_mapping=d_slots, num_decode=ndp,
            dec_block_tables=d_dbt.view(ndp, maxw), dec_context_lens=d_dctx,
            dec_max_splits=h[self.H_SPLITS], dec_part_size=h[self.H_PART], dec_workspace=self.dec_ws,
            num_prefill_tokens=npre, pre_block_tables=d_pbt.view(nb, maxw), pre_cu_seqlens=d_cu,
            pre_context_lens=d_pctx, pre_tiles=d_tiles.view(-1, 2), logits_indices=d_lidx)
        samp = SamplingMeta(d_temps.view(torch.float32), d_seeds.long(),
                            d_topk.long() if h[self.H_FILT] else None,
                            d_topp.view(torch.float32) if h[self.H_FILT] else None)
        return d_ids, meta, samp

    def to_device(self, flat: np.ndarray) -> torch.Tensor:
        host = torch.from_numpy(flat)
        if self.is_cuda:
            host = host.pin_memory()
        return host.to(self.device, non_blocking=True)

    def build(self, sb: ScheduledBatch, pad_decode_to: int = 0):
        flat, hdr, sampled = self.build_host(sb, pad_decode_to)
        ids, meta, _samp = self.meta_from_device(self.to_device(flat), hdr)
        return ids, meta, sampled

    # ------------------------------------------------------------------ run
    def gate_rows(self, reqs, chunks=()) -> None:
        """Order this step's forward after the host-tier restores of the pages its rows read
        (``Request.kv_ready``: a GPU-side event wait, once per request; no host sync)."""
        if self.host_tier is None:
            return
        for r in itertools.chain(reqs, (c.req for c in chunks)):
            ev = r.kv_ready
            if ev is not None:
                r.kv_ready = None
                torch.cuda.current_stream(self.device).wait_event(ev)
                self.host_tier.stats["gates"] += 1

    @torch.inference_mode()
    def execute(self, sb: ScheduledBatch) -> StepResult:
        self.step_id += 1
        self.gate_rows(sb.decode, sb.prefill)
        if self.graphs is not None and not sb.prefill and sb.decode and \
                len(sb.decode) <= self.graphs.max_bucket:
            toks = self.graphs.run(sb)
            return StepResult(toks, list(sb.decode))
        flat, hdr, sampled = self.build_host(sb)
        ids, meta, samp = self.meta_from_device(self.to_device(flat), hdr)
        span = self._span_begin()
        logits = self.model.forward(meta, input_ids=ids)
        if not sampled:
            return StepResult([], [])
        toks = samp.sample(logits)
        self._span_end(span)
        return StepResult(self.fetch(toks), sampled)

    # DGI_GPU_SPAN=1: events around each eager step's device work (forward + sampling);
    # wall time minus the summed spans is the time the GPU waited for the host
    GPU_SPAN = os.environ.get("DGI_GPU_SPAN", "0") == "1"

    def _span_begin(self):
        if not (self.GPU_SPAN and self.is_cuda):
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def _span_end(self, e0) -> None:
        if e0 is None:
            return
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self._spans.append((e0, e1))
        if len(self._spans) > 64:
            self.gpu_span_ms()

    def gpu_span_ms(self) -> float:
        """Summed device time of the recorded eager steps so far (resolves pending events)."""
        for e0, e1 in self._spans:
            e1.synchronize()
            self.span_total_ms += e0.elapsed_time(e1)
        self._spans.clear()
        return self.span_total_ms

    def fetch(self, t: torch.Tensor, host: Optional[torch.Tensor] = None) -> list:
        """Device tokens -> host list.  With a ``wait_hook`` the copy is async and
        the hook runs until its event completes (no blocking synchronize)."""
        if not t.is_cuda:
            return t.tolist()
        if host is None:
            host = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        host.copy_(t, non_blocking=True)
        if self.wait_hook is None:
            torch.cuda.current_stream().synchronize()
        else:
            ev = torch.cuda.Event()
            ev.record()
            while not ev.query():
                self.wait_hook()
                time.sleep(0.00002)
        return host.tolist()


class GraphRunner:
    """hipGraph capture of the decode step (forward + sampling) per batch bucket."""

    def __init__(self, runner: ModelRunner, buckets):
        self.r = runner
        self.buckets = sorted(set(buckets))
        self.max_bucket = self.buckets[-1] if self.buckets else 0
        self.graphs: dict[int, torch.cuda.CUDAGraph] = {}
        # small buckets also get a one-split variant (8-wave workgroups walk each
        # sequence's whole context: no partials, no reduce kernel) replayed when
        # every context is short (DGI_DECODE_SHORT_CTX tokens, 0 = off; the one-split plan wins up to
        # ~700 tokens, the split plan from ~1k: profiles/r4_decode/attn8b_p16_1.jsonl)
        self.short_ctx = int(os.environ.get("DGI_DECODE_SHORT_CTX", "640"))
        self.short_max_b = int(os.environ.get("DGI_DECODE_SHORT_B", "8"))
        self.short_graphs: dict[int, torch.cuda.CUDAGraph] = {}
        self._short = False
        self.pool_handle = None
        dev = runner.device
        maxb = self.max_bucket
        maxw = runner.max_blocks
        # one int32 staging image per replay: ids | pos | slots | ctx | temps | seeds | topk | topp
        # (b entries each) | block tables (b x maxw).  The pinned host copy lands in ``dev_in``
        # with ONE H2D copy and each bucket's graph reads its inputs straight out of it (round 3
        # copied nine device views into separate static tensors: nine copy launches per step)
        self.NSEG = 8
        self.host_in2 = [torch.zeros(maxb * (self.NSEG + maxw), dtype=torch.int32).pin_memory() for _ in range(2)]
        self.host_out2 = [torch.zeros(maxb, dtype=torch.long).pin_memory() for _ in range(2)]
        self._flip = 0
        self.dev_in = torch.zeros(maxb * (self.NSEG + maxw), dtype=torch.int32, device=dev)
        self.out = torch.zeros(maxb, dtype=torch.long, device=dev)
        self.captured = False
        # optional EAGLE-3 feature tap captured with the step: (layer ids, fuse fn) -> [b, H] per bucket
        self.features = None
        self.feats_out: dict = {}

    def split_plan(self, b: int) -> tuple:
        """(max_splits, part_size) captured for bucket ``b``.  Dynamic (the
        default): the kernel splits each sequence's own context into up to
        ~4 workgroups per CU worth of parts of >= 64 tokens, so one graph serves
        every context length without idle splits; DGI_DECODE_DYNAMIC=0 keeps the
        fixed max_model_len / part_size plan."""
        r = self.r
        if os.environ.get("DGI_DECODE_DYNAMIC", "1") == "0":
            return r.graph_splits, r.graph_part
        nkv = r.model.cfg.num_kv_heads
        want = max(1, -(-4 * r.num_cus // max(1, b * nkv)))
        # minimum part: 128 tokens (one 32-token tile per wave) below batch 8, 64 above
        # (profiles/r2_fused_decode_bench.md: best or within 0.3 us at ctx 256-4096)
        mp = int(os.environ.get("DGI_DECODE_MIN_PART", "0")) or (128 if b < 8 else 64)
        return min(r.ws_splits, want), -mp

    def views(self, b: int) -> dict:
        """Bucket ``b``'s inputs: views into the staging image ``dev_in``."""
        S, d = self.NSEG, self.dev_in
        seg = d[: S * b].view(S, b)
        return {"ids": seg[0], "pos": seg[1], "slots": seg[2], "ctx": seg[3], "temps": seg[4].view(torch.float32),
                "seeds": seg[5], "topk": seg[6], "topp": seg[7].view(torch.float32),
                "bt": d[S * b: S * b + b * self.r.max_blocks].view(b, self.r.max_blocks)}

    def _meta(self, b):
        r = self.r
        v = self.views(b)
        splits, part = (1, 1 << 20) if self._short else self.split_plan(b)
        return AttnMeta(positions=v["pos"], slot_mapping=v["slots"], num_decode=b,
                        dec_block_tables=v["bt"], dec_context_lens=v["ctx"],
                        dec_max_splits=splits, dec_part_size=part, dec_workspace=r.dec_ws,
                        num_prefill_tokens=0, logits_indices=None)

    def _body(self, b):
        m = self.r.model
        v = self.views(b)
        ids = v["ids"].long()
        if self.features is not None:
            layers, fuse = self.features
            m.capture_layers, m.captured = tuple(layers), {}
            try:
                logits = m.forward(self._meta(b), input_ids=ids)
                self.feats_out[(b, self._short)] = fuse(torch.cat([m.captured[li] for li in layers], dim=-1))
            finally:
                m.capture_layers, m.captured = (), {}
        else:
            logits = m.forward(self._meta(b), input_ids=ids)
        ops.sample(logits, v["temps"], v["seeds"].long(), 0, out=self.out[:b], top_k=v["topk"].long(),
                   top_p=v["topp"])

    @torch.inference_mode()
    def capture(self):
        if self.captured:
            return
        torch.cuda.synchronize()
        for b in reversed(self.buckets):
            # warm up once outside capture (allocator, hipBLASLt heuristics)
            self._body(b)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with graph_capture(g, pool=self.pool_handle):
                self._body(b)
            if self.pool_handle is None:
                self.pool_handle = g.pool()
            self.graphs[b] = g
            if self.short_ctx > 0 and b <= self.short_max_b and self.r.model.cfg.head_dim in (64, 128):
                self._short = True
                try:
                    self._body(b)
                    torch.cuda.synchronize()
                    gs = torch.cuda.CUDAGraph()
                    with graph_capture(gs, pool=self.pool_handle):
                        self._body(b)
                    self.short_graphs[b] = gs
                finally:
                    self._short = False
        torch.cuda.synchronize()
        self.captured = True

    def run(self, sb: ScheduledBatch) -> list:
        return self.collect(self.launch(sb.decode))

    def launch(self, dec: list, ahead: int = 0) -> tuple:
        """Enqueue one decode step of rows ``dec`` (H2D of the packed inputs, graph replay,
        async D2H of the sampled tokens) without waiting for it; ``collect`` returns its
        tokens.  ``ahead=1``: every row has one token in flight from the previous launch
        (decode lookahead) — positions move on by one and the input tokens are that
        launch's sampled tokens, copied on the device in stream order.  Staging buffers
        alternate, so a launch never rewrites the host buffers of the one before it."""
        if not self.captured:
            self.capture()
        self.r.gate_rows(dec)
        n = len(dec)
        b = next(x for x in self.buckets if x >= n)
        r = self.r
        bs = r.bs
        maxw = r.max_blocks
        S = self.NSEG
        self._flip ^= 1
        host_in, host_out = self.host_in2[self._flip], self.host_out2[self._flip]
        h = host_in.numpy()
        seg = h[: S * b].reshape(S, b)
        ids, pos, slots, ctx = seg[0], seg[1], seg[2], seg[3]
        temps, seeds, topk = seg[4].view(np.float32), seg[5], seg[6]
        topp = seg[7].view(np.float32)
        bt = h[S * b: S * b + b * maxw].reshape(b, maxw)
        seg[:] = 0
        ctx[:] = 1
        topp[:] = 1.0
        bt[:] = 0
        ids[:n], pos[:n], slots[:n], ctx[:n] = decode_rows(dec, bs, bt, ahead)
        tb, seeds[:n], topk[:n], pb, _f = sampling_rows(dec, ahead)
        temps[:n] = tb.view(np.float32)
        topp[:n] = pb.view(np.float32)
        max_ctx = int(ctx[:n].max()) if n else 0
        k = S * b + b * maxw
        self.dev_in[:k].copy_(host_in[:k], non_blocking=True)
        if ahead:
            self.dev_in[:n].copy_(self.out[:n])        # the previous launch's tokens (same rows, same order)
        gs = self.short_graphs.get(b)
        short = gs is not None and max_ctx <= self.short_ctx
        (gs if short else self.graphs[b]).replay()
        self.last_bucket = b
        self.last_key = (b, short)
        host_out[:n].copy_(self.out[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return (ev, host_out, n)

    def collect(self, handle: tuple) -> list:
        ev, host_out, n = handle
        wh = self.r.wait_hook
        if wh is None:
            ev.synchronize()
        else:
            while not ev.query():
                wh()
                time.sleep(0.00002)
        return host_out[:n].tolist()

    def last_features(self, n: int) -> torch.Tensor:
        """Fused EAGLE-3 features of the last replay's first ``n`` rows (feature tap on)."""
        return self.feats_out[self.last_key][:n]
