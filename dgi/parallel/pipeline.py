"""In-node layer pipeline over RCCL p2p (SURVEY §2.10 "Pipeline parallelism").

The reference chains stages with sequential HTTP/JSON hops, keeps no KV on
the shards and has one stage busy at a time (worker/distributed/session.py:
271-337, grpc_server.py:351-388).  Here S stages on S GPUs form an ordered
RCCL channel ring:

    driver (stage 0, scheduler + block tables + layers [0, l1))
      --[header | step metadata | hidden]--> stage 1 --> ... --> stage S-1
      <--------------------- sampled token ids ------------------------'

* every stage keeps the paged KV of its own layers; block ids are chosen by
  the driver's scheduler and are valid in every stage's pool (all pools have
  the same block count, agreed at start-up);
* up to S microbatches (disjoint request sets) are in flight, so all GPUs
  work concurrently (``busy`` requests are skipped by the scheduler);
* activations travel as ONE bf16 residual-stream tensor [T, H] per hop
  (8192 * 2 B = 16 KiB per token on 70B);
* the same channel carries KV-install messages (P/D migration into a decode
  pipeline) and PAUSE/STOP control, so ordering is never ambiguous.
"""
from __future__ import annotations

import collections
import time
from typing import Optional

import numpy as np
import torch

from dgi.engine import EngineConfig, LLMEngine, StepOutput
from dgi.models.config import ModelConfig, get_config
from dgi.models.llama import LlamaModel
from dgi.kv.block_pool import BlockPool, num_blocks_for_budget
from dgi.parallel.fabric import Fabric
from dgi.parallel.plan import plan_layer_split
from dgi import ops
from dgi.runtime.batch import AttnMeta
from dgi.runtime.model_runner import DEFAULT_BUCKETS, ModelRunner, graph_capture
from dgi.utils.trace import mark, phase

KIND_STOP, KIND_FWD, KIND_KV, KIND_PAUSE = 0, 1, 2, 3
HDR = ModelRunner.HEADER_SIZE


def pipeline_buckets(mb_cap: int) -> tuple:
    """Decode microbatch sizes captured as stage graphs: the engine defaults
    plus every multiple of 64 up to the microbatch cap (70B decode pipelines
    run 768-row microbatches)."""
    b = set(x for x in DEFAULT_BUCKETS if x <= mb_cap)
    b.update(range(576, mb_cap + 1, 64))
    b.add(mb_cap)
    return tuple(sorted(b))


class StageGraphs:
    """hipGraph capture of one pipeline stage's decode micro-step per bucket.

    Decode-only microbatches are padded by the driver to a bucket size (pad
    rows write into reserved block 0 and read it back), so every stage sees
    exactly ``b`` rows.  A replay copies the received step buffer's views
    into static tensors (a handful of KB-sized device copies), receives the
    hidden rows straight into the static input, and replays the stage's
    layers — plus, on the last stage, the LM head and the top-k/top-p
    sampler — with no host work per kernel."""

    def __init__(self, model: LlamaModel, runner: ModelRunner, buckets, first: bool, last: bool):
        self.model, self.r = model, runner
        self.first, self.last = first, last
        self.buckets = tuple(sorted(set(buckets)))
        self.max_bucket = self.buckets[-1]
        dev, maxb, maxw = runner.device, self.max_bucket, runner.max_blocks
        H = model.cfg.hidden_size
        self.ids = torch.zeros(maxb, dtype=torch.long, device=dev)
        self.hidden = torch.zeros(maxb, H, dtype=model.dtype, device=dev)
        self.pos = torch.zeros(maxb, dtype=torch.int32, device=dev)
        self.slots = torch.zeros(maxb, dtype=torch.int32, device=dev)
        self.bt = torch.zeros(maxb, maxw, dtype=torch.int32, device=dev)
        self.ctx = torch.ones(maxb, dtype=torch.int32, device=dev)
        self.temps = torch.zeros(maxb, dtype=torch.float32, device=dev)
        self.seeds = torch.zeros(maxb, dtype=torch.long, device=dev)
        self.topk = torch.zeros(maxb, dtype=torch.long, device=dev)
        self.topp = torch.ones(maxb, dtype=torch.float32, device=dev)
        self.tok = torch.zeros(maxb, dtype=torch.long, device=dev)
        self.graphs: dict = {}
        self.outs: dict = {}
        self.pool = None
        self.replays = 0

    def _meta(self, b: int) -> AttnMeta:
        r = self.r
        return AttnMeta(positions=self.pos[:b], slot_mapping=self.slots[:b], num_decode=b,
                        dec_block_tables=self.bt[:b], dec_context_lens=self.ctx[:b],
                        dec_max_splits=r.graph_splits, dec_part_size=r.graph_part, dec_workspace=r.dec_ws,
                        num_prefill_tokens=0, logits_indices=None)

    def _body(self, b: int):
        if self.first:
            out = self.model.forward(self._meta(b), input_ids=self.ids[:b])
        else:
            out = self.model.forward(self._meta(b), hidden=self.hidden[:b])
        if self.last:
            ops.sample(out, self.temps[:b], self.seeds[:b], 0, out=self.tok[:b], top_k=self.topk[:b],
                       top_p=self.topp[:b])
            return self.tok[:b]
        return out

    @torch.inference_mode()
    def capture(self) -> float:
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        mlp_pad, self.model.mlp_pad = self.model.mlp_pad, None   # fixed shapes inside graphs
        try:
            for b in reversed(self.buckets):
                self._body(b)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with graph_capture(g, pool=self.pool):
                    out = self._body(b)
                if self.pool is None:
                    self.pool = g.pool()
                self.graphs[b] = g
                self.outs[b] = out
        finally:
            self.model.mlp_pad = mlp_pad
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    def eligible(self, hdr) -> bool:
        return hdr[ModelRunner.H_NPRE] == 0 and hdr[ModelRunner.H_T] in self.graphs

    def input_hidden(self, T: int) -> torch.Tensor:
        """Where a later stage receives the previous stage's rows for a replay."""
        return self.hidden[:T]

    def run(self, flat: torch.Tensor, hdr) -> torch.Tensor:
        """Replay for a decode-only step buffer ``flat`` of T = bucket rows."""
        b = hdr[ModelRunner.H_T]
        maxw = hdr[ModelRunner.H_MAXW]
        assert maxw == self.r.max_blocks
        o = 0
        views = []
        for sz in (b, b, b, b * maxw, b):
            views.append(flat[o: o + sz])
            o += sz
        ids, pos, slots, bt, ctx = views
        if self.first:
            self.ids[:b].copy_(ids)
        self.pos[:b].copy_(pos)
        self.slots[:b].copy_(slots)
        self.bt[:b].copy_(bt.view(b, maxw))
        self.ctx[:b].copy_(ctx)
        if self.last:
            # [.. | pre_bt(0) | cu(1) | pctx(0) | tiles(0) | lidx(n) | temps(n) | seeds(n) | topk(n) | topp(n)]
            n = hdr[ModelRunner.H_NLOG]
            o += 1 + n
            seg = flat[o: o + 4 * n].view(4, n)
            self.temps[:n].copy_(seg[0].view(torch.float32))
            self.seeds[:n].copy_(seg[1])
            self.topk[:n].copy_(seg[2])
            self.topp[:n].copy_(seg[3].view(torch.float32))
            if n < b:   # pad rows: greedy, unfiltered
                self.temps[n:b].zero_()
                self.topk[n:b].zero_()
                self.topp[n:b].fill_(1.0)
        self.graphs[b].replay()
        self.replays += 1
        return self.outs[b]


def stage_split(mc: ModelConfig, stages: int) -> list[tuple[int, int]]:
    # embedding gather is cheap; the LM head GEMM is ~1.9 layers of 70B decode weight traffic
    head = (mc.vocab_size * mc.hidden_size) / max(1, (mc.qkv_size + mc.q_size + 3 * mc.intermediate_size) * mc.hidden_size)
    return plan_layer_split(mc.num_layers, stages, 1.0, 0.0, head)


def _hdr_tensor(hdr: np.ndarray, kind: int) -> torch.Tensor:
    """Step header as a HOST tensor: headers travel on the gloo control group,
    so a stage reads the shape of the next hop without synchronising its GPU
    (its host runs ahead and enqueues the next receive + forward while the
    current one still computes)."""
    h = np.array(hdr, dtype=np.int64, copy=True)
    h[0] = kind
    return torch.from_numpy(h)


def agree_num_blocks(fabric: Fabric, ranks: list, mine: int) -> int:
    """All stages of a pipeline use the minimum of their block budgets."""
    if len(ranks) == 1:
        return mine
    me = ranks.index(fabric.rank)
    t = torch.tensor([mine], dtype=torch.int64, device=fabric.device)
    if me == 0:
        best = mine
        for r in ranks[1:]:
            fabric.recv(t, r)
            best = min(best, int(t.item()))
        out = torch.tensor([best], dtype=torch.int64, device=fabric.device)
        for r in ranks[1:]:
            fabric.send(out.clone(), r)
        fabric.flush()
        return best
    fabric.send(t, ranks[0])
    fabric.flush()
    fabric.recv(t, ranks[0])
    return int(t.item())


def stage_block_budget(mc: ModelConfig, device: torch.device, n_layers: int, cfg: EngineConfig) -> int:
    if device.type != "cuda":
        return cfg.num_blocks or num_blocks_for_budget(1 << 30, max(1, n_layers), mc.num_kv_heads, mc.head_dim,
                                                       cfg.block_size)
    free, _ = torch.cuda.mem_get_info(device)
    budget = max(0, free - cfg.workspace_bytes) * cfg.kv_fraction
    n = num_blocks_for_budget(int(budget), max(1, n_layers), mc.num_kv_heads, mc.head_dim, cfg.block_size)
    cap = 4 * cfg.max_num_seqs * ((cfg.max_model_len + cfg.block_size - 1) // cfg.block_size) + 1
    if cfg.num_blocks is not None:
        n = min(n, cfg.num_blocks)
    return max(2, min(n, cap))


class PipelineEngine(LLMEngine):
    """Stage 0 of an S-stage pipeline; same API as ``LLMEngine``."""

    def __init__(self, cfg: EngineConfig, fabric: Fabric, stage_ranks: list, microbatches: Optional[int] = None,
                 model_cfg: Optional[ModelConfig] = None, split: Optional[list] = None):
        self.f = fabric
        self.ranks = list(stage_ranks)
        assert self.ranks[0] == fabric.rank
        from dgi.models.weights import resolve_checkpoint
        ckpt = resolve_checkpoint(cfg.model, cfg.model_path)
        mc = model_cfg or get_config(ckpt or cfg.model)
        mc.max_position = max(mc.max_position, cfg.max_model_len)
        self.split = split or stage_split(mc, len(self.ranks))
        a, b = self.split[0]
        device = fabric.device
        model = LlamaModel(mc, device, cfg.dtype, a, b, has_embed=True, has_head=len(self.ranks) == 1, seed=cfg.seed,
                           checkpoint=ckpt)
        nb = stage_block_budget(mc, device, b - a, cfg)
        nb = agree_num_blocks(fabric, self.ranks, nb)
        pcfg = EngineConfig(**{**cfg.__dict__, "device": str(device), "layer_start": a, "layer_end": b,
                               "num_blocks": nb, "use_graphs": False})
        super().__init__(pcfg, model_cfg=mc, model=model)
        self.n_mb = microbatches or len(self.ranks)
        self.mb_cap = max(1, cfg.max_num_seqs // self.n_mb)
        self.inflight: collections.deque = collections.deque()
        self.next_rank = self.ranks[1] if len(self.ranks) > 1 else None
        self.last_rank = self.ranks[-1]
        # decode micro-steps of this stage replay hipGraphs (same buckets on every stage)
        self.sgraphs = None
        if cfg.use_graphs and device.type == "cuda" and len(self.ranks) > 1:
            self.sgraphs = StageGraphs(self.model, self.runner, pipeline_buckets(self.mb_cap), first=True,
                                       last=False)
            self.capture_seconds = self.sgraphs.capture()

    def warmup(self) -> None:
        if self.sgraphs is None:
            super().warmup()

    # ------------------------------------------------------------------ microbatches
    def _launch(self) -> bool:
        from dgi.parallel.fault import plan
        if plan():
            plan().check(self.f.rank, self.stats["steps"])
        sb = self.scheduler.schedule(max_seqs=self.mb_cap,
                                     max_tokens=max(1, self.cfg.max_num_batched_tokens // self.n_mb))
        if sb.empty:
            return False
        for r in sb.decode:
            r.busy = True
        for c in sb.prefill:
            c.req.busy = True
        self.runner.step_id += 1
        pad = 0
        g = self.sgraphs
        if g is not None and not sb.prefill and len(sb.decode) <= g.max_bucket:
            pad = next(b for b in g.buckets if b >= len(sb.decode))
        flat, hdr, sampled = self.runner.build_host(sb, pad_decode_to=pad)
        dev = self.runner.to_device(flat)
        with torch.inference_mode():
            if pad:
                # the graph's output buffer is rewritten by the next replay: send a copy
                hidden = g.run(dev, [int(x) for x in hdr]).clone()
            else:
                ids, meta, _samp = self.runner.meta_from_device(dev, hdr)
                hidden = self.model.forward(meta, input_ids=ids)
        self.f.ctrl_send_tensor(_hdr_tensor(hdr, KIND_FWD), self.next_rank)
        self.f.send(dev, self.next_rank)
        self.f.send(hidden.contiguous(), self.next_rank)
        self.inflight.append((sb, sampled, int(hdr[ModelRunner.H_NLOG])))
        return True

    def _retire(self) -> list[StepOutput]:
        sb, sampled, nlog = self.inflight.popleft()
        # tokens come back on the gloo control group: an RCCL recv here would
        # queue behind the next microbatch's sends on the (0,1) pair channel
        toks = torch.empty(self.mb_cap + 1, dtype=torch.long)
        self.f.ctrl_recv_tensor(toks, self.last_rank)
        tl = toks[1: 1 + int(toks[0])].tolist()
        assert len(tl) == nlog, (len(tl), nlog)
        for r in sb.decode:
            r.busy = False
        for c in sb.prefill:
            c.req.busy = False
        return self._apply(sb, sampled, tl)

    def step(self) -> list[StepOutput]:
        if len(self.ranks) == 1:
            return super().step()
        t0 = time.perf_counter()
        launched = False
        if len(self.inflight) < self.n_mb:
            launched = self._launch()
        outs: list[StepOutput] = []
        if self.inflight and (len(self.inflight) >= self.n_mb or not launched):
            outs = self._retire()
        self.stats["step_time"] += time.perf_counter() - t0
        return outs

    def has_unfinished(self) -> bool:
        return bool(self.inflight) or self.scheduler.has_work()

    def drain(self) -> list[StepOutput]:
        outs = []
        while self.inflight:
            outs += self._retire()
        return outs

    # ------------------------------------------------------------------ control
    def send_kv_notice(self, ids: torch.Tensor, src: int, chunk: int = 0) -> None:
        """Tell later stages that pages ``ids`` of a P/D migration are on their
        way from prefill rank ``src`` (each stage receives its own layer slice,
        in ``chunk``-layer groups when the migration is layer-streamed)."""
        if self.next_rank is None:
            return
        hdr = np.zeros(HDR, np.int64)
        hdr[1] = ids.numel()
        hdr[2] = src
        hdr[3] = chunk
        self.f.ctrl_send_tensor(_hdr_tensor(hdr, KIND_KV), self.next_rank)
        self.f.send(ids.to(self.f.device, torch.int32).contiguous(), self.next_rank)

    def pause_stages(self) -> None:
        """Stage workers return from ``run()`` (e.g. to join a barrier)."""
        self.drain()
        if self.next_rank is not None:
            self.f.ctrl_send_tensor(_hdr_tensor(np.zeros(HDR, np.int64), KIND_PAUSE), self.next_rank)
        self.f.flush()

    def stop_stages(self) -> None:
        self.drain()
        if self.next_rank is not None:
            self.f.ctrl_send_tensor(_hdr_tensor(np.zeros(HDR, np.int64), KIND_STOP), self.next_rank)
        self.f.flush()


class StageWorker:
    """Stages 1..S-1: receive -> local layers -> forward (or sample on the last stage)."""

    def _install_kv(self) -> None:
        """Scatter migrated page slices posted so far into the pool.  The driver
        announced them before any step that reads them, so ordering the
        compute stream after the scatter here is all the sync needed; the
        transfers themselves ran off the compute stream."""
        if not self.kv_pending:
            return
        from dgi import ops
        f = self.f
        if f.on_gpu:
            rs = f.recv_stream
            rs.wait_stream(torch.cuda.current_stream())
            for recs, buf, ids in self.kv_pending:
                for rec in recs:
                    rec.complete()
                with torch.cuda.stream(rs):
                    ops.kv_scatter(self.pool.kv, ids, buf)
                buf.record_stream(rs)
                ids.record_stream(rs)
            torch.cuda.current_stream().wait_stream(rs)
        else:
            for recs, buf, ids in self.kv_pending:
                for rec in recs:
                    rec.complete()
                ops.kv_scatter(self.pool.kv, ids, buf)
        self.kv_pending = []

    def __init__(self, cfg: EngineConfig, fabric: Fabric, stage_ranks: list, model_cfg: Optional[ModelConfig] = None,
                 split: Optional[list] = None, microbatches: Optional[int] = None):
        self.f = fabric
        self.mb_cap = max(1, cfg.max_num_seqs // (microbatches or len(stage_ranks)))
        self.ranks = list(stage_ranks)
        self.idx = self.ranks.index(fabric.rank)
        assert self.idx > 0
        from dgi.models.weights import resolve_checkpoint
        ckpt = resolve_checkpoint(cfg.model, cfg.model_path)
        mc = model_cfg or get_config(ckpt or cfg.model)
        mc.max_position = max(mc.max_position, cfg.max_model_len)
        self.mc = mc
        self.split = split or stage_split(mc, len(self.ranks))
        a, b = self.split[self.idx]
        self.is_last = self.idx == len(self.ranks) - 1
        self.prev = self.ranks[self.idx - 1]
        self.next = None if self.is_last else self.ranks[self.idx + 1]
        self.driver = self.ranks[0]
        dev = fabric.device
        self.model = LlamaModel(mc, dev, cfg.dtype, a, b, has_embed=False, has_head=self.is_last, seed=cfg.seed,
                                checkpoint=ckpt)
        nb = stage_block_budget(mc, dev, b - a, cfg)
        nb = agree_num_blocks(fabric, self.ranks, nb)
        self.pool = BlockPool(nb, cfg.block_size, b - a, mc.num_kv_heads, mc.head_dim, cfg.dtype, dev)
        self.runner = ModelRunner(self.model, self.pool, cfg.max_num_seqs, cfg.max_model_len,
                                  cfg.max_num_batched_tokens, use_graphs=False)
        self.model.kv_cache = self.pool.kv
        self.n_layers = b - a
        self.steps = 0
        self.kv_pending: list = []   # (AsyncRecv, buf, ids) of P/D page slices in flight
        self.sgraphs = None
        if cfg.use_graphs and dev.type == "cuda":
            self.sgraphs = StageGraphs(self.model, self.runner, pipeline_buckets(self.mb_cap), first=False,
                                       last=self.is_last)
            self.capture_seconds = self.sgraphs.capture()

    @torch.inference_mode()
    def run(self) -> str:
        """Serve until PAUSE (returns "pause") or STOP (returns "stop")."""
        f, dev = self.f, self.f.device
        H = self.mc.hidden_size
        from dgi import ops
        while True:
            hb = torch.empty(HDR, dtype=torch.int64)
            f.ctrl_recv_tensor(hb, self.prev)      # host tensor: no GPU sync to read the next hop's shape
            hdr = hb.tolist()
            kind = hdr[0]
            if kind in (KIND_STOP, KIND_PAUSE):
                self._install_kv()
                if self.next is not None:
                    f.ctrl_send_tensor(hb, self.next)
                f.flush()
                return "stop" if kind == KIND_STOP else "pause"
            if kind == KIND_KV:
                n, src, chunk = hdr[1], hdr[2], hdr[3]
                ids = torch.empty(n, dtype=torch.int32, device=dev)
                f.recv(ids, self.prev)
                if self.next is not None:
                    f.ctrl_send_tensor(hb, self.next)
                    f.send(ids, self.next)
                buf = torch.empty(self.n_layers, 2, n, self.mc.num_kv_heads, self.pool.block_size, self.mc.head_dim,
                                  dtype=self.pool.dtype, device=dev)
                from dgi.parallel.pd import layer_groups
                self.kv_pending.append(([f.irecv_async(buf[a:b], src) for a, b in layer_groups(self.n_layers, chunk)],
                                        buf, ids))
                continue
            # KIND_FWD
            from dgi.parallel.fault import plan
            if plan():
                plan().check(f.rank, self.steps)
            self._install_kv()
            flat = torch.empty(hdr[ModelRunner.H_LEN], dtype=torch.int32, device=dev)
            f.recv(flat, self.prev)
            T = hdr[ModelRunner.H_T]
            g = self.sgraphs
            use_graph = g is not None and g.eligible(hdr)
            hidden = g.input_hidden(T) if use_graph else torch.empty(T, H, dtype=self.pool.dtype, device=dev)
            f.recv(hidden, self.prev)
            with phase("stage_forward", rows=T, graph=int(use_graph)):
                if use_graph:
                    out = g.run(flat, hdr)
                    if not self.is_last:
                        out = out.clone()      # the next replay rewrites the graph's output buffer
                else:
                    _ids, meta, samp = self.runner.meta_from_device(flat, hdr)
                    out = self.model.forward(meta, hidden=hidden)
                    if self.is_last and hdr[ModelRunner.H_NLOG]:
                        out = samp.sample(out)
            self.steps += 1
            if self.is_last:
                nlog = hdr[ModelRunner.H_NLOG]
                toks = torch.zeros(self.mb_cap + 1, dtype=torch.long)
                toks[0] = nlog
                if nlog:
                    toks[1: 1 + nlog] = out[:nlog].cpu()
                f.ctrl_send_tensor(toks, self.driver)
            else:
                f.ctrl_send_tensor(hb, self.next)
                f.send(flat, self.next)
                f.send(out.contiguous(), self.next)
