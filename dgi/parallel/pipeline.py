"""In-node layer pipeline over RCCL p2p (SURVEY §2.10 "Pipeline parallelism").

The reference chains stages with sequential HTTP/JSON hops, keeps no KV on
the shards and has one stage busy at a time (worker/distributed/session.py:
271-337, grpc_server.py:351-388).  Here S stages on S GPUs form a chain:

    driver (stage 0, scheduler + block tables + layers [0, l1))
      --[header + step metadata: shm ring | hidden: RCCL pp communicator]--> stage 1 --> ... --> stage S-1
      <------------------- sampled token ids (shm ring, async D2H) -----------------------------'

* every stage keeps the paged KV of its own layers; block ids are chosen by
  the driver's scheduler and are valid in every stage's pool (all pools have
  the same block count, agreed at start-up);
* up to S microbatches (disjoint request sets) are in flight, so all GPUs
  work concurrently (``busy`` requests are skipped by the scheduler);
* only the bf16 residual stream [T, H] moves over RCCL (8192 * 2 B = 16 KiB
  per token on 70B), on the replica's own sub-communicator (``Fabric.
  setup_layout``): activations never share an RCCL stream with KV migrations;
* the step header + packed int32 metadata travel on the node-local
  shared-memory control plane and every stage does its own pinned H2D copy,
  so a stage reads the next hop's shape without touching its GPU;
* the last stage copies sampled tokens to pinned memory asynchronously and
  publishes them when the copy's event completes — no host sync in the stage
  loop; the driver's wait for them keeps servicing its KV handshakes
  (``idle_hook``);
* P/D migrations into a decode pipeline: the driver sends each later stage the
  page ids of an announced migration directly (``send_kv_notice``); the stage
  receives its own layer slice from the prefill rank (``KVReceiver``), installs
  it as soon as it lands — whatever microbatch is flowing — and reports LANDED
  back to the driver (``poll_landed``).  The driver admits the migration's
  requests only once every stage has reported, so the first hop that reads
  those pages follows the install on each stage's stream, and no stage ever
  blocks a microbatch on a migration it does not contain (round 3 installed
  every announced migration before every hop: a decode pipeline stalled for up
  to a prefill step whenever any migration was in flight).
"""
from __future__ import annotations

import collections
import os
import time
from typing import Optional

import numpy as np
import torch

from dgi.engine import EngineConfig, LLMEngine, StepOutput
from dgi.models.config import ModelConfig, get_config
from dgi.models.llama import LlamaModel
from dgi.kv.block_pool import BlockPool, OutOfBlocks, num_blocks_for_budget
from dgi.parallel.fabric import Fabric
from dgi.parallel.plan import plan_layer_split
from dgi import ops
from dgi.runtime.batch import AttnMeta
from dgi.runtime.model_runner import DEFAULT_BUCKETS, ModelRunner, graph_capture
from dgi.sched.request import Status
from dgi.utils.trace import mark, phase

KIND_STOP, KIND_FWD, KIND_KV, KIND_PAUSE = 0, 1, 2, 3
HDR = ModelRunner.HEADER_SIZE
# the pipeline driver builds a microbatch's next step while its tokens are in flight and
# relaunches it as soon as they land (PipelineEngine._retire); DGI_PP_PREBUILD=0: rebuild after
PREBUILD = os.environ.get("DGI_PP_PREBUILD", "1") == "1"


def pipeline_buckets(mb_cap: int) -> tuple:
    """Decode microbatch sizes captured as stage graphs: the engine defaults
    plus every multiple of 64 up to the microbatch cap (70B decode pipelines
    run 768-row microbatches).  With two-batch overlap on (``llama.TBO``) the
    microbatches it takes (>= ``TBO_MIN_ROWS`` rows) run eagerly on the CU-masked
    streams instead: a captured graph would drop the masks."""
    from dgi.models import llama
    top = mb_cap
    if llama.TBO:
        top = min(mb_cap, max(1, llama.TBO_MIN_ROWS - 1))
    b = set(x for x in DEFAULT_BUCKETS if x <= top)
    b.update(range(576, top + 1, 64))
    b.add(top)
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


def hop_ring_bytes(mb_cap: int, max_tokens: int, max_blocks: int) -> int:
    """Capacity of a stage's hop ring: room for two of the largest hop messages
    (``ModelRunner.build_host``: header + packed int32 metadata, whose dense block
    tables grow with rows x max_model_len / page), rounded up to a power of two —
    a 512-row microbatch at a 32k context needs ~17 MiB, more than a fixed ring
    held."""
    T = max(mb_cap, max_tokens) + mb_cap            # decode rows (bucket-padded) + prefill tokens
    nb = mb_cap                                     # prefill chunks
    nlog = mb_cap + nb
    ntiles = T // max(1, ops.PREFILL_TILE) + nb
    words = 3 * T + (mb_cap + nb) * max_blocks + mb_cap + (nb + 1) + nb + 2 * ntiles + 5 * nlog
    need = 2 * (HDR * 8 + 4 * words) + 4096
    cap = 1 << 20
    while cap < need:
        cap <<= 1
    return cap


def stage_split(mc: ModelConfig, stages: int) -> list[tuple[int, int]]:
    # embedding gather is cheap; the LM head GEMM is ~1.9 layers of 70B decode weight traffic
    head = (mc.vocab_size * mc.hidden_size) / max(1, (mc.qkv_size + mc.q_size + 3 * mc.intermediate_size) * mc.hidden_size)
    return plan_layer_split(mc.num_layers, stages, 1.0, 0.0, head)


def _pack(hdr, kind: int, flat: Optional[np.ndarray] = None) -> bytes:
    """Control-plane message of one hop: int64 header (kind in word 0) + int32 metadata."""
    h = np.array(hdr, dtype=np.int64, copy=True)
    h[0] = kind
    return h.tobytes() + (b"" if flat is None else np.ascontiguousarray(flat, np.int32).tobytes())


def _unpack(b: bytes):
    hdr = np.frombuffer(b, dtype=np.int64, count=HDR)
    flat = np.frombuffer(b, dtype=np.int32, offset=HDR * 8) if len(b) > HDR * 8 else None
    return hdr, flat


def agree_num_blocks(fabric: Fabric, ranks: list, mine: int) -> int:
    """All stages of a pipeline use the minimum of their block budgets (host
    control plane: no RCCL traffic before the communicators are warm)."""
    if len(ranks) == 1:
        return mine
    from dgi.parallel.fabric import CtrlChannel
    me = ranks.index(fabric.rank)
    if me == 0:
        chans = [CtrlChannel(fabric, r, 1, tag="agree") for r in ranks[1:]]
        best = min([mine] + [int(c.wait()[0]) for c in chans])
        for c in chans:
            c.send([best])
        return best
    c = CtrlChannel(fabric, ranks[0], 1, tag="agree")
    c.send([mine])
    return int(c.wait()[0])


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
                 model_cfg: Optional[ModelConfig] = None, split: Optional[list] = None,
                 kv_sources: Optional[list] = None):
        from dgi.parallel.fabric import CtrlChannel
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
        self.pp = fabric.pp_group(self.ranks)
        # control plane: hop headers to stage 1, tokens back from the last stage,
        # KV-migration notices straight to every later stage
        ring = hop_ring_bytes(self.mb_cap, cfg.max_num_batched_tokens, self.runner.max_blocks)
        self.hop = CtrlChannel(fabric, self.next_rank, HDR, tag="pp", capacity=ring) if self.next_rank is not None \
            else None
        self.tok = CtrlChannel(fabric, self.last_rank, 1, tag="tok") if self.next_rank is not None else None
        self.notice = {r: CtrlChannel(fabric, r, 1, tag="kvn") for r in self.ranks[1:]} if kv_sources else {}
        # stage -> driver: (src, key) of every migration slice a stage has installed
        self.landed_in = {r: CtrlChannel(fabric, r, 2, tag="kvl") for r in self.ranks[1:]} if kv_sources else {}
        self.stage_landed: collections.Counter = collections.Counter()
        self.idle_hook = None       # called while waiting for a microbatch's tokens (P/D: KV handshakes)
        self.wait_s = 0.0
        self.relaunches = 0         # microbatches launched from metadata built ahead (_retire)
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
    def _launch(self, pre: Optional[dict] = None, pre_ids=None) -> bool:
        """Schedule and launch one microbatch.  ``pre`` (``ModelRunner.prebuild_decode``):
        rows whose metadata was built while their previous microbatch was in flight (input
        tokens ``pre_ids``); they lead the microbatch and the scheduler adds whatever else is
        ready (admitted migrations, prefill chunks) up to the microbatch's size."""
        from dgi.parallel.fault import plan
        if plan():
            plan().check(self.f.rank, self.stats["steps"])
        k = len(pre["rows"]) if pre is not None else 0
        budget = max(1, self.cfg.max_num_batched_tokens // self.n_mb)
        if k:
            for r in pre["rows"]:
                r.busy = True
            extra = self.scheduler.schedule(max_seqs=max(0, self.mb_cap - k), max_tokens=max(0, budget - k)) \
                if k < self.mb_cap and budget > k else None
            from dgi.sched.scheduler import ScheduledBatch
            sb = ScheduledBatch(list(pre["rows"]) + (extra.decode if extra else []),
                                extra.prefill if extra else [], extra.preempted if extra else [])
        else:
            sb = self.scheduler.schedule(max_seqs=self.mb_cap, max_tokens=budget)
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
        flat, hdr, sampled = self.runner.build_host(sb, pad_decode_to=pad, dec_pre=pre if k else None,
                                                    pre_ids=pre_ids)
        # the next stage reads the hop from shared memory and copies it to its own GPU
        self.hop.send_bytes(_pack(hdr, KIND_FWD, flat))
        dev = self.runner.to_device(flat)
        with torch.inference_mode():
            if pad:
                # the graph's output buffer is rewritten by the next replay: send a copy
                hidden = g.run(dev, [int(x) for x in hdr]).clone()
            else:
                ids, meta, _samp = self.runner.meta_from_device(dev, hdr)
                hidden = self.model.forward(meta, input_ids=ids)
        self.f.send(hidden.contiguous(), self.next_rank, group=self.pp)
        self.inflight.append((sb, sampled, int(hdr[ModelRunner.H_NLOG])))
        return True

    def _prebuild(self, sb) -> Optional[dict]:
        """The next step of the oldest microbatch's decode rows, built while its tokens are
        in flight (positions + 1, the page of the next position grown): every row that
        continues after this token by length.  None when nothing qualifies or pages ran out."""
        if not PREBUILD or not sb.decode:
            return None
        cap = self.cfg.max_model_len - 1
        rows = [r for r in sb.decode if r.status is Status.RUNNING and len(r.output) + 1 < r.params.max_tokens
                and len(r.prompt) + len(r.output) + 1 < cap]
        if not rows:
            return None
        try:
            for r in rows:
                self.scheduler._grow(r, r.num_computed + 2)
        except OutOfBlocks:
            return None
        return self.runner.prebuild_decode(rows, ahead=1)

    def _retire(self) -> list[StepOutput]:
        """Collect the oldest microbatch's tokens.  While they are in flight the host builds
        that microbatch's next step (``_prebuild``); when they land, the next step is
        launched right away — before this one's tokens are applied — so the host work of a
        microbatch (scheduling, packing ~800 rows, applying their tokens: ~3-4 ms) no longer
        sits between two stage steps (the 3.3 ms host gaps per hop)."""
        sb, sampled, nlog = self.inflight.popleft()
        t0 = time.perf_counter()
        pre = None
        tried = False
        while True:
            m = self.tok.poll()
            if m is not None:
                break
            if not tried:
                tried = True
                pre = self._prebuild(sb)
                continue
            if self.idle_hook is not None:
                self.idle_hook()
            time.sleep(0.00005)
        self.wait_s += time.perf_counter() - t0
        tl = m[1: 1 + int(m[0])].tolist()
        assert len(tl) == nlog, (len(tl), nlog)
        if pre is None and not tried:
            pre = self._prebuild(sb)
        # rows that ended before this step ran (EOS at the previous token while this step was
        # already in flight, or aborted): their tokens are discarded
        keep = [i for i, r in enumerate(sampled) if r.status is Status.RUNNING]
        if len(keep) != len(sampled):
            dead = {id(r) for r in sampled if r.status is not Status.RUNNING}
            tl = [tl[i] for i in keep]
            sampled = [sampled[i] for i in keep]
            sb = type(sb)([r for r in sb.decode if id(r) not in dead], sb.prefill, sb.preempted)
        relaunched = set()
        if pre is not None and len(self.inflight) < self.n_mb:
            tok = {id(r): t for r, t in zip(sampled, tl)}
            eos = self.model_cfg.eos_token_id
            # a row this token stops (EOS / stop id) is not relaunched: its pages are freed when
            # the token is applied and must not be written by a step still in flight
            keep = np.fromiter((id(r) in tok and (r.params.ignore_eos or (tok[id(r)] != eos and tok[id(r)]
                                                                              not in r.params.stop_token_ids))
                                for r in pre["rows"]), bool, len(pre["rows"]))
            if keep.any():
                if not keep.all():
                    pre = self.runner.subset_prebuilt(pre, keep)
                rows = pre["rows"]
                ids = np.fromiter((tok[id(r)] for r in rows), np.int32, len(rows))
                relaunched = {id(r) for r in rows}
                with phase("pipeline_relaunch", rows=len(rows)):
                    self._launch(pre, ids)
                self.relaunches += 1
        for r in sb.decode:
            if id(r) not in relaunched:
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

    def drain(self) -> list[StepOutput]:
        outs = []
        while self.inflight:
            sb, sampled, nlog = self.inflight[0]
            # no relaunch while draining: every microbatch comes back, nothing new goes out
            global PREBUILD
            old, PREBUILD = PREBUILD, False
            try:
                outs += self._retire()
            finally:
                PREBUILD = old
        return outs

    def has_unfinished(self) -> bool:
        return bool(self.inflight) or self.scheduler.has_work()

    # ------------------------------------------------------------------ control
    def send_kv_notice(self, src: int, key: int, ids: list) -> None:
        """Tell every later stage that migration ``key`` from prefill rank ``src``
        lands in pages ``ids`` (each stage receives its own layer slice from
        ``src``).  Sent before any micro-step that reads those pages."""
        msg = [src, key] + [int(x) for x in ids]
        for ch in self.notice.values():
            ch.send_var(msg)

    def poll_landed(self) -> None:
        """Take in the stages' LANDED reports."""
        for ch in self.landed_in.values():
            while True:
                m = ch.poll()
                if m is None:
                    break
                self.stage_landed[(int(m[0]), int(m[1]))] += 1

    def stages_landed(self, src: int, key: int) -> bool:
        """Every later stage has installed its slice of migration ``key`` from ``src``
        (its scatter is on the stage's stream ahead of any hop sent from now on)."""
        if not self.landed_in:
            return True
        k = (src, key)
        if self.stage_landed[k] >= len(self.landed_in):
            del self.stage_landed[k]
            return True
        return False

    def _ctl(self, kind: int) -> None:
        self.drain()
        if self.hop is not None:
            self.hop.send_bytes(_pack(np.zeros(HDR, np.int64), kind))

    def pause_stages(self) -> None:
        """Stage workers install every announced migration and return from ``run()``."""
        self._ctl(KIND_PAUSE)

    def stop_stages(self) -> None:
        self._ctl(KIND_STOP)


class StageWorker:
    """Stages 1..S-1: receive -> local layers -> forward (or sample on the last stage)."""

    def __init__(self, cfg: EngineConfig, fabric: Fabric, stage_ranks: list, model_cfg: Optional[ModelConfig] = None,
                 split: Optional[list] = None, microbatches: Optional[int] = None,
                 kv_sources: Optional[list] = None):
        from dgi.parallel.fabric import CtrlChannel
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
        self.pp = fabric.pp_group(self.ranks)
        ring = hop_ring_bytes(self.mb_cap, cfg.max_num_batched_tokens, self.runner.max_blocks)
        self.hop_in = CtrlChannel(fabric, self.prev, HDR, tag="pp")
        self.hop_out = CtrlChannel(fabric, self.next, HDR, tag="pp", capacity=ring) if self.next is not None \
            else None
        self.tok = CtrlChannel(fabric, self.driver, 1, tag="tok") if self.is_last else None
        self.tok_pending: collections.deque = collections.deque()   # (event, pinned tokens, n) in order
        # P/D: page-id notices from the driver, slices from the prefill ranks
        self.kvr = None
        self.notice = None
        self.kv_pending: list = []                                  # [src, key, ids_t] not installed yet
        self.landed_out = None
        if kv_sources:
            from dgi.parallel.kv_transfer import KVReceiver
            self.notice = CtrlChannel(fabric, self.driver, 1, tag="kvn")
            self.landed_out = CtrlChannel(fabric, self.driver, 2, tag="kvl")
            self.kvr = KVReceiver(fabric, kv_sources, (2, mc.num_kv_heads, cfg.block_size, mc.head_dim), cfg.dtype)
        self.installed = 0
        self.on_hop = None             # called after every forwarded hop (bench phase clock)
        self.kv_block_s = 0.0          # host time a stage spent blocked on KV (only at PAUSE / STOP)
        self.sgraphs = None
        if cfg.use_graphs and dev.type == "cuda":
            self.sgraphs = StageGraphs(self.model, self.runner, pipeline_buckets(self.mb_cap), first=False,
                                       last=self.is_last)
            self.capture_seconds = self.sgraphs.capture()

    # ------------------------------------------------------------------ P/D installs
    def _take_notices(self) -> None:
        if self.notice is None:
            return
        while True:
            m = self.notice.poll()
            if m is None:
                return
            ids_t = torch.tensor(m[2:], dtype=torch.int32, device=self.f.device)
            self.kv_pending.append((int(m[0]), int(m[1]), ids_t))

    def _service(self) -> None:
        """Everything a stage does between hops and while it waits: KV handshakes,
        notices, token publication, and installing every migration whose slice
        has landed (in landing order, not announcement order: slices from
        different prefill ranks land independently)."""
        self._take_notices()
        if self.kvr is not None:
            self.kvr.service()
            if self.kv_pending:
                keep = []
                for item in self.kv_pending:
                    if self.n_layers == 0 or self.kvr.is_landed(item[0], item[1]):
                        self._install(item, block=False)
                    else:
                        keep.append(item)
                self.kv_pending = keep
        self._publish_tokens()

    def _install(self, item, block: bool) -> None:
        from dgi.parallel.kv_transfer import scatter_groups
        src, key, ids_t = item
        if self.n_layers:               # a layer-less stage (more stages than layers) is sent nothing
            if block:
                t0 = time.perf_counter()
                groups = self.kvr.wait_landed(src, key, idle=self._publish_tokens)
                self.kv_block_s += time.perf_counter() - t0
            else:
                groups = self.kvr.take(src, key)
            scatter_groups(self.pool.kv, ids_t, groups, self.kvr.digests, src, key)
            self.installed += 1
        # the driver admits the migration's requests once every stage has reported
        self.landed_out.send([src, key])

    def _install_all(self) -> None:
        """Phase boundary (PAUSE / STOP): every announced migration is installed.
        The driver quiesces migrations before pausing, so this normally finds
        nothing to wait for."""
        self._take_notices()
        while self.kv_pending:
            self._install(self.kv_pending.pop(0), block=True)

    # ------------------------------------------------------------------ tokens (last stage)
    def _publish_tokens(self, block: bool = False) -> None:
        while self.tok_pending:
            ev, host, n = self.tok_pending[0]
            if ev is not None and not ev.query():
                if not block:
                    return
                ev.synchronize()
            self.tok_pending.popleft()
            self.tok.send_var(np.concatenate([[n], host[:n].numpy()]) if n else [0])

    def _emit_tokens(self, out: torch.Tensor, nlog: int) -> None:
        if not nlog:
            self.tok_pending.append((None, None, 0))
            return
        if out.is_cuda:
            host = torch.empty(nlog, dtype=torch.long, pin_memory=True)
            host.copy_(out[:nlog], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host, ev = out[:nlog].clone(), None
        self.tok_pending.append((ev, host, nlog))

    # ------------------------------------------------------------------ serve
    def _next_hop(self) -> bytes:
        while True:
            b = self.hop_in.poll_bytes()
            if b is not None:
                return b
            self._service()
            time.sleep(0.00005)

    @torch.inference_mode()
    def run(self) -> str:
        """Serve until PAUSE (returns "pause") or STOP (returns "stop")."""
        f, dev = self.f, self.f.device
        H = self.mc.hidden_size
        while True:
            b = self._next_hop()
            hdr, flat_np = _unpack(b)
            kind = int(hdr[0])
            if kind in (KIND_STOP, KIND_PAUSE):
                self._install_all()
                self._publish_tokens(block=True)
                if self.hop_out is not None:
                    self.hop_out.send_bytes(b)
                return "stop" if kind == KIND_STOP else "pause"
            # KIND_FWD
            from dgi.parallel.fault import plan
            if plan():
                plan().check(f.rank, self.steps)
            # installs whatever has landed; never waits (a hop only carries requests the
            # driver admitted after every stage reported their pages installed)
            self._service()
            h = [int(x) for x in hdr]
            if self.hop_out is not None:           # the next stage can post its receive now
                self.hop_out.send_bytes(b)
            flat = self.runner.to_device(flat_np.copy())
            T = h[ModelRunner.H_T]
            g = self.sgraphs
            use_graph = g is not None and g.eligible(h)
            hidden = g.input_hidden(T) if use_graph else torch.empty(T, H, dtype=self.pool.dtype, device=dev)
            f.recv(hidden, self.prev, group=self.pp)
            with phase("stage_forward", rows=T, graph=int(use_graph)):
                if use_graph:
                    out = g.run(flat, h)
                    if not self.is_last:
                        out = out.clone()      # the next replay rewrites the graph's output buffer
                else:
                    _ids, meta, samp = self.runner.meta_from_device(flat, h)
                    out = self.model.forward(meta, hidden=hidden)
                    if self.is_last and h[ModelRunner.H_NLOG]:
                        out = samp.sample(out)
            self.steps += 1
            if self.is_last:
                self._emit_tokens(out, h[ModelRunner.H_NLOG])
                self._publish_tokens()
            else:
                f.send(out.contiguous(), self.next, group=self.pp)
            if self.on_hop is not None:
                self.on_hop()
