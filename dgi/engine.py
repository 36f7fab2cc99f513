"""LLMEngine: the native MI355X serving engine (model + block pool + scheduler).

``LLMEngine.step()`` is one iteration of continuous batching: schedule ->
one model forward (decode rows + prefill chunks) -> sample -> update request
state.  ``NativeLLMEngine`` in ``worker/engines/llm_native.py`` wraps it in
the reference's ``LLMBaseEngine`` contract (worker/engines/llm_base.py:45-188).
"""
from __future__ import annotations

import dataclasses
import math
import time
from typing import Iterable, Optional

import numpy as np
import torch

from dgi.kv.block_pool import BlockPool, OutOfBlocks, num_blocks_for_budget
from dgi.models.config import ModelConfig, get_config
from dgi.models.llama import LlamaModel
from dgi.runtime.model_runner import ModelRunner
from dgi.sched.request import Request, SamplingParams, Status
from dgi.sched.scheduler import Scheduler, SchedulerConfig
from dgi.utils.trace import phase


@dataclasses.dataclass
class EngineConfig:
    model: str = "llama3-8b"
    device: str = "cuda"
    dtype: torch.dtype = torch.bfloat16
    block_size: int = 16
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 8192
    max_model_len: int = 8192
    kv_fraction: float = 0.90          # of (device memory - weights - workspace)
    num_blocks: Optional[int] = None   # override the budget computation
    enable_prefix_caching: bool = True
    use_graphs: bool = True
    seed: int = 0
    workspace_bytes: int = 8 << 30
    layer_start: int = 0
    layer_end: Optional[int] = None
    host_kv_gb: float = 0.0            # pinned host KV tier: evicted prefix pages + swapped-out
                                       # preempted sequences (0 = off, < 0 = auto-size: ``auto_host_kv_gb``)
    graph_buckets: Optional[tuple] = None   # decode batch sizes captured as hipGraphs (None = defaults)
    model_path: Optional[str] = None   # HF safetensors checkpoint dir (None: ``model`` if it is one, else random init)
    token_align: int = -1              # round mixed-step row counts down to a multiple of this (the GEMM
                                       # row tile; -1 = 256 on GPU engines, 0 = off): SchedulerConfig
    tpot_slo_ms: float = 0.0           # > 0: cap each step's rows so a step (= a decode token's wait)
                                       # stays under this (dgi.sched.slo.StepBudget)
    decode_lookahead: bool = True      # pure-decode graph steps: launch step N+1 before step N's
                                       # tokens are back (``LLMEngine._lookahead``); DGI_DECODE_LOOKAHEAD=0


@dataclasses.dataclass
class StepOutput:
    rid: object
    token: int
    finished: bool
    finish_reason: Optional[str]
    request: Request


def _device_free_bytes(device: torch.device) -> int:
    if device.type == "cuda":
        free, _total = torch.cuda.mem_get_info(device)
        return free
    return 2 << 30


def engine_block_budget(cfg: EngineConfig, mc: ModelConfig, n_local: int, device: torch.device) -> int:
    """KV pages for this engine: ``kv_fraction`` of free HBM after weights and the
    activation workspace, capped by what ``max_num_seqs`` full sequences can use."""
    if cfg.num_blocks is not None:
        return cfg.num_blocks
    if device.type == "cuda":
        budget = max(0, _device_free_bytes(device) - cfg.workspace_bytes) * cfg.kv_fraction
    else:
        budget = 1 << 30  # CPU rehearsal runs: a fixed 1 GiB pool
    nblocks = num_blocks_for_budget(int(budget), max(1, n_local), mc.num_kv_heads, mc.head_dim, cfg.block_size)
    # never more than what max_num_seqs full-length sequences can use (+ prefix cache room)
    cap = 2 * cfg.max_num_seqs * ((cfg.max_model_len + cfg.block_size - 1) // cfg.block_size) + 1
    return max(2, min(nblocks, cap))


def auto_host_kv_gb(pool: BlockPool, device: torch.device, pool_share: float = 0.5,
                    ram_share: float = 0.25) -> float:
    """Size of the pinned host KV tier when ``host_kv_gb < 0``: half the HBM KV
    pool (on a 288 GB MI355X serving 70B that is ~55 GB per GPU, enough to hold
    every sequence preempted in a burst), capped by this GPU's share of a quarter
    of the host's available RAM (pinned pages cannot be swapped by the OS)."""
    try:
        import psutil
        avail = psutil.virtual_memory().available
    except Exception:   # pragma: no cover - psutil is optional
        avail = 16 << 30
    gpus = max(1, torch.cuda.device_count()) if device.type == "cuda" else 1
    want = pool.page_bytes() * pool.num_blocks * pool_share
    return min(want, avail * ram_share / gpus) / (1 << 30)


class LLMEngine:
    def __init__(self, cfg: EngineConfig, model_cfg: Optional[ModelConfig] = None, model=None):
        self.cfg = cfg
        self.device = torch.device(cfg.device)
        if self.device.type == "cuda":
            if self.device.index is None:
                self.device = torch.device("cuda", torch.cuda.current_device())
            torch.cuda.set_device(self.device)
        self.checkpoint = None
        if model is None:
            from dgi.models.weights import resolve_checkpoint
            self.checkpoint = resolve_checkpoint(cfg.model, cfg.model_path)
        self.model_cfg = model_cfg or get_config(self.checkpoint or cfg.model)
        self.model_cfg.max_position = max(self.model_cfg.max_position, cfg.max_model_len)
        t0 = time.perf_counter()
        self.model = model or LlamaModel(self.model_cfg, self.device, cfg.dtype, cfg.layer_start, cfg.layer_end,
                                         seed=cfg.seed, checkpoint=self.checkpoint)
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        self.load_seconds = time.perf_counter() - t0
        mc = self.model_cfg
        n_local = self.model.num_local_layers
        nblocks = engine_block_budget(cfg, mc, n_local, self.device)
        self.pool = BlockPool(nblocks, cfg.block_size, max(1, n_local), mc.num_kv_heads, mc.head_dim,
                              cfg.dtype, self.device)
        align = cfg.token_align if cfg.token_align >= 0 else (256 if self.device.type == "cuda" else 0)
        self.scheduler = Scheduler(self.pool, SchedulerConfig(cfg.max_num_seqs, cfg.max_num_batched_tokens,
                                                              cfg.max_model_len, cfg.enable_prefix_caching,
                                                              token_align=align))
        self.host_tier = None
        host_gb = cfg.host_kv_gb
        if host_gb < 0:      # auto: GPU engines only (CPU rehearsals have no HBM to relieve)
            host_gb = auto_host_kv_gb(self.pool, self.device) if self.device.type == "cuda" else 0.0
        if host_gb > 0:
            from dgi.kv.host_tier import HostKVTier
            from dgi.kv.radix_cache import RadixCache
            cap = max(1, int(host_gb * (1 << 30) // self.pool.page_bytes()))
            self.host_tier = HostKVTier(self.pool, cap)
            self.scheduler.host_tier = self.host_tier
            if cfg.enable_prefix_caching:
                self.scheduler.radix = RadixCache(self.pool, self.host_tier)
        rkw = {"graph_buckets": tuple(cfg.graph_buckets)} if cfg.graph_buckets else {}
        self.runner = ModelRunner(self.model, self.pool, cfg.max_num_seqs, cfg.max_model_len,
                                  cfg.max_num_batched_tokens, cfg.use_graphs, **rkw)
        self.runner.host_tier = self.host_tier
        self.requests: dict = {}
        # decode lookahead: (ScheduledBatch, launch handle) of a step in flight, not applied yet
        import os as _os
        self._la = None
        self.lookahead = bool(cfg.decode_lookahead) and _os.environ.get("DGI_DECODE_LOOKAHEAD", "1") == "1"
        # mixed-step lookahead: an eager step in flight, its tokens not committed yet
        # (``_launch_eager`` / ``_step_mixed_lookahead``).  Off by default (DGI_MIXED_LOOKAHEAD=1
        # turns it on): on the 70B closed-loop bench it left throughput unchanged (1,868 vs
        # 1,869-1,887 tok/s: the 203 ms step is GEMM-bound, its host gap ~2 %) and doubled p50 TTFT
        # (408 vs 210 ms), since a request that arrives while step N runs misses the already
        # launched step N+1 (profiles/r5_final/README.md)
        self._mx = None
        self.mixed_lookahead = bool(cfg.decode_lookahead) and _os.environ.get("DGI_MIXED_LOOKAHEAD", "0") == "1"
        self.mixed_chained = 0
        self.step_budget = None
        if cfg.tpot_slo_ms > 0:
            from dgi.sched.slo import StepBudget
            self.step_budget = StepBudget(cfg.tpot_slo_ms)
        # optional callback(ScheduledBatch) between scheduling and execution (P/D streaming)
        self.pre_execute = None
        # optional callback(Request) when a request's first token is sampled, BEFORE any
        # stop check may free its pages (cross-worker KV export)
        self.first_token_hook = None
        self.stats = {"steps": 0, "prefill_tokens": 0, "decode_tokens": 0, "generated": 0,
                      "finished": 0, "step_time": 0.0}
        # MLP row padding measured on this GPU (hipBLASLt kernel-selection cliffs, dgi.runtime.gemm_pad)
        self.mlp_pad_table = None
        if self.device.type == "cuda" and getattr(self.model, "mlp_pad", None) is None:
            from dgi.runtime.gemm_pad import build_for_model
            t1 = time.perf_counter()
            self.mlp_pad_table = build_for_model(self.model, cfg.max_num_batched_tokens)
            if self.mlp_pad_table is not None:
                self.model.mlp_pad = self.mlp_pad_table.pad
                self.model.mlp_impl = self.mlp_pad_table.impl
                self.model.proj_impl = self.mlp_pad_table.proj_impl
                H = self.model.cfg.hidden_size
                self.model.fold_impl = lambda rows, _t=self.mlp_pad_table: _t.fold(rows, H)
                self.mlp_pad_seconds = time.perf_counter() - t1
        # the fused-norm layers need the gains folded into the weights; done once, eagerly, so every
        # engine sharing this model (and every captured graph) computes with the same weights — for
        # the models that will run them (dgi.models.llama.NORM_FOLD: routed production shapes by
        # default); other models keep their weights bit for bit
        if self.device.type == "cuda" and hasattr(self.model, "fold_norms"):
            from dgi.models import llama as _llama
            if _llama.NORM_FOLD == "force" or (_llama.NORM_FOLD in ("1", "table") and self.mlp_pad_table is not None):
                self.model.fold_norms()

    # ------------------------------------------------------------------ API
    def add_request(self, prompt_ids: list[int], params: Optional[SamplingParams] = None, rid=None,
                    user=None) -> Request:
        req = Request(prompt_ids, params or SamplingParams(), rid=rid, user=user)
        self.scheduler.add(req)
        self.requests[req.rid] = req
        if self.step_budget is not None:
            self.step_budget.observe_request(len(req.prompt), req.params.max_tokens)
        return req

    def abort(self, rid) -> bool:
        self.requests.pop(rid, None)
        return self.scheduler.abort(rid)

    def admission_limit(self) -> Optional[int]:
        """Sequences this engine keeps in flight (running + one step of queued prompts)
        without missing its TPOT SLO; None without an SLO or before it has measured
        enough.  A closed-loop client sizes its concurrency to it.

        The queued part is counted from the sequences running NOW, not from the
        steady-state cap: under the SLO the prefill rate is a fixed number of prompts
        per step, so while the running set ramps up (or after a burst of finishes)
        anything queued beyond one step's prompts only waits — its TTFT grows by a
        step per step's worth of prompts ahead of it (round 5: 15 queued behind a
        1.6-prompt step = 827 ms p50 TTFT at SLO 120)."""
        sbud = self.step_budget
        if sbud is None:
            return None
        cap = sbud.admission_cap(self.cfg.max_num_batched_tokens)
        if cap is None:
            return None
        rows = sbud.rows_at_slo() or 0
        # prompts one SLO-sized step prefills, rounded UP: the running set can only grow as fast
        # as prompts are admitted, so rounding 1.5 down to 1 would pin it below the cap
        # (round 5: 128 running instead of ~190, 1.51k tok/s)
        prefill_rows = rows - rows * (sbud.output_avg or 0) / max(1.0, (sbud.prompt_avg or 0) + (sbud.output_avg or 0))
        queued = max(1, math.ceil(prefill_rows / max(1.0, sbud.prompt_avg or 1.0)))
        return min(cap, len(self.scheduler.running)) + queued

    def has_unfinished(self) -> bool:
        return self._la is not None or self._mx is not None or self.scheduler.has_work()

    def warmup(self) -> None:
        """Capture decode graphs ahead of serving."""
        if self.runner.graphs is not None:
            self.runner.graphs.capture()

    def step(self) -> list[StepOutput]:
        t0 = time.perf_counter()
        if self._la is not None:
            n = len(self._la[0].decode)
            outs = self._step_lookahead()
            self._account(n, time.perf_counter() - t0)
            return outs
        if self._mx is not None:
            n = self._mx[0].num_tokens
            outs = self._step_mixed_lookahead()
            self._account(n, time.perf_counter() - t0)
            return outs
        self.model.kv_cache = self.pool.kv   # engines may share one model object
        with phase("schedule"):
            sbud = self.step_budget
            cap = None
            if sbud is not None:
                cap = sbud.budget(self.cfg.max_num_batched_tokens, len(self.scheduler.running))
                self.scheduler.admit_cap = sbud.admission_cap(self.cfg.max_num_batched_tokens)
            sb = self.scheduler.schedule(max_tokens=cap)
        if sb.empty:
            return []
        if self.pre_execute is not None:
            self.pre_execute(sb)
        if self._lookahead_ok(sb):
            # pure decode on the graphs: launch it, then (while it runs) the step after it
            self.runner.step_id += 1
            self._la = (sb, self.runner.graphs.launch(sb.decode))
            out = self._step_lookahead()
            self._account(sb.num_tokens, time.perf_counter() - t0)
            return out
        if self._mixed_ok(sb):
            # eager step: launch it, then (while it runs) schedule and launch the step after it
            self._mx = self._launch_eager(sb)
            outs = self._step_mixed_lookahead()
            self._account(sb.num_tokens, time.perf_counter() - t0)
            return outs
        with phase("execute", decode=len(sb.decode), prefill=len(sb.prefill)):
            res = self.runner.execute(sb)
        with phase("apply"):
            outs = self._apply(sb, res.rows, res.tokens)
        dt = time.perf_counter() - t0
        self._account(sb.num_tokens, dt)
        if sbud is not None and sb.prefill:       # mixed / prefill steps set the per-row cost
            sbud.observe(sb.num_tokens, dt * 1e3)
        return outs

    def _account(self, rows: int, dt: float) -> None:
        """Step wall time and row-count histogram (every step, lookahead chains included)."""
        self.stats["step_time"] += dt
        rh = self.stats.setdefault("rows_hist", {})         # step row counts (GEMM M): tile alignment / SLO
        rh[rows] = rh.get(rows, 0) + 1

    def drain(self) -> list[StepOutput]:
        """Collect and apply a lookahead step still in flight (teardown, or before the
        running set is changed from outside the engine)."""
        outs = []
        if self._mx is not None:
            sb, sampled, _tok, host, ev = self._mx
            self._mx = None
            outs = self._collect_eager(sampled, host, ev)
        if self._la is not None:
            sb, h = self._la
            self._la = None
            toks = self.runner.graphs.collect(h)
            keep = [(r, t) for r, t in zip(sb.decode, toks) if r.status is Status.RUNNING]
            if keep:
                outs = self._apply(type(sb)([r for r, _t in keep], [], []), [r for r, _t in keep],
                                   [t for _r, t in keep])
        return outs

    # ------------------------------------------------------------------ mixed-step lookahead
    def _mixed_ok(self, sb) -> bool:
        """Eager (prefill / mixed / beyond-graph) steps of a plain GPU engine chain: step N+1 is
        scheduled and launched while step N runs, its rows' input tokens read on the device."""
        return (self.mixed_lookahead and self.device.type == "cuda" and type(self) is LLMEngine
                and self.pre_execute is None and self.first_token_hook is None and self.step_budget is None
                and self.host_tier is None and not sb.preempted and all(r.swapped is None for r in sb.decode))

    def _launch_eager(self, sb, prev=None) -> tuple:
        """Enqueue one eager step (forward, sampling, async copy of the tokens to the host) and
        advance its rows' KV cursors.  ``prev`` = (sampled rows, device tokens) of the step in
        flight: a row whose input token is one of those reads it on the device."""
        run = self.runner
        run.step_id += 1
        src, dst, ahead = [], [], None
        if prev is not None:
            where = {id(r): j for j, r in enumerate(prev[0])}
            for k, r in enumerate(sb.decode):
                j = where.get(id(r))
                if j is not None:
                    dst.append(k)
                    src.append(j)
            if dst:
                ahead = [0] * (len(sb.decode) + sum(1 for c in sb.prefill if c.sample))
                for k in dst:
                    ahead[k] = 1
        with phase("execute", decode=len(sb.decode), prefill=len(sb.prefill)):
            flat, hdr, sampled = run.build_host(sb, seed_ahead=ahead)
            n = len(dst)
            if n:      # the token map rides in the step's one H2D copy
                flat = np.concatenate([flat, np.asarray(dst, np.int32), np.asarray(src, np.int32)])
            dev = run.to_device(flat)
            ids, meta, samp = run.meta_from_device(dev, hdr)
            if n:
                L = int(hdr[run.H_LEN])
                ids.index_copy_(0, dev[L:L + n].long(), prev[1].index_select(0, dev[L + n:L + 2 * n].long())
                                .to(ids.dtype))
            logits = self.model.forward(meta, input_ids=ids)
            tok = host = ev = None
            if sampled:
                tok = samp.sample(logits)
                host = torch.empty(tok.shape, dtype=tok.dtype, pin_memory=True)
                host.copy_(tok, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
        self._advance(sb)
        return (sb, sampled, tok, host, ev)

    def _collect_eager(self, sampled, host, ev) -> list[StepOutput]:
        if ev is None:
            return []
        wh = self.runner.wait_hook
        if wh is None:
            ev.synchronize()
        else:
            while not ev.query():
                wh()
                time.sleep(0.00002)
        toks = host.tolist()
        with phase("apply"):
            keep = [(r, t) for r, t in zip(sampled, toks) if r.status is Status.RUNNING]
            return self._commit([r for r, _t in keep], [t for _r, t in keep])

    def _step_mixed_lookahead(self) -> list[StepOutput]:
        """Schedule and launch step N+1, then collect and commit step N (in flight).  Rows whose
        step-N token ends them by length are not scheduled again; a row that step N ends by
        EOS / stop id still runs in N+1 and that token is discarded.  The chain stops when the
        next step is a pure-decode step the captured graphs take."""
        sb, sampled, tok, host, ev = self._mx
        self._mx = None
        cap = self.cfg.max_model_len - 1
        ending = [r for r in sampled if len(r.output) + 1 >= r.params.max_tokens
                  or len(r.prompt) + len(r.output) + 1 >= cap]
        for r in ending:
            r.busy = True
        try:
            with phase("schedule"):
                sb2 = self.scheduler.schedule(preempt=False)
        finally:
            for r in ending:
                r.busy = False
        g = self.runner.graphs
        graph_next = (g is not None and not sb2.prefill and sb2.decode and len(sb2.decode) <= g.max_bucket)
        if not sb2.empty and not graph_next and tok is not None and self._mixed_ok(sb2):
            self._mx = self._launch_eager(sb2, prev=(sampled, tok))
            self.mixed_chained += 1
        return self._collect_eager(sampled, host, ev)

    # ------------------------------------------------------------------ decode lookahead
    def _lookahead_ok(self, sb) -> bool:
        """Decode lookahead applies to pure-decode steps on the captured graphs of a plain
        engine with nothing else to schedule (no waiting prompt, no prefill chunk, no swap)."""
        g = self.runner.graphs
        return (self.lookahead and g is not None and type(self) is LLMEngine and not sb.prefill and sb.decode
                and not sb.preempted and len(sb.decode) <= g.max_bucket and not self.scheduler.waiting
                and self.pre_execute is None and self.step_budget is None
                and all(r.swapped is None for r in sb.decode))

    def _step_lookahead(self) -> list[StepOutput]:
        """Collect and apply the step in flight — after launching the next one when every
        row continues (no length stop due, nothing waiting to be scheduled): the host work
        of applying step N and packing step N+1 overlaps step N+1 on the GPU instead of
        leaving the GPU idle between graph replays.  A row whose step-N token ends it
        (EOS / stop id) still runs in step N+1; that token is discarded when applied."""
        sb, h = self._la
        self._la = None
        g = self.runner.graphs
        nxt = None
        cap = self.cfg.max_model_len - 1
        live = [r for r in sb.decode if r.status is Status.RUNNING]
        # the running set must be exactly these rows: a sequence admitted meanwhile (P/D import,
        # swap-in) ends the chain so the next step schedules it
        if live and len(live) == len(sb.decode) == len(self.scheduler.running) and not self.scheduler.waiting and all(
                len(r.output) + 1 < r.params.max_tokens and len(r.prompt) + len(r.output) + 1 < cap for r in live):
            try:
                for r in live:                       # the page of position num_computed + 1
                    self.scheduler._grow(r, r.num_computed + 2)
                nxt = live
            except OutOfBlocks:                      # out of pages: no lookahead this step (pages grown
                nxt = None                           # for earlier rows are the ones they need next step)
        if nxt is not None:
            self.runner.step_id += 1
            self._la = (type(sb)(list(nxt), [], []), g.launch(nxt, ahead=1))
        with phase("execute", decode=len(sb.decode), prefill=0):
            toks = g.collect(h)
        with phase("apply"):
            keep = [(r, t) for r, t in zip(sb.decode, toks) if r.status is Status.RUNNING]
            if len(keep) != len(sb.decode):          # finished at the previous step: tokens discarded
                sb = type(sb)([r for r, _t in keep], [], [])
            outs = self._apply(sb, [r for r, _t in keep], [t for _r, t in keep])
        if self._la is not None and not any(r.status is Status.RUNNING for r in self._la[0].decode):
            # every row of the launch in flight stopped at this step (EOS / stop id): collect it now
            # (its tokens are discarded) instead of leaving the engine with work and no requests
            self.drain()
        return outs

    def _apply(self, sb, rows, tokens) -> list[StepOutput]:
        """Commit one executed batch: advance KV cursors, append tokens, stop checks."""
        self._advance(sb)
        return self._commit(rows, tokens)

    def _advance(self, sb) -> None:
        """The KV-cursor half of applying a step (what scheduling the next step needs)."""
        st = self.stats
        st["steps"] += 1
        st["decode_tokens"] += len(sb.decode)
        radix = self.scheduler.radix
        for c in sb.prefill:
            c.req.num_computed += c.length
            st["prefill_tokens"] += c.length
            if c.sample and radix is not None:      # prompt fully computed: publish its pages
                self.scheduler.on_prefilled(c.req)
        for r in sb.decode:
            r.num_computed += 1

    def _commit(self, rows, tokens) -> list[StepOutput]:
        """The token half: append the sampled tokens, stop checks, finish requests."""
        now = time.perf_counter()
        st = self.stats
        outs = []
        eos = self.model_cfg.eos_token_id
        len_cap = self.cfg.max_model_len - 1
        hook = self.first_token_hook
        finish = self.scheduler.finish
        for req, tok in zip(rows, tokens):
            tok = int(tok)
            out = req.output
            out.append(tok)
            req.token_times.append(now)
            if req.first_token_time is None:
                req.first_token_time = now
                if hook is not None:
                    hook(req)
            p = req.params
            # stop checks (``_check_stop``) inlined: this loop runs once per sampled row
            if len(out) >= p.max_tokens:
                reason = "length"
            elif not p.ignore_eos and (tok == eos or tok in p.stop_token_ids):
                reason = "stop"
            elif len(req.prompt) + len(out) >= len_cap:
                reason = "length"
            else:
                reason = None
            if reason is not None:
                finish(req, reason)
                st["finished"] += 1
                self.requests.pop(req.rid, None)
                if self.step_budget is not None:
                    self.step_budget.observe_finished(len(req.prompt), len(out))
            outs.append(StepOutput(req.rid, tok, reason is not None, reason, req))
        st["generated"] += len(outs)
        return outs

    def _check_stop(self, req: Request, tok: int) -> Optional[str]:
        p = req.params
        if len(req.output) >= p.max_tokens:
            return "length"
        if not p.ignore_eos and (tok == self.model_cfg.eos_token_id or tok in p.stop_token_ids):
            return "stop"
        if req.total_len >= self.cfg.max_model_len - 1:
            return "length"
        return None

    # ------------------------------------------------------------------ cross-worker KV (dgi.kv.transfer)
    def export_request_kv(self, req: Request) -> torch.Tensor:
        """The pages holding ``req``'s computed tokens, all local layers, on the host:
        [L, 2, n_pages, n_kv, page, head_dim]."""
        from dgi import ops
        nb = (req.num_computed + self.pool.block_size - 1) // self.pool.block_size
        ids = torch.tensor(req.blocks[:nb], dtype=torch.int32, device=self.device)
        return ops.kv_gather(self.pool.kv, ids).cpu()

    def import_prefilled(self, prompt: list[int], first_token: int, kv: torch.Tensor,
                         params: Optional[SamplingParams] = None, rid=None, seed: Optional[int] = None) -> Request:
        """Adopt a sequence another worker prefilled: its pages ``kv`` (``export_request_kv``
        layout) go into fresh pages of this pool and decoding continues from
        ``first_token`` — no prompt recompute.  ``seed``: the exporting request's
        sampling seed (a seeded request then draws the same tokens as on one
        worker).  The first token goes through the same stop checks as a local
        one: a sequence that ended there (EOS / stop id / max_tokens) comes back
        FINISHED with its pages released."""
        from dgi import ops
        L, two, n, nkv, bs, hd = kv.shape
        pool = self.pool
        if (L, nkv, bs, hd) != (pool.kv.shape[0], pool.kv.shape[3], pool.kv.shape[4], pool.kv.shape[5]):
            raise ValueError(f"KV geometry {tuple(kv.shape)} does not match this engine's pool "
                             f"{tuple(pool.kv.shape)}")
        if n != (len(prompt) + bs - 1) // bs:
            raise ValueError(f"{n} pages for a {len(prompt)}-token prompt")
        ids = pool.allocate(n)
        ops.kv_scatter(pool.kv, torch.tensor(ids, dtype=torch.int32, device=self.device),
                       kv.to(self.device, pool.dtype))
        req = Request(prompt, params or SamplingParams(), rid=rid)
        if seed is not None:
            req.seed = int(seed) & 0x7FFFFFFF
        req.output = [int(first_token)]
        req.first_token_time = time.perf_counter()
        req.token_times.append(req.first_token_time)
        self.scheduler.add_prefilled(req, ids)
        reason = self._check_stop(req, int(first_token))
        if reason is not None:
            self.scheduler.finish(req, reason)
            self.stats["finished"] += 1
            return req
        self.requests[req.rid] = req
        return req

    def generate(self, prompts: Iterable[list[int]], params: Optional[SamplingParams] = None) -> list[Request]:
        reqs = [self.add_request(p, params) for p in prompts]
        while any(r.status is not Status.FINISHED for r in reqs):
            self.step()
        return reqs
