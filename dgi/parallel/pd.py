"""Prefill/decode disaggregation inside one MI355X node (DistServe style).

The reference's P/D path is an in-memory scheduler whose KV migration is
``asyncio.sleep(0.05)`` (server/app/services/pd_scheduler.py:404-479,
SURVEY §3.5).  Here:

* **Prefill ranks** (``PrefillServer``) run a prefill-only engine: full
  model per GPU (Llama-3-70B bf16 fits in 288 GB), batched/chunked prefill.
  When a prompt completes, its first token is sampled locally and its KV
  pages are packed per decode stage with the ``kv_gather`` HIP kernel (that
  stage's layer slice, one contiguous buffer per layer group); each group goes
  straight to its stage over RCCL — after a ready-to-send / clear-to-send
  handshake (``dgi.parallel.kv_transfer``) that makes the data plane
  deadlock-free by construction.  Request metadata rides the control plane.
* **Decode replicas**: the node runs R decode replicas (``NodeLayout.
  decode_groups``), each a whole-model decode GPU or a decode layer pipeline.
  A replica's **driver** (``DecodeDriver``) allocates pages when a migration
  is announced and tells its later stages the page ids (each stage receives its
  own slice straight from the prefill rank, installs it when it lands and
  reports LANDED); the driver admits the requests once its own slice has landed
  and every stage has reported, so sequences already decoding never wait for a
  migration in flight (reference semantics: a job moves to decode and is
  placed independently of its transfer, pd_scheduler.py:207-232).
* **Placement**: each prefill rank runs a node-local instance of the
  reference's ``PrefillDecodeScheduler`` (server/app/services/pd_scheduler.py
  API, reference :274-323): every replica is a registered DECODE worker whose
  KV headroom is the credit it granted this rank, and ``assign_job`` picks the
  replica by bandwidth x headroom / (1 + active) at admission.  Migrations
  are accounted through ``KVCacheMigrator.record`` (the reference's stub
  transfer, pd_scheduler.py:452-479, is the RCCL path here).
* **Flow control**: every driver grants block *credits* to every prefill
  rank; a prefill rank admits a prompt only when some replica holds credit
  for the whole sequence (prompt + max_tokens), and credits flow back — with
  the ids of the finished requests — when sequences finish, so no decode pool
  can run out and nothing is ever preempted on the decode side.

Control messages (int64, "ctrl" tag, prefill <-> driver):
  MIGRATE n_reqs total_blocks meta_len tok_len chunk_layers key | CREDIT blocks seqs rid* | DONE |
  FENCE n_migrations | FINISHED rid tok code | TOKENS (rid tok code)* | FIRST n (tok code)*

Layer-streamed migration (``stream_layers`` = C > 0): the
prefill rank announces the prompts that finish in a step BEFORE it runs
(MIGRATE, first tokens unknown), and a model layer hook gathers each C-layer
group of their pages as soon as the step's forward has written those layers;
each group is its own handshake transfer, so the data overlaps the remaining
layers' compute.  The first tokens follow in a FIRST message once sampled.
"""
from __future__ import annotations

import collections
import importlib.util
import os
import time
from typing import Optional

import numpy as np
import torch

from dgi import ops
from dgi.engine import EngineConfig, LLMEngine, StepOutput
from dgi.models.config import get_config
from dgi.parallel.fabric import CtrlChannel, Fabric
from dgi.parallel.kv_transfer import KVReceiver, KVSender, scatter_groups
from dgi.parallel.pipeline import PipelineEngine
from dgi.parallel.plan import NodeLayout
from dgi.sched.request import Request, SamplingParams, Status
from dgi.utils.trace import mark, phase

MSG_MIGRATE, MSG_CREDIT, MSG_DONE, MSG_FINISHED, MSG_TOKENS, MSG_FIRST = 1, 2, 3, 4, 5, 6
# a prefill rank has stopped stepping and drained every transfer it started: the
# message carries how many migrations it announced to this driver in total
MSG_FENCE = 7
REASONS = {0: None, 1: "length", 2: "stop"}
CTRL = 8
META_FIELDS = 12
# per-GPU figures registered with the node-local P/D scheduler (MI355X: ~2.5 PF
# dense bf16, 8 TB/s HBM3E); only their ratios matter for placement
MI355X_TFLOPS = 2500.0
MI355X_HBM_GBPS = 8000.0


def pd_scheduler_module():
    """The reference-compatible ``PrefillDecodeScheduler`` / ``KVCacheMigrator``
    (server/app/services/pd_scheduler.py), imported without the server app."""
    try:
        from server.app.services import pd_scheduler as m   # repo root on sys.path
        return m
    except ImportError:
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        path = os.path.join(root, "server", "app", "services", "pd_scheduler.py")
        spec = importlib.util.spec_from_file_location("dgi_pd_scheduler", path)
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        return m


def run_sync(coro):
    """Drive a coroutine that never suspends (the scheduler's bookkeeping
    methods) to completion without an event loop."""
    try:
        coro.send(None)
    except StopIteration as e:
        return e.value
    coro.close()
    raise RuntimeError("coroutine suspended outside an event loop")


def layer_groups(n_layers: int, chunk: int) -> list:
    """[a, b) layer groups a stage receives a migration in (chunk 0: all at once)."""
    if chunk <= 0:
        return [(0, n_layers)]
    return [(a, min(n_layers, a + chunk)) for a in range(0, n_layers, chunk)]


def _blocks_for(n_tokens: int, bs: int) -> int:
    return (n_tokens + bs - 1) // bs


def _code(o) -> int:
    return {"length": 1, "stop": 2}.get(o.finish_reason, 2) if o.finished else -1


def _req_meta(r: Request, nblocks: int, first: Optional[int] = None) -> list:
    p = r.params
    age_us = int((time.perf_counter() - r.arrival) * 1e6)    # time since arrival on the prefill rank
    return [int(r.rid) & 0x7FFFFFFF, 0, len(r.prompt), r.output[0] if first is None else first, nblocks,
            p.max_tokens,
            int(np.float32(p.temperature).view(np.int32)), int(r.seed) & 0x7FFFFFFF, int(p.ignore_eos), p.top_k,
            int(np.float32(p.top_p).view(np.int32)), age_us]


class PrefillServer:
    """One prefill rank: admits prompts against decode credit, prefills them and
    migrates each finished prompt's KV to the decode replica chosen for it."""

    def __init__(self, cfg: EngineConfig, fabric: Fabric, layout: NodeLayout, seed_offset: int = 0,
                 local_cap: int = 0, report_tokens: bool = False, router: Optional[int] = None,
                 stream_layers: int = 8):
        self.f = fabric
        self.layout = layout
        self.drivers = list(layout.drivers)
        self.groups = {g[0]: list(g) for g in layout.decode_groups}
        self.driver = self.drivers[0]
        # overflow tokens / done-at-first-token reports go to the node router
        self.router = self.drivers[0] if router is None else router
        # overflow decoding: when no replica has credit left, up to ``local_cap``
        # sequences stay on this rank and decode inside its mixed
        # prefill+decode steps instead of the rank idling until credit returns
        # (decode-bound layouts: profiles/r1_pd_capacity_70b.md).  ``report_tokens``
        # streams their tokens to the router once per step.
        self.local_cap = local_cap
        self.local: set = set()
        self.local_tokens = 0
        self.report_tokens = report_tokens
        pcfg = EngineConfig(**{**cfg.__dict__, "device": str(fabric.device),
                               "use_graphs": bool(cfg.use_graphs and local_cap > 0)})
        self.engine = LLMEngine(pcfg)
        self.engine.warmup()
        self.bs = self.engine.pool.block_size
        self.ch = {d: CtrlChannel(fabric, d, CTRL) for d in self.drivers}
        # KV data plane: ready-to-send / clear-to-send with every decode rank
        self.sender = KVSender(fabric, layout.decode_ranks)
        # while the host waits for a step's sampled tokens it keeps the handshakes moving
        self.engine.runner.wait_hook = self.sender.service
        self.credit, self.seq_credit = {}, {}
        for d in self.drivers:   # initial credit grant of every replica
            msg = self.ch[d].wait()
            assert msg[0] == MSG_CREDIT, msg
            self.credit[d], self.seq_credit[d] = int(msg[1]), int(msg[2])
        self.credit_total = dict(self.credit)
        self.pending: collections.deque = collections.deque()
        self.target: dict = {}     # rid -> (driver, blocks reserved)
        self.migrated = 0
        self.migrate_time = 0.0
        self.sent_bytes = 0
        self.announced = collections.Counter()     # migrations announced per driver (FENCE count)
        self.next_key = 1
        # each replica's stages are sent their own layer slice of every page
        from dgi.parallel.pipeline import stage_split
        self.splits = {d: stage_split(self.engine.model_cfg, len(g)) for d, g in self.groups.items()}
        self.first_tokens = 0
        self.ttfts: list = []
        # node-local P/D scheduler: replicas are DECODE workers, headroom = our credit
        m = pd_scheduler_module()
        self._pdm = m
        self.pd = m.PrefillDecodeScheduler()
        self.me = f"prefill-{fabric.rank}"
        self.pd.register_worker(self.me, m.WorkerCapability(self.me, m.WorkerRole.PREFILL,
                                                            compute_flops=MI355X_TFLOPS))
        for d, g in self.groups.items():
            self.pd.register_worker(str(d), m.WorkerCapability(
                str(d), m.WorkerRole.DECODE, memory_bandwidth_gbps=MI355X_HBM_GBPS * len(g),
                kv_cache_tokens_total=self.credit_total[d] * self.bs))
        self.migrator = m.KVCacheMigrator(self.pd)
        self.placed: dict = {d: set() for d in self.drivers}
        # layer-streamed migration: C-layer groups leave while later layers compute
        self.stream_layers = int(stream_layers)
        self._streams: list = []       # this step's (driver, reqs, ids_t, {end layer: [...]}, t0)
        self.streamed_bytes = 0
        self._plans = {d: self.chunk_plan(self.splits[d], self.stream_layers) for d in self.drivers}
        if self.stream_layers > 0:
            self.engine.pre_execute = self._plan_stream

    @staticmethod
    def chunk_plan(split: list, C: int) -> list:
        """(stage, c0, c1, group, ngroups) layer groups of at most C layers inside
        each stage slice, in layer order (C <= 0: one group per stage)."""
        out = []
        for si, (a, b) in enumerate(split):
            gs = [(a, b)] if C <= 0 else [(c0, min(b, c0 + C)) for c0 in range(a, b, C)]
            for gi, (c0, c1) in enumerate(gs):
                out.append((si, c0, c1, gi, len(gs)))
        return out

    # ------------------------------------------------------------------ API
    def submit(self, prompt: list, params: SamplingParams, rid=None) -> Request:
        r = Request(prompt, params, rid=rid)
        self.pending.append(r)
        return r

    def busy(self) -> bool:
        """Work left: prompts, engine steps, or KV transfers not yet delivered."""
        return bool(self.pending) or self.engine.has_unfinished() or self.sender.pending() > 0

    def service(self) -> None:
        """Move the KV handshakes forward (also called from inside engine waits)."""
        self.sender.service()

    def _poll_credit(self) -> None:
        for d, ch in self.ch.items():
            while True:
                m = ch.poll()
                if m is None:
                    break
                if m[0] == MSG_CREDIT:
                    self.credit[d] += int(m[1])
                    self.seq_credit[d] += int(m[2])
                    for rid in m[3:3 + int(m[2])]:      # exactly the sequences that finished
                        key = str(int(rid))
                        if key in self.placed[d]:
                            self.placed[d].discard(key)
                            run_sync(self.pd.complete_job(key, self._pdm.JobPhase.DECODE))

    def _pick(self, r: Request, need: int) -> Optional[int]:
        """Replica for a prompt needing ``need`` blocks: the P/D scheduler's
        decode placement over the replicas that hold enough of our credit."""
        ok = {d: self.credit[d] >= need and self.seq_credit[d] > 0 for d in self.drivers}
        if not any(ok.values()):
            return None
        for d in self.drivers:
            tot = self.credit_total[d]
            used = tot - self.credit[d] if ok[d] else tot
            self.pd.update_worker_stats(str(d), {"kv_cache_tokens_used": used * self.bs,
                                                 "kv_cache_tokens_total": tot * self.bs})
        m = self._pdm
        job = m.PendingJob(0.0, time.time(), str(int(r.rid) & 0x7FFFFFFF), m.JobPhase.DECODE, len(r.prompt),
                           r.params.max_tokens, kv_cache_key=f"kv:{r.rid}", kv_cache_worker=self.me)
        a = run_sync(self.pd.assign_job(job))
        d = int(a.worker_id)
        if not ok.get(d):
            run_sync(self.pd.complete_job(job.job_id, m.JobPhase.DECODE))
            return None
        self.placed[d].add(job.job_id)
        return d

    def _unplace(self, d: int, rid) -> None:
        key = str(int(rid) & 0x7FFFFFFF)
        if key in self.placed[d]:
            self.placed[d].discard(key)
            run_sync(self.pd.complete_job(key, self._pdm.JobPhase.DECODE))

    def _admit(self) -> None:
        while self.pending:
            r = self.pending[0]
            need = _blocks_for(len(r.prompt) + r.params.max_tokens, self.bs)
            d = self._pick(r, need)
            if d is not None:
                self.credit[d] -= need
                self.seq_credit[d] -= 1
                self.target[r.rid] = (d, need)
            elif len(self.local) < self.local_cap:
                self.local.add(r.rid)   # decoded here (overflow)
            else:
                break
            self.pending.popleft()
            self.engine.scheduler.add(r)
            self.engine.requests[r.rid] = r

    def _announce(self, d: int, rs: list, streamed: bool) -> tuple:
        """MIGRATE message for requests ``rs`` to replica ``d``; returns (key, ids_t, nblk).
        A streamed migration is announced before its step (first tokens follow in FIRST)."""
        ids, meta, toks = [], [], []
        for r in rs:
            nb = _blocks_for(len(r.prompt) if streamed else r.num_computed, self.bs)
            ids += r.blocks[:nb]
            meta += _req_meta(r, nb, first=-1 if streamed else None) + [int(self.target[r.rid][1])]
            toks += r.prompt
        key = self.next_key
        self.next_key += 1
        self.announced[d] += 1
        ids_t = torch.tensor(ids, dtype=torch.int32, device=self.f.device)
        chunk = self.stream_layers if streamed else 0
        self.ch[d].send([MSG_MIGRATE, len(rs), len(ids), len(meta), len(toks), chunk, key])
        self.ch[d].send_var(np.asarray(meta + toks, dtype=np.int64))
        return key, ids_t, len(ids)

    # ------------------------------------------------------------------ layer-streamed migration
    def _plan_stream(self, sb) -> None:
        """Before a step runs: announce the prompts whose prefill completes in it
        and arm the layer hook that ships their pages group by group."""
        self._streams = []
        fin = [c.req for c in sb.prefill if c.sample and c.req.rid not in self.local and c.req.rid in self.target]
        if not fin:
            return
        by_d: dict = collections.defaultdict(list)
        for r in fin:
            by_d[self.target[r.rid][0]].append(r)
        for d, rs in by_d.items():
            key, ids_t, nblk = self._announce(d, rs, streamed=True)
            by_end: dict = collections.defaultdict(list)
            for item in self._plans[d]:
                by_end[item[2] - 1].append(item)
            self._streams.append((d, rs, ids_t, by_end, time.perf_counter(), key, nblk))
        self.engine.model.layer_hook = self._layer_done

    def _layer_done(self, li: int) -> None:
        from dgi.parallel.fault import plan
        if plan():      # fault site 200000 + layer: a slow layer mid-migration (handshakes stay live)
            plan().check(self.f.rank, 200000 + li, idle=self.sender.service)
        kv = self.engine.pool.kv
        for d, _rs, ids_t, by_end, _t0, key, nblk in self._streams:
            for si, c0, c1, gi, ng in by_end.get(li, ()):
                buf = ops.kv_gather(kv[c0:c1], ids_t)
                a = self.splits[d][si][0]
                self.sender.submit(self.groups[d][si], buf, key, gi, ng, c0 - a, c1 - a, nblk)
                self.streamed_bytes += buf.numel() * buf.element_size()
        self.sender.service()

    def _finish_streams(self, outs) -> set:
        """After the step: first tokens (and finish codes) of the streamed prompts."""
        self.engine.model.layer_hook = None
        done = set()
        if not self._streams:
            return done
        by_rid = {o.rid: o for o in outs}
        eng = self.engine
        for d, rs, ids_t, by_end, t0, key, nblk in self._streams:
            msg = [MSG_FIRST, len(rs)]
            for r in rs:
                o = by_rid[r.rid]
                code = _code(o)
                msg += [int(o.token), code]
                _d, need = self.target.pop(r.rid)
                if o.finished:        # done at the first token: the decode side frees its pages
                    self.credit[d] += need
                    self.seq_credit[d] += 1
                    self._unplace(d, r.rid)
                    self.ch[self.router].send([MSG_FINISHED, int(o.rid), int(o.token), max(0, code)])
                else:
                    eng.scheduler.finish(r, "migrated")
                    eng.requests.pop(r.rid, None)
                done.add(r.rid)
            self.ch[d].send_var(msg)
            dt = time.perf_counter() - t0
            pb = nblk * self.engine.pool.page_bytes()
            self.migrator.record(f"kv:{rs[0].rid}", self.me, str(d), pb, dt * 1000.0)
            self.migrated += sum(1 for r in rs if not by_rid[r.rid].finished)
            self.sent_bytes += pb
            self.migrate_time += dt
        self._streams = []
        return done

    def step(self) -> list[StepOutput]:
        from dgi.parallel.fault import plan
        self.service()
        self._poll_credit()
        self._admit()
        if not self.engine.has_unfinished():
            return []
        if plan():      # fault sites count engine steps (a call that only services transfers is not one)
            plan().check(self.f.rank, self.engine.stats["steps"])
        outs = self.engine.step()
        streamed = self._finish_streams(outs)
        ready = []
        report = []
        for o in outs:
            if o.rid in streamed:
                self.first_tokens += 1
                if o.request.ttft is not None:
                    self.ttfts.append(o.request.ttft)
                continue
            if o.rid in self.local:
                self.local_tokens += 1
                if len(o.request.output) == 1 and o.request.ttft is not None:
                    self.first_tokens += 1
                    self.ttfts.append(o.request.ttft)
                if o.finished:
                    self.local.discard(o.rid)
                if self.report_tokens:
                    report += [int(o.rid), int(o.token), _code(o)]
                continue
            self.first_tokens += 1
            if o.request.ttft is not None:
                self.ttfts.append(o.request.ttft)
            if o.finished:  # max_tokens == 1 or EOS at the first token: nothing to migrate
                d, need = self.target.pop(o.rid)
                self.credit[d] += need
                self.seq_credit[d] += 1
                self._unplace(d, o.rid)
                code = {"length": 1, "stop": 2}.get(o.finish_reason, 0)
                self.ch[self.router].send([MSG_FINISHED, int(o.rid), int(o.token), code])
            else:
                ready.append(o.request)
        if ready:
            with phase("migrate_send", reqs=len(ready)):
                self._migrate(ready)
        if report:
            self.ch[self.router].send_var([MSG_TOKENS] + report)
        self.service()
        return outs

    def _migrate(self, reqs: list) -> None:
        """Hand finished prefills to their decode replicas (bulk: one transfer per
        stage slice).  Each stage of the target replica receives ONLY its own layer
        slice, straight from this rank over its own xGMI link."""
        eng = self.engine
        by_d: dict = collections.defaultdict(list)
        for r in reqs:
            by_d[self.target[r.rid][0]].append(r)
        for d, rs in by_d.items():
            t0 = time.perf_counter()
            key, ids_t, nblk = self._announce(d, rs, streamed=False)
            for r in rs:
                self.target.pop(r.rid)
            bufs = [ops.kv_gather(eng.pool.kv[a:b], ids_t) for a, b in self.splits[d]]
            from dgi.parallel.fault import plan
            if plan():
                def corrupt():
                    bufs[0].view(-1)[: max(1, bufs[0].numel() // 64)] = float("nan")
                plan().check(self.f.rank, self.migrated + 100000, corrupt=corrupt)
            for si, (rank, buf) in enumerate(zip(self.groups[d], bufs)):
                a, b = self.splits[d][si]
                self.sender.submit(rank, buf, key, 0, 1, 0, b - a, nblk)
            for r in rs:
                eng.scheduler.finish(r, "migrated")
                eng.requests.pop(r.rid, None)
            nbytes = sum(b.numel() * b.element_size() for b in bufs)
            dt = time.perf_counter() - t0
            self.migrator.record(f"kv:{rs[0].rid}", self.me, str(d), nbytes, dt * 1000.0)
            self.migrated += len(rs)
            self.sent_bytes += nbytes
            self.migrate_time += dt

    def pd_stats(self) -> dict:
        st = self.pd.get_stats()
        lat = self.migrator.latencies_ms
        st["migration_ms_p50"] = round(float(np.median(lat)), 3) if lat else None
        st["kv_transport"] = self.sender.stats()
        return st

    def fence(self, timeout_s: float = 600.0) -> None:
        """Phase boundary: finish every transfer this rank started (the decode ranks
        keep servicing their handshakes meanwhile), then tell every replica driver
        how many migrations it was announced in total.  Afterwards this rank has
        nothing in flight and may synchronise its device."""
        self.sender.drain(timeout_s)
        for d, ch in self.ch.items():
            ch.send([MSG_FENCE, self.announced[d]])

    def finish(self) -> None:
        """End of stream: drain, then every replica driver keeps serving until DONE."""
        self.sender.drain()
        for ch in self.ch.values():
            ch.send([MSG_DONE])
        self.f.flush()


class _Migration:
    __slots__ = ("p", "key", "ids", "ids_t", "meta", "toks", "first_known", "installed", "t_announced")

    def __init__(self, p, key, ids, ids_t, meta, toks, first_known):
        self.p, self.key, self.ids, self.ids_t = p, key, ids, ids_t
        self.meta, self.toks, self.first_known = meta, toks, first_known
        self.installed = False          # the driver's own slice is in its pool
        self.t_announced = time.perf_counter()


class DecodeDriver:
    """Driver of one decode replica: a single engine or stage 0 of a decode pipeline."""

    def __init__(self, cfg: EngineConfig, fabric: Fabric, layout: NodeLayout, credit_margin: float = 0.02,
                 local_fraction: float = 0.0, router: Optional[int] = None):
        self.f = fabric
        self.layout = layout
        self.group = layout.group_of(fabric.rank)
        assert self.group[0] == fabric.rank, "DecodeDriver runs on a replica's first rank"
        dcfg = EngineConfig(**{**cfg.__dict__, "device": str(fabric.device), "enable_prefix_caching": False})
        self.prefill = list(layout.prefill_ranks)
        if len(self.group) > 1:
            self.engine = PipelineEngine(dcfg, fabric, self.group, kv_sources=self.prefill)
        else:
            self.engine = LLMEngine(dcfg)
            # decode graphs before any migration is in flight
            self.engine.warmup()
        self.L_local = self.engine.model.num_local_layers
        mc = self.engine.model_cfg
        self.mc = mc
        self.bs = self.engine.pool.block_size
        self.chans = {p: CtrlChannel(fabric, p, CTRL) for p in self.prefill}
        self.kvr = KVReceiver(fabric, self.prefill, (2, mc.num_kv_heads, self.bs, mc.head_dim),
                              self.engine.pool.dtype)
        # waits inside the engine (sampled tokens, pipeline token returns) keep the
        # receive queue moving
        self.engine.runner.wait_hook = self.kvr.service
        if isinstance(self.engine, PipelineEngine):
            self.engine.idle_hook = self.kvr.service
        # node router (serving): the other replicas' drivers forward their tokens to it
        self.router = layout.drivers[0] if router is None else router
        self.is_router = fabric.rank == self.router
        self.fwd = None
        self.fwd_in: dict = {}
        if self.is_router:
            self.fwd_in = {d: CtrlChannel(fabric, d, CTRL, tag="fwd") for d in layout.drivers if d != fabric.rank}
        else:
            self.fwd = CtrlChannel(fabric, self.router, CTRL, tag="fwd")
        self.forward_tokens = False     # serving mode: stream outputs to the router
        free = self.engine.pool.num_free
        total = int(free * (1.0 - credit_margin - local_fraction))
        # hybrid decode: a slice of the pool serves prompts admitted locally (mixed
        # prefill+decode steps on the decode GPU) so it is never idle when the
        # prefill side cannot saturate it; migrated sequences keep their credits
        self.local_cap_blocks = int(free * local_fraction)
        self.local_used: dict = {}
        P = max(1, len(self.prefill))
        share = total // P
        seq_share = max(1, cfg.max_num_seqs // P)
        for p in self.prefill:
            self.chans[p].send([MSG_CREDIT, share, seq_share])
        self.origin: dict = {}
        self.arrivals: list = []   # migrated requests not yet reported (first token known)
        self.track_arrivals = False
        self.prefill_finished: list = []   # (rid, token, reason) of sequences done at their first token
        self.remote_tokens: list = []      # (rid, token, reason|None) from prefill ranks / other replicas
        self.refund = collections.Counter()
        self.refund_rids: dict = collections.defaultdict(list)
        self.done = set()
        self.fenced: dict = {}      # prefill rank -> migrations it announced (MSG_FENCE)
        self.announced = collections.Counter()
        self.inflight: list = []    # announced migrations not admitted yet
        self.await_first: dict = {p: collections.deque() for p in self.prefill}
        self.received = 0
        self.recv_bytes = 0
        self.admit_ms: list = []    # MIGRATE -> admitted (whole replica landed), ms

    # ------------------------------------------------------------------ migrations
    def _announced(self, p: int, msg) -> None:
        """MIGRATE from ``p``: allocate pages and tell the later pipeline stages
        (each receives its own layer slice straight from ``p``)."""
        n_reqs, nblk, meta_len, tok_len, chunk, key = (int(x) for x in msg[1:7])
        payload = self.chans[p].wait()
        meta = payload[:meta_len].reshape(n_reqs, META_FIELDS + 1).tolist()
        toks = payload[meta_len:meta_len + tok_len].tolist()
        ids = self.engine.pool.allocate(nblk)
        ids_t = torch.tensor(ids, dtype=torch.int32, device=self.f.device)
        if isinstance(self.engine, PipelineEngine):
            self.engine.send_kv_notice(p, key, ids)
        item = _Migration(p, key, ids, ids_t, meta, toks, chunk == 0)
        self.inflight.append(item)
        self.announced[p] += 1
        if chunk:
            self.await_first[p].append(item)

    def _first(self, p: int, m) -> None:
        """FIRST message of the oldest streamed migration from ``p``."""
        item = self.await_first[p].popleft()
        n = int(m[1])
        for i in range(n):
            item.meta[i][3] = int(m[2 + 2 * i])           # first token
            item.meta[i][1] = int(m[3 + 2 * i])           # finish code (-1: keeps decoding)
        item.first_known = True

    def _admit_arrived(self, block: bool = False) -> None:
        """Admit every migration that is complete on the whole replica: the driver's
        own slice has landed and is installed, its first tokens are known and every
        later stage has reported its slice installed (``PipelineEngine.
        stages_landed``).  Migrations still in flight hold nothing up: the replica
        keeps stepping the sequences it has."""
        keep = []
        self.kvr.service()
        pipe = self.engine if isinstance(self.engine, PipelineEngine) else None
        if pipe is not None:
            pipe.poll_landed()
        for item in self.inflight:
            if not item.installed:
                if block:
                    while not item.first_known:      # FIRST follows its MIGRATE on the same channel
                        self._poll_ctrl(item.p)
                        self.kvr.service()
                        time.sleep(0.0002)
                    groups = self.kvr.wait_landed(item.p, item.key) if self.L_local else []
                elif item.first_known and (self.L_local == 0 or self.kvr.is_landed(item.p, item.key)):
                    groups = self.kvr.take(item.p, item.key)
                else:
                    keep.append(item)
                    continue
                scatter_groups(self.engine.pool.kv, item.ids_t, groups, self.kvr.digests, item.p, item.key)
                self.recv_bytes += sum(b.numel() * b.element_size() for _a, _b, b in groups)
                item.installed = True
            if pipe is not None and not pipe.stages_landed(item.p, item.key):
                if not block:
                    keep.append(item)
                    continue
                while not pipe.stages_landed(item.p, item.key):
                    self.kvr.service()
                    pipe.poll_landed()
                    time.sleep(0.0002)
            mark("kv_migration_landed", len(item.meta))
            self.admit_ms.append((time.perf_counter() - item.t_announced) * 1e3)
            self._admit(item.p, item.ids, item.meta, item.toks)
        self.inflight = keep

    def _admit(self, p: int, ids: list, meta: list, toks: list) -> None:
        sch = self.engine.scheduler
        o = k = 0
        for m in meta:
            rid, code, plen, first, nb, max_tok, tbits, seed, ign, topk, pbits, age_us, credit = m
            if code > 0:
                # streamed prompt that finished at its first token: release its pages
                # (the prefill rank refunded the credit and reported it to the router)
                self.engine.pool.free(ids[k:k + nb])
                o += plen
                k += nb
                continue
            temp = float(np.int32(tbits).view(np.float32))
            top_p = float(np.int32(pbits).view(np.float32))
            sp = SamplingParams(max_tokens=max_tok, temperature=temp, top_p=top_p, top_k=topk,
                                ignore_eos=bool(ign), seed=seed)
            r = Request(toks[o:o + plen], sp)
            r.user = rid            # the prefill side's request id (node router key)
            r.seed = seed
            r.output = [first]
            r.first_token_time = time.perf_counter()
            r.arrival = r.first_token_time - age_us / 1e6     # ~ original arrival on the prefill rank
            o += plen
            sch.add_prefilled(r, ids[k:k + nb])
            self.engine.requests[r.rid] = r
            self.origin[r.rid] = (p, credit, rid)
            if self.track_arrivals:
                self.arrivals.append(r)
            k += nb
        self.received += len(meta)

    def local_blocks_free(self) -> int:
        return self.local_cap_blocks - sum(self.local_used.values())

    def admit_local(self, prompt: list, params: SamplingParams) -> Optional[Request]:
        need = _blocks_for(len(prompt) + params.max_tokens, self.bs)
        if need > self.local_blocks_free():
            return None
        r = self.engine.add_request(prompt, params)
        self.local_used[r.rid] = need
        return r

    # ------------------------------------------------------------------ control
    def _poll_ctrl(self, p: int) -> None:
        ch = self.chans[p]
        while True:
            m = ch.poll()
            if m is None:
                break
            self._handle(p, m)

    def _handle(self, p: int, m) -> None:
        if m[0] == MSG_MIGRATE:
            self._announced(p, m)
        elif m[0] == MSG_FIRST:
            self._first(p, m)
        elif m[0] == MSG_DONE:
            self.done.add(p)
        elif m[0] == MSG_FENCE:
            self.fenced[p] = int(m[1])
        elif m[0] == MSG_FINISHED:
            if self.track_arrivals:
                self.prefill_finished.append((int(m[1]), int(m[2]), REASONS.get(int(m[3]))))
        elif m[0] == MSG_TOKENS:
            if self.track_arrivals:
                self._take_tokens(m)

    def poll(self) -> None:
        for p in self.chans:
            self._poll_ctrl(p)
        for ch in self.fwd_in.values():      # router: tokens of the other replicas
            while True:
                m = ch.poll()
                if m is None:
                    break
                if self.track_arrivals:
                    self._take_tokens(m)
        self._admit_arrived()

    def _take_tokens(self, m) -> None:
        for i in range(1, len(m) - 2, 3):
            code = int(m[i + 2])
            self.remote_tokens.append((int(m[i]), int(m[i + 1]), None if code < 0 else REASONS.get(code) or "stop"))

    def _forward(self, arrivals: list, outs: list) -> None:
        """Non-router replicas: stream first tokens and step outputs to the router."""
        msg = []
        for r in arrivals:
            msg += [int(r.user), int(r.output[0]), -1]
        for o in outs:
            if o.request.user is None:
                continue
            msg += [int(o.request.user), int(o.token), _code(o)]
        if msg:
            self.fwd.send_var([MSG_TOKENS] + msg)

    def step(self, poll: bool = True) -> list[StepOutput]:
        """One decode iteration.  ``poll`` first takes in control messages and
        admits landed migrations (callers that emit first tokens of arrivals
        before the step poll themselves and pass ``poll=False``)."""
        if poll:
            self.poll()
        arr = []
        if self.forward_tokens and not self.is_router:
            arr, self.arrivals = self.arrivals, []
        outs = self.engine.step() if self.engine.has_unfinished() else []
        for o in outs:
            if o.finished:
                self.local_used.pop(o.rid, None)
                p, credit, prid = self.origin.pop(o.rid, (None, 0, 0))
                if p is not None:
                    self.refund[p] += credit
                    self.refund_rids[p].append(prid)
        for p, rids in list(self.refund_rids.items()):
            self.chans[p].send_var([MSG_CREDIT, self.refund[p], len(rids)] + rids)
        self.refund.clear()
        self.refund_rids.clear()
        if self.forward_tokens and not self.is_router:
            self._forward(arr, outs)
        return outs

    def quiesced(self) -> bool:
        """Every prefill rank has fenced and every migration it announced is admitted."""
        return (len(self.fenced) == len(self.prefill) and not self.inflight
                and all(self.announced[p] >= n for p, n in self.fenced.items()))

    def await_fences(self, timeout_s: float = 600.0) -> None:
        """Keep servicing control messages and KV handshakes until each prefill rank
        has fenced and everything it announced has been admitted, then clear."""
        from dgi.parallel.kv_transfer import DIAG_S, _diag
        t0 = time.perf_counter()
        nxt = t0 + DIAG_S
        while True:
            for p in self.chans:
                self._poll_ctrl(p)
            self._admit_arrived()
            if self.quiesced():
                break
            if time.perf_counter() > nxt:
                nxt += DIAG_S
                _diag(f"driver {self.f.rank} awaiting fences: fenced {self.fenced}, announced "
                      f"{dict(self.announced)}, not admitted {[(m.p, m.key) for m in self.inflight][:8]}; "
                      + self.kvr.describe())
            if time.perf_counter() - t0 > timeout_s:
                raise TimeoutError(f"prefill fences: got {sorted(self.fenced)} of {self.prefill}, "
                                   f"{len(self.inflight)} migrations not landed")
            time.sleep(0.0002)
        self.fenced.clear()

    def all_prefill_done(self) -> bool:
        if len(self.done) == len(self.prefill) and self.inflight:
            self._admit_arrived(block=True)
        return len(self.done) == len(self.prefill) and not self.inflight

    def finish(self) -> None:
        self._admit_arrived(block=True)
        if isinstance(self.engine, PipelineEngine):
            self.engine.stop_stages()
        self.f.flush()

    def stats(self) -> dict:
        a = sorted(self.admit_ms)
        return {"kv_transport": self.kvr.stats(),
                "announce_to_admit_ms_p50": round(a[len(a) // 2], 3) if a else None,
                "announce_to_admit_ms_p95": round(a[int(0.95 * (len(a) - 1))], 3) if a else None}


def build_engine_config(model: str, **kw) -> EngineConfig:
    mc = get_config(model)
    del mc
    return EngineConfig(model=model, **kw)
