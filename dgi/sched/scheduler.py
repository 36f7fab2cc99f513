"""Iteration-level continuous-batching scheduler.

The reference batches at *request* level: it waits for up to
``max_batch_size`` jobs and hands them to the engine as one static batch
(worker/batch_processor.py:60-365), and the live worker runs one job at a
time (worker/main.py:321).  This scheduler re-forms the batch every model
step:

1. every running sequence in the decode phase gets one token (a new KV page
   when it crosses a block boundary); if the pool is exhausted the most
   recently admitted sequence is preempted.  With a pinned host KV tier
   (``dgi.kv.host_tier``) its pages are swapped out (``kv_gather`` + async
   DMA) and copied back when it is re-admitted, so no prefill is recomputed;
   without one (or with the tier full) its pages are released and recomputed
   later, usually from the radix cache;
2. the remaining token budget (``max_num_batched_tokens``) is filled with
   prefill chunks — first unfinished chunks of running sequences, then new
   requests in FCFS/priority order, each admission starting from its longest
   radix-cache prefix hit (chunked prefill).

The result is a ``ScheduledBatch`` whose rows are ordered
[decode rows | prefill rows] for the model runner.
"""
from __future__ import annotations

import collections
import dataclasses
import time
from typing import Optional

from dgi.kv.block_pool import BlockPool, OutOfBlocks
from dgi.kv.radix_cache import RadixCache
from dgi.sched.request import Request, Status


@dataclasses.dataclass
class SchedulerConfig:
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 8192
    max_model_len: int = 8192
    enable_prefix_caching: bool = True
    decode_first: bool = True
    # Tile-aligned steps: when a step mixes decode rows and prefill into more than ``token_align`` rows,
    # its row count is rounded DOWN to a multiple of ``token_align`` and the rest of
    # the prefill waits for the next step.  The projection GEMMs cost whole 256-row
    # tiles (an M = 1917 step pays for 2048 rows), so a closed-loop load that packs
    # 1536 prefill + ~380 decode rows runs 7- and 8-tile steps instead of
    # 8-tile steps with a half-empty last tile; the prefill tokens are the same,
    # some prompts just finish their prefill one step later.
    token_align: int = 0


@dataclasses.dataclass
class PrefillChunk:
    req: Request
    start: int       # first token index of the chunk (== req.num_computed)
    length: int
    sample: bool     # chunk completes the prefill target -> sample a token


@dataclasses.dataclass
class ScheduledBatch:
    decode: list
    prefill: list
    preempted: list

    @property
    def num_tokens(self) -> int:
        return len(self.decode) + sum(c.length for c in self.prefill)

    @property
    def empty(self) -> bool:
        return not self.decode and not self.prefill


class RunningSet:
    """Insertion-ordered set of running requests with the list operations the
    engines use (append / remove / in / iteration / reversed / len), all O(1)
    per element — decode rows reach 1-2k per step in the P/D layouts, where a
    list's ``in`` / ``remove`` made every step quadratic."""
    __slots__ = ("_d",)

    def __init__(self):
        self._d: dict = {}

    def append(self, r: Request) -> None:
        self._d[r] = None

    def remove(self, r: Request) -> None:
        del self._d[r]

    def discard(self, r: Request) -> None:
        self._d.pop(r, None)

    def __contains__(self, r) -> bool:
        return r in self._d

    def __iter__(self):
        return iter(list(self._d))

    def __reversed__(self):
        return reversed(list(self._d))

    def __len__(self) -> int:
        return len(self._d)

    def __bool__(self) -> bool:
        return bool(self._d)


class Scheduler:
    def __init__(self, pool: BlockPool, cfg: SchedulerConfig):
        self.pool = pool
        self.cfg = cfg
        self.bs = pool.block_size
        self.waiting: collections.deque = collections.deque()
        self.running = RunningSet()
        self.radix: Optional[RadixCache] = RadixCache(pool) if cfg.enable_prefix_caching else None
        self.num_preemptions = 0
        self.host_tier = None          # HostKVTier: swap preempted sequences out instead of recomputing
        self.num_swapped_out = 0
        self.num_swapped_in = 0
        # running sequences admitted at most (None: max_num_seqs); the TPOT-SLO budget sets it
        # to what the engine sustains at the SLO (dgi.sched.slo.StepBudget.admission_cap)
        self.admit_cap: Optional[int] = None

    # ------------------------------------------------------------------ queue
    def add(self, req: Request) -> None:
        if req.total_len >= self.cfg.max_model_len:
            raise ValueError(f"prompt of {req.total_len} tokens exceeds max_model_len {self.cfg.max_model_len}")
        req.status = Status.WAITING
        self.waiting.append(req)

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    def abort(self, rid) -> bool:
        for q in (self.waiting, self.running):
            for r in q:
                if r.rid == rid:
                    q.remove(r)
                    if r.swapped is not None:
                        slots, _n, pre = r.swapped
                        if slots:
                            self.host_tier.release(slots)
                        if pre:
                            self.pool.free(pre)
                        r.swapped = None
                    self._release(r, cache=False)
                    r.status = Status.FINISHED
                    r.finish_reason = "abort"
                    return True
        return False

    # ------------------------------------------------------------------ blocks
    def _blocks_needed(self, req: Request, upto: int) -> int:
        return max(0, (upto + self.bs - 1) // self.bs - len(req.blocks))

    def _grow(self, req: Request, upto: int) -> None:
        n = self._blocks_needed(req, upto)
        if n:
            req.blocks.extend(self.pool.allocate(n))

    def _release(self, req: Request, cache: bool = True) -> None:
        if self.radix is not None:
            if cache and req.num_computed > 0:
                toks = req.all_tokens()[: req.num_computed]
                self.radix.insert(toks, req.blocks)
            self.radix.release(req.radix_path)
            req.radix_path = []
        self.pool.free(req.blocks)
        req.blocks = []

    def _preempt(self, victim: Request) -> None:
        self.running.remove(victim)
        n = victim.num_computed
        nb = (n + self.bs - 1) // self.bs
        tier = self.host_tier
        if tier is not None and n > 0 and nb <= len(victim.blocks) and nb <= tier.num_free:
            # swap out: the computed pages go to pinned host memory, nothing is recomputed
            victim.swapped = (tier.spill(victim.blocks[:nb]), n, None)
            self._release(victim, cache=False)
            self.num_swapped_out += 1
        else:
            self._release(victim, cache=True)
            victim.num_computed = 0
            victim.prefill_target = victim.total_len
        victim.num_cached = 0
        victim.status = Status.WAITING
        victim.preempted += 1
        self.num_preemptions += 1
        self.waiting.appendleft(victim)

    def _swap_in(self, req: Request) -> bool:
        """Re-admit a swapped-out sequence: fresh pages, KV copied back from the
        host tier on its copy stream (the next forward gates on it).  A sequence
        ``_prefetch`` already restored one step ahead just takes its pages."""
        slots, n, pre = req.swapped
        if pre is not None:
            blocks = pre
        else:
            nb = len(slots)
            if nb > self.pool.num_free and not self.pool.can_allocate(nb):
                return False
            try:
                blocks = self.pool.allocate(nb)
            except OutOfBlocks:
                return False
            req.kv_ready = self.host_tier.restore(slots, blocks)
            self.host_tier.release(slots)
        req.swapped = None
        req.blocks = blocks
        req.radix_path = []
        req.num_computed = n
        req.status = Status.RUNNING
        self.running.append(req)
        self.num_swapped_in += 1
        return True

    # restores issued one step ahead: at most this many waiting sequences, and only while the
    # pool keeps PREFETCH_RESERVE of its pages free for the running set's growth
    PREFETCH_SEQS = 4
    PREFETCH_RESERVE = 0.05

    def _prefetch(self) -> None:
        """Start the host -> GPU restore of the swapped-out sequences still at the head of the
        waiting queue (the step's budget admitted no more), so the copy overlaps the step about
        to run and their re-admission finds the pages in place (restores one
        step ahead, gated by an event)."""
        tier = self.host_tier
        if tier is None or not self.waiting:
            return
        reserve = int(self.PREFETCH_RESERVE * self.pool.num_blocks)
        for req in list(self.waiting)[: self.PREFETCH_SEQS]:
            if req.swapped is None:
                break                       # FCFS: a prompt ahead of it is admitted first
            slots, n, pre = req.swapped
            if pre is not None:
                continue
            if self.pool.num_free - len(slots) < reserve:
                break
            try:
                blocks = self.pool.allocate(len(slots))
            except OutOfBlocks:
                break
            req.kv_ready = tier.restore(slots, blocks, prefetch=True)
            tier.release(slots)
            req.swapped = (None, n, blocks)

    def on_prefilled(self, req: Request) -> None:
        """A prompt's prefill completed: publish its full pages in the radix cache now (not
        only when the request finishes), so prompts arriving while it decodes share them;
        the request holds the published path locked until it is released."""
        if self.radix is None:
            return
        old = req.radix_path
        req.radix_path = self.radix.insert_locked(req.all_tokens()[: req.num_computed], req.blocks)
        self.radix.release(old)

    # ------------------------------------------------------------------ schedule
    def add_prefilled(self, req: Request, blocks: list[int]) -> None:
        """Adopt a sequence prefilled elsewhere (P/D migration): its KV already
        sits in ``blocks`` and its first token is in ``req.output``."""
        req.blocks = list(blocks)
        req.num_computed = req.total_len - 1
        req.prefill_target = req.num_computed
        req.status = Status.RUNNING
        self.running.append(req)

    def schedule(self, max_seqs: Optional[int] = None, max_tokens: Optional[int] = None,
                 allow_prefill: bool = True, preempt: bool = True) -> ScheduledBatch:
        """Form one batch.  ``max_seqs``/``max_tokens`` bound a pipeline
        microbatch; requests already in flight (``busy``) are skipped.  ``preempt``
        False: a decode row whose next page cannot be allocated waits for a later step
        instead of preempting another sequence (a step scheduled while the previous one
        is still in flight must not release pages that step is using)."""
        budget = self.cfg.max_num_batched_tokens if max_tokens is None else max_tokens
        seq_cap = max_seqs if max_seqs is not None else 1 << 30
        decode: list[Request] = []
        preempted: list[Request] = []
        # 1) decode rows
        bs = self.bs
        for req in self.running:            # a snapshot: preemption may remove entries
            if len(decode) >= seq_cap or budget <= 0:
                break
            if req.busy:
                continue
            pos = req.num_computed  # position of the token being fed (== total_len - 1)
            if pos < req.prefill_target:     # still prefilling
                continue
            if len(req.blocks) * bs > pos:   # fast path: the page for this token exists (a preempted
                decode.append(req)           # request has no pages and takes the slow path)
                budget -= 1
                continue
            if req not in self.running:
                continue
            while True:
                try:
                    self._grow(req, pos + 1)
                    break
                except OutOfBlocks:
                    if not preempt:
                        break
                    victim = next((r for r in reversed(self.running._d) if not r.busy), None)
                    if victim is None:
                        break
                    self._preempt(victim)
                    preempted.append(victim)
                    if victim is req:
                        break
            if req.status is Status.RUNNING and req in self.running and \
                    len(req.blocks) * self.bs > pos:
                decode.append(req)
                budget -= 1
        # 2) prefill chunks: running (partial) first, then waiting
        prefill: list[PrefillChunk] = []
        n_seqs = len(decode)
        if not allow_prefill:
            return ScheduledBatch(decode, prefill, preempted)
        align = self.cfg.token_align
        if align > 0 and budget > 0 and decode:     # mixed steps only: a pure prefill step
            budget = self._aligned_budget(len(decode), budget, align, seq_cap)   # keeps its TTFT
        for req in self.running:
            if budget <= 0 or n_seqs >= seq_cap:
                break
            if req.busy or not req.in_prefill:
                continue
            n = min(req.prefill_target - req.num_computed, budget)
            try:
                self._grow(req, req.num_computed + n)
            except OutOfBlocks:
                break
            prefill.append(PrefillChunk(req, req.num_computed, n, req.num_computed + n == req.prefill_target))
            budget -= n
            n_seqs += 1
        max_running = self.cfg.max_num_seqs if self.admit_cap is None else min(self.cfg.max_num_seqs, self.admit_cap)
        while self.waiting and budget > 0 and len(self.running) < max_running and n_seqs < seq_cap:
            req = self.waiting[0]
            if req.swapped is not None:
                # back in the next step's batch (decode row or its remaining prefill chunk)
                if not self._swap_in(req):
                    break
                self.waiting.popleft()
                continue
            toks = req.all_tokens()
            target = req.prefill_target
            cached_blocks: list[int] = []
            path: list = []
            if self.radix is not None and not req.blocks:
                # keep >= 1 token to compute so the chunk produces logits
                cached_blocks, path = self.radix.match(toks[: target - 1])
                ev = self.radix.take_restore_event()
                if ev is not None:
                    req.kv_ready = ev
            start = len(cached_blocks) * self.bs
            n = min(target - start, budget)
            need = (start + n + self.bs - 1) // self.bs - len(cached_blocks)
            if need > self.pool.num_free and not self.pool.can_allocate(need):
                self._unmatch(req, path, cached_blocks)
                break
            try:
                own = self.pool.allocate(need)
            except OutOfBlocks:
                self._unmatch(req, path, cached_blocks)
                break
            self.waiting.popleft()
            req.blocks = cached_blocks + own
            req.radix_path = path
            req.num_computed = start
            req.num_cached = start
            req.status = Status.RUNNING
            self.running.append(req)
            prefill.append(PrefillChunk(req, start, n, start + n == target))
            budget -= n
            n_seqs += 1
        self._prefetch()
        return ScheduledBatch(decode, prefill, preempted)

    def _unmatch(self, req: Request, path: list, cached_blocks: list) -> None:
        """Undo a prefix match whose admission failed.  Pages it restored from the host tier
        stay GPU-resident in the tree for the next reader, so the compute stream is ordered
        after that restore now (GPU-side wait) rather than by this request's forward."""
        if self.radix is None:
            return
        self.radix.release(path)
        self.pool.free(cached_blocks)
        ev, req.kv_ready = req.kv_ready, None
        if ev is not None:
            import torch
            torch.cuda.current_stream(self.pool.kv.device).wait_event(ev)

    def _aligned_budget(self, nd: int, budget: int, align: int, seq_cap: int) -> int:
        """Prefill budget that ends the step on a multiple of ``align`` rows (see
        SchedulerConfig.token_align); unchanged when the step would not exceed
        one tile or the alignment would leave no prefill at all."""
        avail, n = 0, nd
        for req in self.running:
            if avail >= budget:
                break
            if req.in_prefill and not req.busy and n < seq_cap:
                avail += req.prefill_target - req.num_computed
                n += 1
        room = min(self.cfg.max_num_seqs - len(self.running), seq_cap - n)
        for req in self.waiting:
            if avail >= budget or room <= 0:
                break
            avail += req.prefill_target - req.num_computed
            room -= 1
        rows = nd + min(avail, budget)
        if avail <= 0 or rows <= align:
            return budget
        aligned = rows // align * align
        return aligned - nd if aligned > nd else budget

    # ------------------------------------------------------------------ update
    def finish(self, req: Request, reason: str) -> None:
        req.status = Status.FINISHED
        req.finish_reason = reason
        req.finish_time = time.perf_counter()
        self.running.discard(req)
        self._release(req, cache=True)

    def stats(self) -> dict:
        return {
            "waiting": len(self.waiting),
            "running": len(self.running),
            "free_blocks": self.pool.num_free,
            "used_blocks": self.pool.num_used,
            "preemptions": self.num_preemptions,
            "swapped_out": self.num_swapped_out,
            "swapped_in": self.num_swapped_in,
            "prefix_hit_rate": self.radix.hit_rate() if self.radix else 0.0,
        }
