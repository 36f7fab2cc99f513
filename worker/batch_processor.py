"""Job-level admission batching in front of an engine.

API-compatible with the reference's ``worker/batch_processor.py``
(``ContinuousBatcher``, ``AdaptiveBatcher``, ``PendingRequest``,
``RequestPriority``).  Role in this framework: the worker's
*admission* front-end.  It groups concurrently arriving jobs (priority
order, optional grouping by shared system prompt so prefix-cache hits land
together) and hands each group to the engine's batch API.  With the native
MI355X engine the group goes straight into the iteration-level scheduler
(``dgi.sched``), which re-forms the real GPU batch every decode step.

Execution preference: ``batch_inference_async`` -> ``batch_inference`` in a
thread -> per-request ``inference_async`` / ``inference``.
"""
from __future__ import annotations

import asyncio
import hashlib
import heapq
import logging
import time
from collections import defaultdict
from dataclasses import dataclass, field
from enum import Enum
from typing import Any, Dict, List, Optional

logger = logging.getLogger(__name__)


class RequestPriority(Enum):
    HIGH = 0
    NORMAL = 1
    LOW = 2


@dataclass(order=True)
class PendingRequest:
    priority: int
    timestamp: float
    job_id: str = field(compare=False)
    params: Dict[str, Any] = field(compare=False)
    future: Any = field(compare=False)
    prefix_hash: str = field(compare=False, default="")

    @classmethod
    def create(cls, job_id: str, params: Dict[str, Any], priority: RequestPriority = RequestPriority.NORMAL,
               prefix_hash: str = "") -> "PendingRequest":
        loop = asyncio.get_event_loop()
        return cls(priority.value, time.time(), job_id, params, loop.create_future(), prefix_hash)


class ContinuousBatcher:
    def __init__(self, engine, max_batch_size: int = 32, max_wait_ms: float = 50,
                 enable_prefix_grouping: bool = True, max_queue_size: int = 1000):
        self.engine = engine
        self.max_batch_size = max_batch_size
        self.max_wait_ms = max_wait_ms
        self.enable_prefix_grouping = enable_prefix_grouping
        self.max_queue_size = max_queue_size
        self._pending: List[PendingRequest] = []          # heap ordered by (priority, timestamp)
        self._pending_by_prefix: Dict[str, List[PendingRequest]] = defaultdict(list)
        self._lock = asyncio.Lock()
        self._wakeup: Optional[asyncio.Event] = None
        self._batch_task: Optional[asyncio.Task] = None
        self._inflight: set = set()
        self._running = False
        self._stats = {"total_requests": 0, "total_batches": 0, "avg_batch_size": 0.0, "avg_wait_time_ms": 0.0,
                       "timeouts": 0, "errors": 0}

    # ------------------------------------------------------------------ lifecycle
    async def start(self) -> None:
        self._running = True
        self._wakeup = asyncio.Event()
        self._batch_task = asyncio.create_task(self._dispatch_loop())

    async def stop(self) -> None:
        self._running = False
        async with self._lock:
            for r in self._pending:
                if not r.future.done():
                    r.future.cancel()
            self._pending.clear()
            self._pending_by_prefix.clear()
        if self._wakeup is not None:
            self._wakeup.set()
        for t in [self._batch_task, *self._inflight]:
            if t is not None and not t.done():
                t.cancel()
                try:
                    await t
                except (asyncio.CancelledError, Exception):
                    pass
        self._batch_task = None
        self._inflight.clear()

    # ------------------------------------------------------------------ submit
    async def submit(self, job_id: str, params: Dict[str, Any], priority: RequestPriority = RequestPriority.NORMAL,
                     timeout: Optional[float] = None) -> Dict[str, Any]:
        if not self._running:
            raise RuntimeError("Batcher is not running")
        async with self._lock:
            if len(self._pending) >= self.max_queue_size:
                raise RuntimeError(f"Queue full ({self.max_queue_size})")
            prefix = self._compute_prefix_hash(params) if self.enable_prefix_grouping else ""
            req = PendingRequest(priority.value, time.time(), job_id, params,
                                 asyncio.get_running_loop().create_future(), prefix)
            heapq.heappush(self._pending, req)
            if prefix:
                self._pending_by_prefix[prefix].append(req)
            self._stats["total_requests"] += 1
        if self._wakeup is not None:
            self._wakeup.set()
        try:
            if timeout is None:
                return await req.future
            return await asyncio.wait_for(asyncio.shield(req.future), timeout)
        except asyncio.TimeoutError:
            self._stats["timeouts"] += 1
            async with self._lock:
                self._remove(req)
            if not req.future.done():
                req.future.cancel()
            raise

    def _remove(self, req: PendingRequest) -> None:
        if req in self._pending:
            self._pending.remove(req)
            heapq.heapify(self._pending)
        if req.prefix_hash and req in self._pending_by_prefix.get(req.prefix_hash, []):
            self._pending_by_prefix[req.prefix_hash].remove(req)
            if not self._pending_by_prefix[req.prefix_hash]:
                del self._pending_by_prefix[req.prefix_hash]

    # ------------------------------------------------------------------ dispatch
    async def _dispatch_loop(self) -> None:
        while self._running:
            if not self._pending:
                self._wakeup.clear()
                await self._wakeup.wait()
                continue
            oldest = min(r.timestamp for r in self._pending)
            wait = self.max_wait_ms / 1000.0 - (time.time() - oldest)
            if len(self._pending) < self.max_batch_size and wait > 0:
                self._wakeup.clear()
                try:
                    await asyncio.wait_for(self._wakeup.wait(), wait)
                except asyncio.TimeoutError:
                    pass
                if len(self._pending) < self.max_batch_size and \
                        time.time() - min((r.timestamp for r in self._pending), default=time.time()) \
                        < self.max_wait_ms / 1000.0:
                    continue
            await self._process_batch()

    async def _process_batch(self) -> None:
        async with self._lock:
            batch = self._select_batch_with_prefix_grouping() if self.enable_prefix_grouping \
                else self._select_batch_fifo()
            for r in batch:
                self._remove(r)
        batch = [r for r in batch if not r.future.done()]
        if not batch:
            return
        now = time.time()
        n = self._stats["total_batches"]
        self._stats["avg_batch_size"] = (self._stats["avg_batch_size"] * n + len(batch)) / (n + 1)
        wait_ms = sum((now - r.timestamp) * 1000 for r in batch) / len(batch)
        self._stats["avg_wait_time_ms"] = (self._stats["avg_wait_time_ms"] * n + wait_ms) / (n + 1)
        self._stats["total_batches"] = n + 1
        task = asyncio.create_task(self._run_batch(batch))
        self._inflight.add(task)
        task.add_done_callback(self._inflight.discard)

    async def _run_batch(self, batch: List[PendingRequest]) -> None:
        t0 = time.time()
        try:
            results = await self._execute_batch([r.params for r in batch])
        except Exception as e:
            self._stats["errors"] += 1
            for r in batch:
                if not r.future.done():
                    r.future.set_exception(e)
            return
        for r, res in zip(batch, results):
            if r.future.done():
                continue
            if isinstance(res, BaseException):
                r.future.set_exception(res)
            else:
                r.future.set_result(res)
        self._on_batch_done(len(batch), (time.time() - t0) * 1000)

    def _on_batch_done(self, size: int, latency_ms: float) -> None:
        pass

    def _select_batch_fifo(self) -> List[PendingRequest]:
        return heapq.nsmallest(self.max_batch_size, self._pending)

    def _select_batch_with_prefix_grouping(self) -> List[PendingRequest]:
        """Largest shared-prefix groups first (their KV prefix is computed once),
        then fill by priority order."""
        chosen: List[PendingRequest] = []
        seen = set()
        groups = sorted(self._pending_by_prefix.values(), key=len, reverse=True)
        for g in groups:
            if len(g) < 2:
                continue
            for r in g:
                if len(chosen) >= self.max_batch_size:
                    break
                chosen.append(r)
                seen.add(id(r))
        for r in sorted(self._pending):
            if len(chosen) >= self.max_batch_size:
                break
            if id(r) not in seen:
                chosen.append(r)
                seen.add(id(r))
        return chosen

    async def _execute_batch(self, params_list: List[Dict[str, Any]]) -> List[Any]:
        eng = self.engine
        if hasattr(eng, "batch_inference_async"):
            return list(await eng.batch_inference_async(params_list))
        loop = asyncio.get_running_loop()
        if hasattr(eng, "batch_inference"):
            return list(await loop.run_in_executor(None, eng.batch_inference, params_list))
        if hasattr(eng, "inference_async"):
            return list(await asyncio.gather(*[eng.inference_async(p) for p in params_list],
                                             return_exceptions=True))
        out = []
        for p in params_list:
            try:
                out.append(await loop.run_in_executor(None, eng.inference, p))
            except Exception as e:  # per-request failure
                out.append(e)
        return out

    def _compute_prefix_hash(self, params: Dict[str, Any]) -> str:
        """Group key = the system messages (shared prompt prefix)."""
        sys_parts = [m.get("content", "") for m in params.get("messages", []) if m.get("role") == "system"]
        if not sys_parts:
            return ""
        return hashlib.sha256("\x00".join(sys_parts).encode()).hexdigest()[:16]

    def get_stats(self) -> Dict[str, Any]:
        return {**self._stats, "queue_size": len(self._pending), "prefix_groups": len(self._pending_by_prefix),
                "running": self._running, "inflight_batches": len(self._inflight)}


class AdaptiveBatcher(ContinuousBatcher):
    """Moves the batch size toward ``target_latency_ms`` (x0.8 / x1.2 steps)."""

    def __init__(self, engine, min_batch_size: int = 1, max_batch_size: int = 64, target_latency_ms: float = 1000,
                 **kw):
        super().__init__(engine, max_batch_size=max_batch_size, **kw)
        self.min_batch_size = min_batch_size
        self.max_batch_size_limit = max_batch_size
        self.target_latency_ms = target_latency_ms
        self._current_batch_size = max(min_batch_size, min(max_batch_size, max_batch_size // 2 or 1))
        self._latency_history: List[float] = []

    def _on_batch_done(self, size: int, latency_ms: float) -> None:
        self._latency_history.append(latency_ms)
        self._latency_history = self._latency_history[-10:]
        if len(self._latency_history) >= 10:
            self._adapt_batch_size()

    def _adapt_batch_size(self) -> None:
        if not self._latency_history:
            return
        avg = sum(self._latency_history[-10:]) / len(self._latency_history[-10:])
        if avg > self.target_latency_ms * 1.1:
            self._current_batch_size = max(self.min_batch_size, int(self._current_batch_size * 0.8))
        elif avg < self.target_latency_ms * 0.9:
            self._current_batch_size = min(self.max_batch_size_limit, max(self._current_batch_size + 1,
                                                                          int(self._current_batch_size * 1.2)))
        self.max_batch_size = self._current_batch_size

    def get_stats(self) -> Dict[str, Any]:
        s = super().get_stats()
        s["current_batch_size"] = self._current_batch_size
        s["avg_latency_ms"] = (sum(self._latency_history) / len(self._latency_history)) if self._latency_history else 0.0
        return s
