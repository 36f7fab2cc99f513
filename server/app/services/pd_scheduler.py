"""Prefill/decode (DistServe-style) job scheduler — cluster level.

Same public API as reference server/app/services/pd_scheduler.py:25-479
(``JobPhase``, ``WorkerRole``, ``WorkerCapability``, ``PendingJob``,
``WorkerAssignment``, ``PrefillDecodeScheduler``, ``KVCacheMigrator``).

Changes:
* assignments increment the chosen worker's ``active_*_jobs`` and
  ``complete_job`` releases them, so load balancing actually sees load
  (the reference never incremented them, Appendix E-16);
* prefill placement is FLOP-weighted, decode placement prefers the KV
  holder and otherwise the highest ``bandwidth / (1 + active)`` worker, with
  KV-cache headroom taken into account;
* ``KVCacheMigrator`` performs the transfer through a pluggable async
  ``transport(kv_key, src, dst)`` — inside one MI355X node that is the RCCL
  page migration of ``dgi.parallel.pd`` — instead of ``sleep(0.05)``.
"""
from __future__ import annotations

import asyncio
import heapq
import logging
import time
from dataclasses import dataclass, field
from enum import Enum
from typing import Any, Awaitable, Callable, Dict, List, Optional, Tuple

logger = logging.getLogger(__name__)


class JobPhase(Enum):
    PREFILL = "prefill"
    DECODE = "decode"


class WorkerRole(Enum):
    PREFILL = "prefill"
    DECODE = "decode"
    HYBRID = "hybrid"


@dataclass
class WorkerCapability:
    worker_id: str
    role: WorkerRole = WorkerRole.HYBRID
    compute_flops: float = 0.0           # dense bf16 TFLOPS (MI355X: ~2500)
    memory_bandwidth_gbps: float = 0.0   # HBM GB/s (MI355X: ~8000)
    gpu_memory_gb: float = 0.0
    active_prefill_jobs: int = 0
    active_decode_jobs: int = 0
    kv_cache_tokens_used: int = 0
    kv_cache_tokens_total: int = 0
    prefill_latency_ms: float = 0.0
    decode_latency_ms: float = 0.0
    reliability_score: float = 1.0

    @property
    def prefill_capacity(self) -> float:
        return 0.0 if self.role == WorkerRole.DECODE else self.compute_flops * self.reliability_score

    @property
    def decode_capacity(self) -> float:
        return 0.0 if self.role == WorkerRole.PREFILL else self.memory_bandwidth_gbps * self.reliability_score

    @property
    def kv_cache_utilization(self) -> float:
        return self.kv_cache_tokens_used / self.kv_cache_tokens_total if self.kv_cache_tokens_total else 0.0


@dataclass(order=True)
class PendingJob:
    priority: float
    created_at: float
    job_id: str = field(compare=False)
    phase: JobPhase = field(compare=False)
    prompt_tokens: int = field(compare=False, default=0)
    max_tokens: int = field(compare=False, default=512)
    kv_cache_key: str = field(compare=False, default="")
    kv_cache_worker: str = field(compare=False, default="")
    metadata: Dict[str, Any] = field(compare=False, default_factory=dict)


@dataclass
class WorkerAssignment:
    worker_id: str
    phase: JobPhase
    estimated_latency_ms: float = 0.0
    kv_migration_needed: bool = False
    migration_source: str = ""


class PrefillDecodeScheduler:
    def __init__(self, enable_migration: bool = True, migration_threshold_ms: float = 50.0,
                 prefill_batch_timeout_ms: float = 20.0, decode_batch_timeout_ms: float = 5.0):
        self.enable_migration = enable_migration
        self.migration_threshold_ms = migration_threshold_ms
        self.prefill_batch_timeout_ms = prefill_batch_timeout_ms
        self.decode_batch_timeout_ms = decode_batch_timeout_ms
        self._workers: Dict[str, WorkerCapability] = {}
        self._prefill_queue: List[PendingJob] = []
        self._decode_queue: List[PendingJob] = []
        self._kv_cache_locations: Dict[str, str] = {}
        self._assigned: Dict[Tuple[str, JobPhase], str] = {}
        self._stats = {"prefill_jobs": 0, "decode_jobs": 0, "migrations": 0, "migration_bytes": 0,
                       "avg_prefill_latency_ms": 0.0, "avg_decode_latency_ms": 0.0}

    # ------------------------------------------------------------------ workers
    def register_worker(self, worker_id: str, capability: WorkerCapability) -> None:
        self._workers[worker_id] = capability

    def unregister_worker(self, worker_id: str) -> None:
        self._workers.pop(worker_id, None)
        for k in [k for k, w in self._kv_cache_locations.items() if w == worker_id]:
            del self._kv_cache_locations[k]

    def update_worker_stats(self, worker_id: str, stats: Dict[str, Any]) -> None:
        w = self._workers.get(worker_id)
        if w is None:
            return
        for k in ("active_prefill_jobs", "active_decode_jobs", "kv_cache_tokens_used", "kv_cache_tokens_total",
                  "prefill_latency_ms", "decode_latency_ms", "reliability_score"):
            if k in stats:
                setattr(w, k, stats[k])

    # ------------------------------------------------------------------ jobs
    async def submit_job(self, job_id: str, prompt_tokens: int, max_tokens: int = 512, priority: float = 1.0,
                         metadata: Optional[Dict[str, Any]] = None) -> str:
        heapq.heappush(self._prefill_queue, PendingJob(-priority, time.time(), job_id, JobPhase.PREFILL,
                                                       prompt_tokens, max_tokens, metadata=metadata or {}))
        self._stats["prefill_jobs"] += 1
        return job_id

    async def transition_to_decode(self, job_id: str, kv_cache_key: str, kv_cache_worker: str) -> None:
        # the prefill slot frees up when its KV is handed over
        self._release(job_id, JobPhase.PREFILL)
        heapq.heappush(self._decode_queue, PendingJob(0, time.time(), job_id, JobPhase.DECODE,
                                                      kv_cache_key=kv_cache_key, kv_cache_worker=kv_cache_worker))
        self._kv_cache_locations[kv_cache_key] = kv_cache_worker
        self._stats["decode_jobs"] += 1

    async def complete_job(self, job_id: str, phase: JobPhase = JobPhase.DECODE, latency_ms: float = 0.0) -> None:
        wid = self._release(job_id, phase)
        if wid and latency_ms > 0:
            key = "avg_prefill_latency_ms" if phase == JobPhase.PREFILL else "avg_decode_latency_ms"
            n = self._stats["prefill_jobs" if phase == JobPhase.PREFILL else "decode_jobs"] or 1
            self._stats[key] += (latency_ms - self._stats[key]) / n

    def _release(self, job_id: str, phase: JobPhase) -> Optional[str]:
        wid = self._assigned.pop((job_id, phase), None)
        w = self._workers.get(wid) if wid else None
        if w is not None:
            if phase == JobPhase.PREFILL:
                w.active_prefill_jobs = max(0, w.active_prefill_jobs - 1)
            else:
                w.active_decode_jobs = max(0, w.active_decode_jobs - 1)
        return wid

    async def assign_job(self, job: PendingJob) -> WorkerAssignment:
        a = await (self._assign_prefill(job) if job.phase == JobPhase.PREFILL else self._assign_decode(job))
        w = self._workers[a.worker_id]
        if job.phase == JobPhase.PREFILL:
            w.active_prefill_jobs += 1
        else:
            w.active_decode_jobs += 1
        self._assigned[(job.job_id, job.phase)] = a.worker_id
        return a

    async def _assign_prefill(self, job: PendingJob) -> WorkerAssignment:
        cands = [(w.prefill_capacity / (1 + w.active_prefill_jobs), w) for w in self._workers.values()
                 if w.role in (WorkerRole.PREFILL, WorkerRole.HYBRID) and w.prefill_capacity > 0]
        if not cands:
            raise RuntimeError("No available workers for prefill")
        _, best = max(cands, key=lambda c: c[0])
        return WorkerAssignment(best.worker_id, JobPhase.PREFILL, self._estimate_prefill_latency(best, job.prompt_tokens))

    async def _assign_decode(self, job: PendingJob) -> WorkerAssignment:
        holder = job.kv_cache_worker or self._kv_cache_locations.get(job.kv_cache_key, "")
        hw = self._workers.get(holder) if holder else None
        if hw is not None and hw.role in (WorkerRole.DECODE, WorkerRole.HYBRID) and hw.kv_cache_utilization < 0.95:
            return WorkerAssignment(holder, JobPhase.DECODE, self._estimate_decode_latency(hw))
        cands = [(w.decode_capacity * (1.0 - w.kv_cache_utilization) / (1 + w.active_decode_jobs), w)
                 for w in self._workers.values()
                 if w.role in (WorkerRole.DECODE, WorkerRole.HYBRID) and w.decode_capacity > 0]
        if not cands:
            raise RuntimeError("No available workers for decode")
        _, best = max(cands, key=lambda c: c[0])
        migrate = bool(self.enable_migration and holder and holder != best.worker_id)
        lat = self._estimate_decode_latency(best) + (self.migration_threshold_ms if migrate else 0.0)
        return WorkerAssignment(best.worker_id, JobPhase.DECODE, lat, migrate, holder if migrate else "")

    def _estimate_prefill_latency(self, worker: WorkerCapability, prompt_tokens: int) -> float:
        if worker.prefill_latency_ms > 0:
            return worker.prefill_latency_ms * (prompt_tokens / 512)
        return 100.0 * (prompt_tokens / 512) * (10.0 / max(1.0, worker.compute_flops))

    def _estimate_decode_latency(self, worker: WorkerCapability) -> float:
        if worker.decode_latency_ms > 0:
            return worker.decode_latency_ms
        return 10.0 * (1000.0 / max(1.0, worker.memory_bandwidth_gbps))

    async def get_batch(self, phase: JobPhase, max_batch_size: int = 32) -> List[Tuple[PendingJob, WorkerAssignment]]:
        q = self._prefill_queue if phase == JobPhase.PREFILL else self._decode_queue
        timeout = self.prefill_batch_timeout_ms if phase == JobPhase.PREFILL else self.decode_batch_timeout_ms
        deadline = time.time() + timeout / 1000.0
        batch, failed = [], []
        while q and len(batch) < max_batch_size:
            if batch and time.time() > deadline:
                break
            job = heapq.heappop(q)
            try:
                batch.append((job, await self.assign_job(job)))
            except Exception as e:
                logger.warning("cannot assign %s: %s", job.job_id, e)
                failed.append(job)
                break
        for j in failed:
            heapq.heappush(q, j)
        return batch

    def get_stats(self) -> Dict[str, Any]:
        ws = self._workers.values()
        return {**self._stats, "prefill_queue_size": len(self._prefill_queue),
                "decode_queue_size": len(self._decode_queue), "total_workers": len(self._workers),
                "prefill_workers": sum(w.role in (WorkerRole.PREFILL, WorkerRole.HYBRID) for w in ws),
                "decode_workers": sum(w.role in (WorkerRole.DECODE, WorkerRole.HYBRID) for w in ws),
                "kv_cache_entries": len(self._kv_cache_locations)}


Transport = Callable[[str, str, str], Awaitable[int]]


class KVCacheMigrator:
    """De-duplicated KV migrations through a transport returning bytes moved."""

    def __init__(self, scheduler: PrefillDecodeScheduler, transport: Optional[Transport] = None):
        self.scheduler = scheduler
        self.transport = transport
        self._pending_migrations: Dict[str, asyncio.Task] = {}
        self.latencies_ms: List[float] = []

    async def migrate(self, kv_cache_key: str, source_worker: str, target_worker: str) -> bool:
        mid = f"{kv_cache_key}:{source_worker}:{target_worker}"
        if mid in self._pending_migrations:
            return await asyncio.shield(self._pending_migrations[mid])
        task = asyncio.ensure_future(self._do_migrate(kv_cache_key, source_worker, target_worker))
        self._pending_migrations[mid] = task
        try:
            return await task
        finally:
            self._pending_migrations.pop(mid, None)

    def record(self, kv_cache_key: str, source_worker: str, target_worker: str, nbytes: int,
               latency_ms: float) -> None:
        """Account a migration a synchronous in-node transport already performed
        (dgi.parallel.pd: RCCL page sends from a prefill rank to a decode replica)."""
        self.scheduler._stats["migrations"] += 1
        self.scheduler._stats["migration_bytes"] += int(nbytes)
        self.latencies_ms.append(float(latency_ms))
        if len(self.latencies_ms) > 4096:
            del self.latencies_ms[:2048]

    async def _do_migrate(self, kv_cache_key: str, source_worker: str, target_worker: str) -> bool:
        t0 = time.perf_counter()
        try:
            moved = 0
            if self.transport is not None:
                moved = int(await self.transport(kv_cache_key, source_worker, target_worker) or 0)
            else:
                await asyncio.sleep(0)  # location-only move (same node / shared tier)
            self.scheduler._kv_cache_locations[kv_cache_key] = target_worker
            self.scheduler._stats["migrations"] += 1
            self.scheduler._stats["migration_bytes"] += moved
            self.latencies_ms.append((time.perf_counter() - t0) * 1000)
            return True
        except Exception as e:
            logger.error("KV migration %s failed: %s", kv_cache_key, e)
            return False
