"""Cluster-level prefill/decode job path: the P/D scheduler wired into the control plane.

The reference defines ``PrefillDecodeScheduler`` / ``KVCacheMigrator``
(server/app/services/pd_scheduler.py:106-479) but no entry point ever
instantiates them.  Here one process-wide ``PDCoordinator``
drives them from the pull-based job API:

* workers registering or heart-beating with a P/D role (``prefill`` /
  ``decode`` / ``hybrid``) become scheduler workers; their capabilities
  (``compute_flops``, ``memory_bandwidth_gbps``, KV tokens) come from the
  register payload and the engine stats of each heartbeat;
* a job created with ``params.pd = true`` enters as ``phase = "prefill"``
  (``submit_job``); prefill-role workers pull it (role-aware
  ``SmartScheduler.atomic_assign_job``) and finish it with the first token and
  a ``kv_cache_key``;
* on that completion the coordinator calls ``transition_to_decode`` and the
  scheduler's decode placement (``assign_job``: the KV holder if it can
  decode, else the best decode worker by bandwidth x headroom / load), and
  requeues the job as ``phase = "decode"`` pinned to that worker
  (``target_worker_id``), with ``params.kv_source`` naming the holder when the
  KV has to move and ``params.kv_url`` where to pull it from (``KVCacheMigrator``
  accounts it; inside one MI355X node the move is dgi's RCCL migration, across
  workers the decode worker pulls the exported pages over HTTP —
  dgi/kv/transfer.py — and re-prefills only when they are gone);
* the decode completion releases the scheduler's load accounting.

``/api/v1/admin/pd/stats`` reports ``get_stats()``; the observability
``queue_size{phase}`` gauges are fed from the same numbers.
"""
from __future__ import annotations

import heapq
import logging
import threading
import time
from typing import Any, Dict, Optional

from app.services.pd_scheduler import (JobPhase, KVCacheMigrator, PendingJob, PrefillDecodeScheduler,
                                       WorkerCapability, WorkerRole)

logger = logging.getLogger(__name__)

# defaults when a worker does not report capabilities (one MI355X: ~2.5 PF dense bf16, 8 TB/s)
DEFAULT_TFLOPS = 2500.0
DEFAULT_HBM_GBPS = 8000.0
# decode-job params the coordinator owns (stripped from what the client sent)
CLIENT_STRIP = ("kv_url", "kv_token", "kv_source", "pd_phase", "first_token", "prefill_text", "kv_cache_key")


def _run(coro):
    """The scheduler's bookkeeping coroutines never suspend: run them inline."""
    try:
        coro.send(None)
    except StopIteration as e:
        return e.value
    coro.close()
    raise RuntimeError("P/D scheduler coroutine suspended")


class PDCoordinator:
    def __init__(self):
        self.scheduler = PrefillDecodeScheduler()
        self.migrator = KVCacheMigrator(self.scheduler)
        self._lock = threading.Lock()
        self.transitions = 0
        self.decode_done = 0

    # ------------------------------------------------------------------ workers
    def sync_worker(self, w, engine_stats: Optional[Dict[str, Any]] = None) -> None:
        role = (getattr(w, "role", None) or "hybrid").lower()
        if role not in ("prefill", "decode", "hybrid"):
            role = "hybrid"
        caps = dict(getattr(w, "extra_caps", None) or {})
        n = max(1, int(getattr(w, "gpu_count", 1) or 1))
        with self._lock:
            wid = str(w.id)
            cur = self.scheduler._workers.get(wid)
            cap = WorkerCapability(
                wid, WorkerRole(role),
                compute_flops=float(caps.get("compute_flops", DEFAULT_TFLOPS * n)),
                memory_bandwidth_gbps=float(caps.get("memory_bandwidth_gbps", DEFAULT_HBM_GBPS * n)),
                gpu_memory_gb=float(getattr(w, "gpu_memory_gb", 0.0) or 0.0),
                kv_cache_tokens_total=int(caps.get("kv_cache_tokens_total", 0)),
                reliability_score=float(getattr(w, "reliability_score", 1.0) or 1.0))
            if cur is not None:      # keep live load counters
                cap.active_prefill_jobs, cap.active_decode_jobs = cur.active_prefill_jobs, cur.active_decode_jobs
                cap.kv_cache_tokens_used = cur.kv_cache_tokens_used
            self.scheduler.register_worker(wid, cap)
            if engine_stats:
                bs = int(engine_stats.get("block_size", 16) or 16)
                upd = {}
                if "num_blocks" in engine_stats:
                    upd["kv_cache_tokens_total"] = int(engine_stats["num_blocks"]) * bs
                if "used_blocks" in engine_stats:
                    upd["kv_cache_tokens_used"] = int(engine_stats["used_blocks"]) * bs
                self.scheduler.update_worker_stats(wid, upd)

    def drop_worker(self, worker_id: str) -> None:
        with self._lock:
            self.scheduler.unregister_worker(str(worker_id))

    # ------------------------------------------------------------------ jobs
    @staticmethod
    def wants_pd(params: Optional[dict]) -> bool:
        return bool((params or {}).get("pd"))

    def on_created(self, job) -> None:
        p = job.params or {}
        prompt_tokens = int(p.get("prompt_tokens") or len(str(p.get("prompt", ""))) // 4 or 1)
        with self._lock:
            _run(self.scheduler.submit_job(str(job.id), prompt_tokens, int(p.get("max_tokens", 512)),
                                           priority=float(job.priority or 0) + 1.0))

    def on_assigned(self, job, worker) -> None:
        """A worker pulled a P/D job: count it as that worker's active prefill/decode job."""
        phase = JobPhase.DECODE if job.phase == "decode" else JobPhase.PREFILL
        with self._lock:
            s = self.scheduler
            if phase == JobPhase.PREFILL:
                s._prefill_queue = [j for j in s._prefill_queue if j.job_id != str(job.id)]
                heapq.heapify(s._prefill_queue)
            w = s._workers.get(str(worker.id))
            if w is not None and (str(job.id), phase) not in s._assigned:
                if phase == JobPhase.PREFILL:
                    w.active_prefill_jobs += 1
                s._assigned[(str(job.id), phase)] = str(worker.id)

    def on_prefill_done(self, job, worker, result: Optional[dict], live: Optional[set] = None) -> Dict[str, Any]:
        """Prefill phase finished on ``worker``: choose the decode worker and return
        the fields to requeue the job with (phase, target, kv source).  ``live``:
        ids of the workers currently online; others leave the scheduler first."""
        res = result or {}
        kv_key = str(res.get("kv_cache_key") or f"kv:{job.id}")
        t0 = time.perf_counter()
        with self._lock:
            if live is not None:
                for wid in [w for w in self.scheduler._workers if w not in live]:
                    self.scheduler.unregister_worker(wid)
            _run(self.scheduler.transition_to_decode(str(job.id), kv_key, str(worker.id)))
            pending = PendingJob(0.0, time.time(), str(job.id), JobPhase.DECODE, kv_cache_key=kv_key,
                                 kv_cache_worker=str(worker.id))
            # drop the heap copy transition_to_decode queued: we place this job right now
            self.scheduler._decode_queue = [j for j in self.scheduler._decode_queue if j.job_id != str(job.id)]
            heapq.heapify(self.scheduler._decode_queue)
            try:
                a = _run(self.scheduler.assign_job(pending))
            except RuntimeError:
                a = None
            self.transitions += 1
            if a is not None and a.kv_migration_needed:
                # the byte move itself is the decode worker's (dgi RCCL in-node, re-prefill across nodes)
                self.migrator.record(kv_key, a.migration_source, a.worker_id, int(res.get("kv_bytes", 0)),
                                     (time.perf_counter() - t0) * 1000.0)
        # fields only the coordinator may set: a client-supplied kv_url / kv_token /
        # kv_source never reaches the decode worker
        params = {k: v for k, v in (job.params or {}).items() if k not in CLIENT_STRIP}
        params["pd_phase"] = "decode"
        params["first_token"] = res.get("first_token")
        params["prefill_text"] = res.get("response", "")
        params["kv_cache_key"] = kv_key
        if a is not None and a.kv_migration_needed:
            params["kv_source"] = a.migration_source
            # the decode worker pulls the pages from the prefill worker (dgi.kv.transfer)
            # instead of re-running the prompt, when the prefill worker exported them
            if res.get("kv_url"):
                params["kv_url"] = res["kv_url"]
                if res.get("kv_token"):
                    params["kv_token"] = res["kv_token"]
        return {"phase": "decode", "target_worker_id": a.worker_id if a is not None else None, "params": params,
                "estimated_latency_ms": a.estimated_latency_ms if a is not None else None}

    def on_decode_done(self, job, latency_ms: float = 0.0) -> None:
        with self._lock:
            _run(self.scheduler.complete_job(str(job.id), JobPhase.DECODE, latency_ms))
            self.scheduler._kv_cache_locations.pop(str((job.params or {}).get("kv_cache_key", "")), None)
            self.decode_done += 1

    def on_failed(self, job) -> None:
        with self._lock:
            for ph in (JobPhase.PREFILL, JobPhase.DECODE):
                self.scheduler._release(str(job.id), ph)

    def stats(self) -> Dict[str, Any]:
        with self._lock:
            st = self.scheduler.get_stats()
            lat = self.migrator.latencies_ms
        st.update(transitions=self.transitions, decode_completed=self.decode_done,
                  migration_latency_ms_avg=round(sum(lat) / len(lat), 3) if lat else None)
        return st


coordinator = PDCoordinator()
