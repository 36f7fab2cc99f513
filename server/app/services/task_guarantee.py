"""Task guarantee: requeue on worker loss, stale-job and dead-worker sweeps
(reference services/task_guarantee.py:17-263).

``get_job_with_fallback`` waits on an in-process completion event (set by the
complete endpoint) instead of only polling the DB every 0.5 s.
"""
from __future__ import annotations

import asyncio
import logging
from datetime import datetime, timedelta
from typing import Dict, Optional

from sqlalchemy import select
from sqlalchemy.orm import Session

from app.config import settings
from app.models.models import Job, JobStatus, Worker, WorkerStatus
from app.services.job_signal import job_queued
from app.services.reliability import ReliabilityService

logger = logging.getLogger(__name__)

_completion_events: Dict[str, asyncio.Event] = {}


def notify_job_done(job_id: str) -> None:
    ev = _completion_events.get(job_id)
    if ev is not None:
        try:
            loop = ev._loop if hasattr(ev, "_loop") and ev._loop else None
            if loop is not None and loop.is_running():
                loop.call_soon_threadsafe(ev.set)
            else:
                ev.set()
        except Exception:
            ev.set()


class TaskGuaranteeService:
    STALE_JOB_MINUTES = 30

    def __init__(self, db: Session):
        self.db = db
        self.reliability = ReliabilityService(db)

    def handle_worker_offline(self, worker_id: str, graceful: bool = False) -> dict:
        w = self.db.get(Worker, worker_id)
        jobs = list(self.db.execute(select(Job).where(Job.worker_id == worker_id,
                                                      Job.status == JobStatus.RUNNING.value)).scalars())
        requeued = failed = 0
        for j in jobs:
            if (j.retry_count or 0) < (j.max_retries or 3):
                j.status = JobStatus.QUEUED.value
                j.retry_count = (j.retry_count or 0) + 1
                j.worker_id = None
                j.started_at = None
                j.target_worker_id = None      # a P/D decode pin dies with its worker
                requeued += 1
            else:
                j.status = JobStatus.FAILED.value
                j.error = "worker went offline; retries exhausted"
                j.completed_at = datetime.utcnow()
                failed += 1
                notify_job_done(j.id)
        # unpin queued P/D decode phases waiting for this worker, and drop it from the P/D scheduler
        for j in self.db.execute(select(Job).where(Job.target_worker_id == worker_id,
                                                   Job.status == JobStatus.QUEUED.value)).scalars():
            j.target_worker_id = None
        from app.services.pd_runtime import coordinator
        coordinator.drop_worker(worker_id)
        if w is not None:
            w.status = WorkerStatus.OFFLINE.value
            w.current_job_id = None
            self.reliability.update_score(w, "graceful_offline" if graceful else "unexpected_offline", commit=False)
        self.db.commit()
        if requeued:
            job_queued.notify()
        return {"requeued": requeued, "failed": failed}

    def check_stale_jobs(self) -> int:
        now = datetime.utcnow()
        n = requeued = 0
        for j in self.db.execute(select(Job).where(Job.status == JobStatus.RUNNING.value)).scalars():
            limit = max(self.STALE_JOB_MINUTES * 60, j.timeout_seconds or settings.job_timeout_seconds)
            if j.started_at and (now - j.started_at).total_seconds() > limit:
                if (j.retry_count or 0) < (j.max_retries or 3):
                    j.status, j.worker_id, j.started_at = JobStatus.QUEUED.value, None, None
                    j.retry_count = (j.retry_count or 0) + 1
                    requeued += 1
                else:
                    j.status, j.error, j.completed_at = JobStatus.TIMEOUT.value, "job timed out", now
                    notify_job_done(j.id)
                n += 1
        self.db.commit()
        if requeued:
            job_queued.notify()
        return n

    def check_dead_workers(self, timeout_seconds: Optional[int] = None) -> int:
        cutoff = datetime.utcnow() - timedelta(seconds=timeout_seconds or settings.heartbeat_timeout_seconds)
        dead = [w.id for w in self.db.execute(select(Worker).where(
            Worker.status.in_([WorkerStatus.ONLINE.value, WorkerStatus.BUSY.value]))).scalars()
            if w.last_heartbeat is None or w.last_heartbeat < cutoff]
        for wid in dead:
            self.handle_worker_offline(wid, graceful=False)
        return len(dead)

    async def get_job_with_fallback(self, job_id: str, wait_if_running: bool = True,
                                    max_wait_seconds: float = 60.0) -> Job:
        ev = _completion_events.setdefault(job_id, asyncio.Event())
        deadline = asyncio.get_running_loop().time() + max_wait_seconds
        try:
            while True:
                self.db.expire_all()
                job = self.db.get(Job, job_id)
                if job is None:
                    raise KeyError(job_id)
                if job.status in (JobStatus.COMPLETED.value, JobStatus.FAILED.value, JobStatus.CANCELLED.value,
                                  JobStatus.TIMEOUT.value) or not wait_if_running:
                    return job
                left = deadline - asyncio.get_running_loop().time()
                if left <= 0:
                    raise TimeoutError(job_id)
                try:
                    await asyncio.wait_for(ev.wait(), min(0.5, left))
                except asyncio.TimeoutError:
                    pass
                ev.clear()
        finally:
            _completion_events.pop(job_id, None)


class TaskGuaranteeBackgroundWorker:
    def __init__(self, session_factory, interval: Optional[int] = None):
        self.session_factory = session_factory
        self.interval = interval or settings.stale_job_check_interval
        self._running = False

    async def start(self) -> None:
        self._running = True
        while self._running:
            try:
                await asyncio.to_thread(self.run_once)
            except Exception:
                logger.exception("task guarantee sweep failed")
            await asyncio.sleep(self.interval)

    def run_once(self) -> dict:
        db = self.session_factory()
        try:
            svc = TaskGuaranteeService(db)
            return {"dead_workers": svc.check_dead_workers(), "stale_jobs": svc.check_stale_jobs()}
        finally:
            db.close()

    def stop(self) -> None:
        self._running = False
