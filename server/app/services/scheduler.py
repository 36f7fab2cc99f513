"""Smart job scheduler: region-, reliability- and role-aware assignment
(reference services/scheduler.py:18-280).

``atomic_assign_job`` (what the pull API uses) claims one queued job with a
conditional UPDATE (``... WHERE id=? AND status='queued'``), which is atomic
on SQLite and Postgres alike; among the top candidate jobs it prefers ones
matching the worker's region and P/D role, and it enforces the worker's
acceptance rate / hourly cap from its remote config (reference E-33, E-35).
"""
from __future__ import annotations

import logging
from datetime import datetime
from typing import List, Optional

from sqlalchemy import or_, select, update
from sqlalchemy.orm import Session

from app.models.models import Job, JobStatus, QueueStats, Worker, WorkerStatus
from app.services.reliability import ReliabilityService

logger = logging.getLogger(__name__)

REGIONS = ["asia-east", "asia-south", "europe-west", "europe-east", "america-north", "america-south", "oceania"]
REGION_DISTANCES = {
    ("asia-east", "asia-south"): 1, ("asia-east", "europe-west"): 3, ("asia-east", "europe-east"): 2,
    ("america-north", "asia-east"): 3, ("america-south", "asia-east"): 4, ("asia-east", "oceania"): 2,
    ("asia-south", "europe-west"): 3, ("asia-south", "oceania"): 2, ("europe-east", "europe-west"): 1,
    ("america-north", "europe-west"): 2, ("america-north", "europe-east"): 3, ("america-north", "america-south"): 2,
}


def get_region_distance(a: str, b: str) -> int:
    if not a or not b or a == b:
        return 0 if a == b else 4
    return REGION_DISTANCES.get(tuple(sorted((a, b))), 4)


JOB_BASE_MINUTES = {"llm": 0.5, "image_gen": 2.0, "whisper": 3.0, "embedding": 0.2, "vision": 0.5, "custom": 1.0}


class SmartScheduler:
    WEIGHT_RELIABILITY = 35
    WEIGHT_REGION = 25
    WEIGHT_PREDICTED_ONLINE = 20
    WEIGHT_PERFORMANCE = 15
    WEIGHT_LOAD = 5

    def __init__(self, db: Session):
        self.db = db
        self.reliability_service = ReliabilityService(db)

    # ------------------------------------------------------------------ push-style assignment
    def _available_workers(self, job: Job) -> List[Worker]:
        q = select(Worker).where(Worker.status == WorkerStatus.ONLINE.value)
        if job.preferred_region and not job.allow_cross_region:
            q = q.where(Worker.region == job.preferred_region)
        return [w for w in self.db.execute(q).scalars() if w.supports(job.type)]

    def _calculate_worker_score(self, worker: Worker, job: Job) -> float:
        score = (worker.reliability_score or 0.0) * self.WEIGHT_RELIABILITY
        target = job.preferred_region or job.client_region
        if target:
            score += (5 - get_region_distance(worker.region, target)) / 5 * self.WEIGHT_REGION
        else:
            score += self.WEIGHT_REGION * 0.5
        need = self._estimate_job_duration(job)
        online = self.reliability_service.predict_remaining_online_time(worker)
        if online > 2 * need:
            score += self.WEIGHT_PREDICTED_ONLINE
        elif online > need:
            score += self.WEIGHT_PREDICTED_ONLINE * 0.7
        elif online > 0.5 * need:
            score += self.WEIGHT_PREDICTED_ONLINE * 0.3
        mem = worker.gpu_memory_gb
        # full marks at 288 GB (MI355X); consumer GPUs score proportionally
        score += (min(mem / 288.0, 1.0) if mem else 0.3) * self.WEIGHT_PERFORMANCE
        score += self.WEIGHT_LOAD if worker.status == WorkerStatus.ONLINE.value else self.WEIGHT_LOAD * 0.2
        return score

    def _estimate_job_duration(self, job: Job) -> float:
        base = JOB_BASE_MINUTES.get(job.type, 1.0)
        p = job.params or {}
        if job.type == "llm":
            base *= p.get("max_tokens", 1000) / 1000
        elif job.type == "image_gen":
            base *= (p.get("steps", 20) / 20) * (p.get("width", 1024) * p.get("height", 1024) / 1024 ** 2)
        return base

    def assign_job(self, job: Job) -> Optional[Worker]:
        ws = self._available_workers(job)
        if not ws:
            return None
        best = max(ws, key=lambda w: self._calculate_worker_score(w, job))
        job.worker_id = best.id
        job.status = JobStatus.RUNNING.value
        job.started_at = datetime.utcnow()
        job.actual_region = best.region
        best.status = WorkerStatus.BUSY.value
        best.current_job_id = job.id
        self.db.commit()
        return best

    # ------------------------------------------------------------------ pull-style (atomic) assignment
    def _accepts(self, worker: Optional[Worker], job_type: str = "llm") -> bool:
        """Enforce the worker's remote load-control config (acceptance rate, hourly cap, working hours)."""
        if worker is None:
            return True
        from app.services.worker_config import WorkerConfigService, effective_load_control
        lc = effective_load_control(worker)
        hour = int(datetime.utcnow().timestamp() // 3600)
        if worker.hour_bucket != hour:
            worker.hour_bucket, worker.jobs_this_hour = hour, 0
        ok, _ = WorkerConfigService.should_accept_job(lc, job_type, worker.jobs_this_hour or 0)
        return ok

    def atomic_assign_job(self, worker_id: str, supported_types: List[str], worker: Optional[Worker] = None,
                          candidates: int = 8) -> Optional[Job]:
        jobs = self.atomic_assign_jobs(worker_id, supported_types, worker, 1, candidates)
        return jobs[0] if jobs else None

    def atomic_assign_jobs(self, worker_id: str, supported_types: List[str], worker: Optional[Worker] = None,
                           n: int = 1, candidates: int = 8) -> List[Job]:
        """Claim up to ``n`` queued jobs for the worker in one transaction (one commit: a burst of
        jobs reaches a worker in one round trip instead of one claim + commit each).  Each claim is
        a conditional UPDATE on QUEUED, so concurrent claimers never share a job."""
        if not supported_types or n <= 0:
            return []
        q = (select(Job).where(Job.status == JobStatus.QUEUED.value, Job.type.in_(list(supported_types)),
                               or_(Job.target_worker_id.is_(None), Job.target_worker_id == str(worker_id)))
             .order_by(Job.priority.desc(), Job.created_at.asc()).limit(max(candidates, 2 * n)))
        jobs = list(self.db.execute(q).scalars())
        if worker is not None and (worker.role or "hybrid") in ("prefill", "decode"):
            # a P/D-phase job only goes to a worker of that role (or a hybrid one)
            jobs = [j for j in jobs if not j.phase or j.phase == worker.role]
        if worker is not None and jobs:
            top = jobs[0].priority
            role = (worker.role or "hybrid")

            def pref(j: Job):
                region_ok = (not j.preferred_region) or j.preferred_region == worker.region
                phase_ok = role == "hybrid" or (j.phase or "prefill") == role or j.phase is None
                return (j.priority < top, not phase_ok, not region_ok, j.created_at)
            jobs.sort(key=pref)
        got: List[Job] = []
        for job in jobs:
            if len(got) >= n:
                break
            if not self._accepts(worker, job.type):
                break
            if worker is not None and job.preferred_region and not job.allow_cross_region \
                    and job.preferred_region != worker.region:
                continue
            now = datetime.utcnow()
            res = self.db.execute(update(Job).where(Job.id == job.id, Job.status == JobStatus.QUEUED.value)
                                  .values(status=JobStatus.RUNNING.value, worker_id=worker_id, started_at=now,
                                          actual_region=worker.region if worker is not None else None))
            if res.rowcount == 1:
                got.append(job)
                if worker is not None:
                    worker.current_job_id = job.id
                    worker.jobs_this_hour = (worker.jobs_this_hour or 0) + 1
        self.db.commit()       # the claims (and the hour-bucket roll-over) in one transaction
        for job in got:
            self.db.refresh(job)
        return got

    def get_queue_stats(self, region: Optional[str] = None) -> dict:
        q = select(Job).where(Job.status == JobStatus.QUEUED.value)
        if region:
            q = q.where(or_(Job.preferred_region == region, Job.preferred_region.is_(None)))
        queued = list(self.db.execute(q).scalars())
        by_type: dict = {}
        for j in queued:
            by_type[j.type] = by_type.get(j.type, 0) + 1
        wq = select(Worker).where(Worker.status == WorkerStatus.ONLINE.value)
        if region:
            wq = wq.where(Worker.region == region)
        workers = len(list(self.db.execute(wq).scalars()))
        st = QueueStats(len(queued), by_type, workers, self._estimate_wait_time(len(queued), workers))
        return {"total_queued": st.total_queued, "by_type": st.by_type, "available_workers": st.available_workers,
                "estimated_wait_seconds": st.estimated_wait_seconds}

    @staticmethod
    def _estimate_wait_time(queued: int, workers: int) -> int:
        if workers == 0:
            return -1
        return int(queued / max(1, workers) * 30)
