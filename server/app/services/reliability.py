"""Worker reliability scoring and online-time prediction (reference services/reliability.py:15-180).

Same event deltas; the long-session bonus is granted once per 4-hour block
(the reference re-granted it on every heartbeat of a qualifying hour, E-34).
"""
from __future__ import annotations

import logging
from datetime import datetime
from typing import List, Optional

from sqlalchemy import select
from sqlalchemy.orm import Session

from app.models.models import Worker, WorkerStatus

logger = logging.getLogger(__name__)


class ReliabilityService:
    SCORE_JOB_COMPLETED = 0.02
    SCORE_JOB_FAILED = -0.05
    SCORE_UNEXPECTED_OFFLINE = -0.15
    SCORE_GRACEFUL_OFFLINE = -0.02
    SCORE_LONG_SESSION = 0.05
    SCORE_QUICK_RESPONSE = 0.01
    LONG_SESSION_THRESHOLD = 4 * 3600

    def __init__(self, db: Optional[Session] = None):
        self.db = db

    def update_score(self, worker: Worker, event: str, commit: bool = True, **kw) -> None:
        s = worker.reliability_score if worker.reliability_score is not None else 1.0
        if event == "job_completed":
            s = min(1.0, s + self.SCORE_JOB_COMPLETED)
            worker.completed_jobs = (worker.completed_jobs or 0) + 1
            worker.total_jobs = (worker.total_jobs or 0) + 1
        elif event == "job_failed":
            s = max(0.1, s + self.SCORE_JOB_FAILED)
            worker.failed_jobs = (worker.failed_jobs or 0) + 1
            worker.total_jobs = (worker.total_jobs or 0) + 1
        elif event == "unexpected_offline":
            s = max(0.1, s + self.SCORE_UNEXPECTED_OFFLINE)
            worker.unexpected_offline_count = (worker.unexpected_offline_count or 0) + 1
        elif event == "graceful_offline":
            s = max(0.2, s + self.SCORE_GRACEFUL_OFFLINE)
            self._end_session(worker)
        elif event == "long_session":
            s = min(1.0, s + self.SCORE_LONG_SESSION)
        elif event == "heartbeat":
            self._update_online_pattern(worker)
            if worker.current_session_start:
                secs = (datetime.utcnow() - worker.current_session_start).total_seconds()
                blocks = int(secs // self.LONG_SESSION_THRESHOLD)
                pattern = dict(worker.online_pattern or {})
                if blocks > int(pattern.get("_long_blocks", 0)):
                    pattern["_long_blocks"] = blocks
                    worker.online_pattern = pattern
                    s = min(1.0, s + self.SCORE_LONG_SESSION)
        worker.reliability_score = s
        if worker.total_jobs:
            worker.success_rate = (worker.completed_jobs or 0) / worker.total_jobs
        lat = kw.get("latency_ms")
        if lat is not None:
            if lat < 100:
                worker.reliability_score = min(1.0, worker.reliability_score + self.SCORE_QUICK_RESPONSE)
            worker.avg_latency_ms = int(worker.avg_latency_ms * 0.9 + lat * 0.1) if worker.avg_latency_ms else int(lat)
        if commit and self.db is not None:
            self.db.commit()

    def _update_online_pattern(self, worker: Worker) -> None:
        pattern = dict(worker.online_pattern or {str(i): 0.0 for i in range(24)})
        h = str(datetime.utcnow().hour)
        pattern[h] = 0.1 + 0.9 * float(pattern.get(h, 0.0))
        worker.online_pattern = pattern

    def _end_session(self, worker: Worker) -> None:
        if worker.current_session_start:
            secs = (datetime.utcnow() - worker.current_session_start).total_seconds()
            worker.total_online_seconds = (worker.total_online_seconds or 0) + int(secs)
            worker.avg_session_minutes = worker.total_online_seconds / 60 / max(1, worker.total_sessions or 1)
            worker.current_session_start = None

    def start_session(self, worker: Worker, commit: bool = True) -> None:
        worker.current_session_start = datetime.utcnow()
        worker.total_sessions = (worker.total_sessions or 0) + 1
        if commit and self.db is not None:
            self.db.commit()

    def predict_online_probability(self, worker: Worker, hours_ahead: int = 1) -> float:
        if not worker.online_pattern:
            return 0.5
        h = str((datetime.utcnow().hour + hours_ahead) % 24)
        base = float(worker.online_pattern.get(h, 0.5))
        return min(1.0, base * (0.5 + 0.5 * (worker.reliability_score or 0.0)))

    def predict_remaining_online_time(self, worker: Worker) -> float:
        """Minutes the worker is expected to stay online."""
        if not worker.current_session_start:
            return 0.0
        elapsed = (datetime.utcnow() - worker.current_session_start).total_seconds() / 60
        remaining = max(5.0, (worker.avg_session_minutes or 60.0) - elapsed)
        return remaining * (0.5 + 0.5 * (worker.reliability_score or 0.0))

    def get_reliable_workers(self, min_score: float = 0.5, region: Optional[str] = None,
                             job_type: Optional[str] = None) -> List[Worker]:
        q = select(Worker).where(Worker.status.in_([WorkerStatus.ONLINE.value, WorkerStatus.BUSY.value]),
                                 Worker.reliability_score >= min_score)
        if region:
            q = q.where(Worker.region == region)
        ws = list(self.db.execute(q.order_by(Worker.reliability_score.desc())).scalars())
        return [w for w in ws if job_type is None or w.supports(job_type)]
