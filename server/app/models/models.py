"""Core ORM: workers, jobs (schema reconstructed per SURVEY Appendix D)."""
from __future__ import annotations

import enum
import uuid
from dataclasses import dataclass, field
from datetime import datetime
from typing import Dict

from sqlalchemy import JSON, Boolean, DateTime, Float, ForeignKey, Integer, String, Text, func
from sqlalchemy.orm import Mapped, mapped_column

from app.db.database import Base


def _uuid() -> str:
    return str(uuid.uuid4())


class WorkerStatus(str, enum.Enum):
    ONLINE = "online"
    BUSY = "busy"
    OFFLINE = "offline"
    GOING_OFFLINE = "going_offline"


class JobStatus(str, enum.Enum):
    QUEUED = "queued"
    RUNNING = "running"
    COMPLETED = "completed"
    FAILED = "failed"
    CANCELLED = "cancelled"
    TIMEOUT = "timeout"


class Worker(Base):
    __tablename__ = "workers"
    id: Mapped[str] = mapped_column(String(36), primary_key=True, default=_uuid)
    name: Mapped[str | None] = mapped_column(String(128))
    machine_id: Mapped[str | None] = mapped_column(String(128), index=True)
    hardware_hash: Mapped[str | None] = mapped_column(String(128))
    hardware_details: Mapped[dict | None] = mapped_column(JSON)
    status: Mapped[str] = mapped_column(String(32), default=WorkerStatus.OFFLINE.value, index=True)
    region: Mapped[str] = mapped_column(String(64), default="asia-east", index=True)
    country: Mapped[str | None] = mapped_column(String(64))
    city: Mapped[str | None] = mapped_column(String(64))
    timezone: Mapped[str | None] = mapped_column(String(64))
    gpu_model: Mapped[str | None] = mapped_column(String(128))
    gpu_memory_gb: Mapped[float | None] = mapped_column(Float)
    gpu_memory_used_gb: Mapped[float | None] = mapped_column(Float)
    gpu_count: Mapped[int] = mapped_column(Integer, default=1)
    cpu_cores: Mapped[int | None] = mapped_column(Integer)
    ram_gb: Mapped[float | None] = mapped_column(Float)
    supported_types: Mapped[list] = mapped_column(JSON, default=list)
    loaded_models: Mapped[list] = mapped_column(JSON, default=list)
    direct_url: Mapped[str | None] = mapped_column(String(256))
    supports_direct: Mapped[bool] = mapped_column(Boolean, default=False)
    auth_token_hash: Mapped[str | None] = mapped_column(String(256))
    refresh_token_hash: Mapped[str | None] = mapped_column(String(256))
    signing_secret: Mapped[str | None] = mapped_column(String(128))
    token_expires_at: Mapped[datetime | None] = mapped_column(DateTime)
    failed_auth_attempts: Mapped[int] = mapped_column(Integer, default=0)
    last_failed_auth: Mapped[datetime | None] = mapped_column(DateTime)
    locked_until: Mapped[datetime | None] = mapped_column(DateTime)
    current_job_id: Mapped[str | None] = mapped_column(String(36))
    reliability_score: Mapped[float] = mapped_column(Float, default=1.0)
    success_rate: Mapped[float] = mapped_column(Float, default=1.0)
    total_jobs: Mapped[int] = mapped_column(Integer, default=0)
    completed_jobs: Mapped[int] = mapped_column(Integer, default=0)
    failed_jobs: Mapped[int] = mapped_column(Integer, default=0)
    avg_latency_ms: Mapped[int | None] = mapped_column(Integer)
    unexpected_offline_count: Mapped[int] = mapped_column(Integer, default=0)
    total_online_seconds: Mapped[int] = mapped_column(Integer, default=0)
    total_sessions: Mapped[int] = mapped_column(Integer, default=0)
    avg_session_minutes: Mapped[float | None] = mapped_column(Float)
    current_session_start: Mapped[datetime | None] = mapped_column(DateTime)
    online_pattern: Mapped[dict | None] = mapped_column(JSON)
    config_override: Mapped[dict | None] = mapped_column(JSON)
    config_version: Mapped[int] = mapped_column(Integer, default=0)
    last_config_sync: Mapped[datetime | None] = mapped_column(DateTime)
    last_heartbeat: Mapped[datetime | None] = mapped_column(DateTime)
    registered_at: Mapped[datetime] = mapped_column(DateTime, default=datetime.utcnow)
    # build-only additions: P/D role and accelerator capabilities for the pd scheduler
    role: Mapped[str] = mapped_column(String(16), default="hybrid")
    extra_caps: Mapped[dict | None] = mapped_column(JSON)
    jobs_this_hour: Mapped[int] = mapped_column(Integer, default=0)
    hour_bucket: Mapped[int] = mapped_column(Integer, default=-1)

    def supports(self, job_type: str) -> bool:
        return job_type in (self.supported_types or [])


class Job(Base):
    __tablename__ = "jobs"
    id: Mapped[str] = mapped_column(String(36), primary_key=True, default=_uuid)
    type: Mapped[str] = mapped_column(String(32), index=True)
    status: Mapped[str] = mapped_column(String(32), default=JobStatus.QUEUED.value, index=True)
    priority: Mapped[int] = mapped_column(Integer, default=0, index=True)
    params: Mapped[dict] = mapped_column(JSON, default=dict)
    result: Mapped[dict | None] = mapped_column(JSON)
    error: Mapped[str | None] = mapped_column(Text)
    preferred_region: Mapped[str | None] = mapped_column(String(64))
    actual_region: Mapped[str | None] = mapped_column(String(64))
    allow_cross_region: Mapped[bool] = mapped_column(Boolean, default=True)
    worker_id: Mapped[str | None] = mapped_column(String(36), ForeignKey("workers.id"), index=True)
    timeout_seconds: Mapped[int] = mapped_column(Integer, default=300)
    retry_count: Mapped[int] = mapped_column(Integer, default=0)
    max_retries: Mapped[int] = mapped_column(Integer, default=3)
    client_ip: Mapped[str | None] = mapped_column(String(64))
    client_region: Mapped[str | None] = mapped_column(String(64))
    enterprise_id: Mapped[str | None] = mapped_column(String(36))
    api_key_id: Mapped[str | None] = mapped_column(String(36))
    phase: Mapped[str | None] = mapped_column(String(16))   # P/D: prefill | decode
    # P/D: the decode phase is pinned to the worker the P/D scheduler chose (services/pd_runtime.py)
    target_worker_id: Mapped[str | None] = mapped_column(String(36), index=True)
    created_at: Mapped[datetime] = mapped_column(DateTime, default=datetime.utcnow, index=True)
    started_at: Mapped[datetime | None] = mapped_column(DateTime)
    completed_at: Mapped[datetime | None] = mapped_column(DateTime)
    actual_duration_ms: Mapped[int | None] = mapped_column(Integer)


@dataclass
class QueueStats:
    total_queued: int = 0
    by_type: Dict[str, int] = field(default_factory=dict)
    available_workers: int = 0
    estimated_wait_seconds: int = -1
