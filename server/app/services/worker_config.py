"""Server-managed worker configuration (reference services/worker_config.py:20-251).

The remote config is the pydantic ``WorkerRemoteConfig`` (load control,
security, per-type model configs).  Workers fetch it through
``GET /api/v1/workers/{id}/config``; admins edit the ``load_control``
section.  Unlike the reference, ``should_accept_job`` is *enforced*: the
scheduler's ``atomic_assign_job`` consults it (acceptance rate, hourly cap,
working hours, type weights) before handing a worker a job (SURVEY E-33).
"""
from __future__ import annotations

import random
from datetime import datetime
from typing import Any, Dict, List, Optional

from pydantic import BaseModel, Field
from sqlalchemy import func, select
from sqlalchemy.orm import Session

from app.models.models import Job, Worker


class LoadControlConfig(BaseModel):
    acceptance_rate: float = Field(default=1.0, ge=0.0, le=1.0)
    max_concurrent_jobs: int = Field(default=1, ge=1, le=1024)   # a dgi engine batches hundreds of requests
    max_jobs_per_hour: int = Field(default=0, ge=0)               # 0 = unlimited
    max_gpu_memory_percent: float = Field(default=90.0, ge=0.0, le=100.0)
    working_hours_start: Optional[int] = Field(default=None, ge=0, le=23)
    working_hours_end: Optional[int] = Field(default=None, ge=0, le=23)
    type_weights: Dict[str, float] = Field(default_factory=lambda: {
        "llm": 1.0, "image_gen": 1.0, "whisper": 1.0, "embedding": 1.0})
    cooldown_seconds: int = Field(default=0, ge=0)


class SecurityConfig(BaseModel):
    token_validity_hours: int = Field(default=24, ge=1)
    require_https: bool = True
    enable_request_signing: bool = True
    ip_whitelist: List[str] = Field(default_factory=list)
    allow_direct_connection: bool = True


class ModelConfig(BaseModel):
    model_config = {"protected_namespaces": ()}
    model_id: str
    revision: Optional[str] = None
    max_new_tokens: int = 2048
    temperature: float = 0.7
    load_in_8bit: bool = False
    load_in_4bit: bool = False
    extra_params: Dict[str, Any] = Field(default_factory=dict)


class WorkerRemoteConfig(BaseModel):
    model_config = {"protected_namespaces": ()}
    config_version: int = 1
    updated_at: datetime = Field(default_factory=datetime.utcnow)
    load_control: LoadControlConfig = Field(default_factory=LoadControlConfig)
    security: SecurityConfig = Field(default_factory=SecurityConfig)
    model_configs: Dict[str, ModelConfig] = Field(default_factory=dict)
    server_message: Optional[str] = None
    update_required: bool = False
    update_url: Optional[str] = None


def _in_window(hour: int, start: Optional[int], end: Optional[int]) -> bool:
    if start is None or end is None:
        return True
    if start <= end:
        return start <= hour < end
    return hour >= start or hour < end    # window wraps past midnight


def effective_load_control(worker: Worker) -> LoadControlConfig:
    """A worker's load control: the admin override where one is set; otherwise the defaults,
    with the concurrency the worker advertised at registration (``capabilities.
    max_concurrent_jobs``: a continuous-batching engine serves many jobs at once).  A worker
    that advertises nothing keeps the reference's one job at a time."""
    raw = dict((worker.config_override or {}).get("load_control") or {})
    if "max_concurrent_jobs" not in raw:
        adv = (getattr(worker, "extra_caps", None) or {}).get("max_concurrent_jobs")
        if isinstance(adv, int) and adv >= 1:
            raw["max_concurrent_jobs"] = min(adv, 1024)
    try:
        return LoadControlConfig(**raw)
    except Exception:
        return LoadControlConfig()


class WorkerConfigService:
    DEFAULT_MODEL_CONFIGS = {
        "llm": ModelConfig(model_id="llama3-70b", max_new_tokens=2048, temperature=0.7),
        "image_gen": ModelConfig(model_id="black-forest-labs/FLUX.1-schnell", extra_params={"num_inference_steps": 4}),
        "whisper": ModelConfig(model_id="openai/whisper-large-v3"),
        "embedding": ModelConfig(model_id="BAAI/bge-large-zh-v1.5"),
    }

    def __init__(self, db: Session):
        self.db = db

    def get_worker_config(self, worker: Worker) -> WorkerRemoteConfig:
        override = dict(worker.config_override or {})
        lc = effective_load_control(worker)
        sec = SecurityConfig(**(override.get("security") or {}))
        models = {t: self.DEFAULT_MODEL_CONFIGS[t] for t in (worker.supported_types or [])
                  if t in self.DEFAULT_MODEL_CONFIGS}
        for t, mc in (override.get("model_configs") or {}).items():
            models[t] = ModelConfig(**mc)
        cfg = WorkerRemoteConfig(config_version=max(1, worker.config_version or 0), load_control=lc,
                                 security=sec, model_configs=models,
                                 server_message=override.get("server_message"))
        worker.last_config_sync = datetime.utcnow()
        self.db.commit()
        return cfg

    def update_worker_load_config(self, worker: Worker, config: LoadControlConfig) -> WorkerRemoteConfig:
        override = dict(worker.config_override or {})
        override["load_control"] = config.model_dump()
        worker.config_override = override
        worker.config_version = (worker.config_version or 0) + 1
        self.db.commit()
        return self.get_worker_config(worker)

    @staticmethod
    def should_accept_job(config: LoadControlConfig, job_type: str, current_hour_jobs: int = 0,
                          now: Optional[datetime] = None, rng: Optional[random.Random] = None) -> tuple:
        """(accept, reason). Checks working hours, hourly cap, type weight, acceptance rate."""
        now = now or datetime.now()
        if not _in_window(now.hour, config.working_hours_start, config.working_hours_end):
            return False, "outside_working_hours"
        if config.max_jobs_per_hour and current_hour_jobs >= config.max_jobs_per_hour:
            return False, "hourly_limit_reached"
        weight = float(config.type_weights.get(job_type, 1.0))
        if weight <= 0:
            return False, "job_type_disabled"
        p = config.acceptance_rate * min(1.0, weight)
        if p < 1.0 and (rng or random).random() >= p:
            return False, "random_rejection"
        return True, "accepted"

    def get_hourly_job_count(self, worker: Worker) -> int:
        since = datetime.utcnow().replace(minute=0, second=0, microsecond=0)
        q = select(func.count(Job.id)).where(Job.worker_id == worker.id, Job.started_at >= since)
        return int(self.db.execute(q).scalar() or 0)
