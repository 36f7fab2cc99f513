"""Worker API (reference server/app/api/workers.py:188-648).

Registration (token + refresh token + signing secret), heartbeat, pull-style
``next-job`` with atomic conditional-UPDATE assignment, completion (usage
metering + sync-waiter wake-up), graceful / immediate offline, token verify
and refresh, versioned remote config, listing and detail with online
predictions.

MI355X-specific: one worker runs a continuous-batching ``dgi`` engine, so a
worker may hold up to ``load_control.max_concurrent_jobs`` running jobs at
once (the reference allowed exactly one); it is BUSY only at that limit.
"""
from __future__ import annotations

import time
from datetime import datetime
from typing import Any, Dict, List, Optional

from fastapi import APIRouter, Depends, Header, HTTPException, Query, Request
from pydantic import BaseModel, Field
from sqlalchemy import func, select
from sqlalchemy.orm import Session

from app.api.deps import authenticate_worker, check_signature
from app.db.database import get_db
from app.models.models import Job, JobStatus, Worker, WorkerStatus
from app.models.usage import Enterprise
from app.services.pd_runtime import coordinator
from app.services.job_signal import RECHECK_S, job_queued
from app.services.reliability import ReliabilityService
from app.services.scheduler import SmartScheduler
from app.services.security import SecurityService
from app.services.task_guarantee import TaskGuaranteeService, notify_job_done
from app.services.usage import UsageService
from app.services.worker_config import LoadControlConfig, WorkerConfigService

router = APIRouter(prefix="/api/v1/workers", tags=["workers"])


class WorkerRegisterRequest(BaseModel):
    name: Optional[str] = None
    region: str
    country: Optional[str] = None
    city: Optional[str] = None
    timezone: Optional[str] = None
    gpu_model: Optional[str] = None
    gpu_memory_gb: Optional[float] = None
    gpu_count: int = 1
    cpu_cores: Optional[int] = None
    ram_gb: Optional[float] = None
    supported_types: List[str] = []
    direct_url: Optional[str] = None
    supports_direct: bool = False
    # build additions (all optional): identity, P/D role, accelerator capabilities
    machine_id: Optional[str] = None
    hardware_details: Optional[Dict[str, Any]] = None
    role: str = "hybrid"
    capabilities: Optional[Dict[str, Any]] = None


class WorkerRegisterResponse(BaseModel):
    worker_id: str
    token: str
    refresh_token: str
    signing_secret: str
    token_expires_at: datetime
    message: str = "Worker registered successfully"


class HeartbeatRequest(BaseModel):
    status: str = Field(..., description="online | busy | going_offline")
    current_job_id: Optional[str] = None
    gpu_memory_used_gb: Optional[float] = None
    supported_types: Optional[List[str]] = None
    loaded_models: Optional[List[str]] = None
    direct_url: Optional[str] = None
    config_version: int = 0
    engine_stats: Optional[Dict[str, Any]] = None


class HeartbeatResponse(BaseModel):
    status: str = "ok"
    action: Optional[str] = None
    message: Optional[str] = None
    config_changed: bool = False


class JobAssignment(BaseModel):
    job_id: str
    type: str
    params: dict
    timeout_seconds: int = 300
    priority: int = 0


class JobCompleteRequest(BaseModel):
    success: bool
    result: Optional[dict] = None
    error: Optional[str] = None
    processing_time_ms: Optional[int] = None
    usage: Optional[Dict[str, Any]] = None


class RefreshTokenRequest(BaseModel):
    refresh_token: str


class WorkerInfo(BaseModel):
    id: str
    name: Optional[str] = None
    status: str
    region: str
    gpu_model: Optional[str] = None
    gpu_memory_gb: Optional[float] = None
    supported_types: List[str]
    reliability_score: float
    success_rate: float
    total_jobs: int
    supports_direct: bool
    direct_url: Optional[str] = None
    last_heartbeat: Optional[datetime] = None


def _ip(request: Request) -> Optional[str]:
    return request.client.host if request.client else None


def _load_control(w: Worker) -> LoadControlConfig:
    from app.services.worker_config import effective_load_control
    return effective_load_control(w)


def _running(db: Session, worker_id: str) -> int:
    return int(db.execute(select(func.count(Job.id)).where(Job.worker_id == worker_id,
                                                           Job.status == JobStatus.RUNNING.value)).scalar() or 0)


@router.post("/register", response_model=WorkerRegisterResponse)
def register_worker(payload: WorkerRegisterRequest, db: Session = Depends(get_db)):
    w = Worker(name=payload.name, region=payload.region, country=payload.country, city=payload.city,
               timezone=payload.timezone, gpu_model=payload.gpu_model, gpu_memory_gb=payload.gpu_memory_gb,
               gpu_count=payload.gpu_count, cpu_cores=payload.cpu_cores, ram_gb=payload.ram_gb,
               supported_types=list(payload.supported_types), direct_url=payload.direct_url,
               supports_direct=payload.supports_direct, machine_id=payload.machine_id,
               hardware_details=payload.hardware_details, role=payload.role or "hybrid",
               extra_caps=payload.capabilities, status=WorkerStatus.ONLINE.value,
               last_heartbeat=datetime.utcnow(), registered_at=datetime.utcnow())
    sec = SecurityService(db)
    token, refresh = sec.issue_tokens(w)
    db.add(w)
    ReliabilityService(db).start_session(w, commit=False)
    db.commit()
    db.refresh(w)
    coordinator.sync_worker(w)
    return WorkerRegisterResponse(worker_id=str(w.id), token=token, refresh_token=refresh,
                                  signing_secret=w.signing_secret, token_expires_at=w.token_expires_at)


@router.post("/{worker_id}/heartbeat", response_model=HeartbeatResponse)
async def heartbeat(worker_id: str, payload: HeartbeatRequest, request: Request,
                    x_worker_token: Optional[str] = Header(None), db: Session = Depends(get_db)):
    w = authenticate_worker(db, worker_id, x_worker_token, _ip(request))
    await check_signature(request, db, w)
    if w.status != WorkerStatus.GOING_OFFLINE.value or payload.status == WorkerStatus.OFFLINE.value:
        w.status = payload.status
    w.last_heartbeat = datetime.utcnow()
    if w.current_session_start is None:
        ReliabilityService(db).start_session(w, commit=False)
    w.current_job_id = payload.current_job_id or None
    if payload.gpu_memory_used_gb is not None:
        w.gpu_memory_used_gb = payload.gpu_memory_used_gb
    if payload.supported_types:
        w.supported_types = list(payload.supported_types)
    if payload.loaded_models:
        w.loaded_models = list(payload.loaded_models)
    if payload.direct_url:
        w.direct_url = payload.direct_url
    if payload.engine_stats:
        w.extra_caps = {**(w.extra_caps or {}), "engine_stats": payload.engine_stats}
    ReliabilityService(db).update_score(w, "heartbeat", commit=False)
    db.commit()
    coordinator.sync_worker(w, payload.engine_stats)
    changed = (w.config_version or 0) > payload.config_version
    action = "reload_config" if changed else None
    if SecurityService(db).should_refresh_token(w):
        action = action or "refresh_token"
    return HeartbeatResponse(status="ok", action=action, config_changed=changed)


async def _claim(db: Session, request: Request, worker_id: str, token: Optional[str], n: int,
                 wait: float) -> List[JobAssignment]:
    """Up to ``n`` jobs (bounded by the worker's free job slots) claimed in one transaction.
    ``wait`` > 0 long-polls: an empty queue keeps the request open until a job is queued
    (``services/job_signal.py``) or ``wait`` runs out."""
    w = authenticate_worker(db, worker_id, token, _ip(request))
    w.last_heartbeat = datetime.utcnow()
    if w.status in (WorkerStatus.GOING_OFFLINE.value, WorkerStatus.OFFLINE.value):
        db.commit()
        return []
    lc = _load_control(w)
    free = lc.max_concurrent_jobs - _running(db, w.id)
    if free <= 0:
        db.commit()
        return []
    deadline = time.monotonic() + wait
    while True:
        jobs = SmartScheduler(db).atomic_assign_jobs(str(w.id), list(w.supported_types or []), worker=w,
                                                     n=min(n, free))
        if jobs:
            break
        db.commit()
        left = deadline - time.monotonic()
        if left <= 0:
            return []
        await job_queued.wait(min(left, RECHECK_S))
        db.expire_all()
        w = db.get(Worker, w.id)
        if w is None or w.status in (WorkerStatus.GOING_OFFLINE.value, WorkerStatus.OFFLINE.value):
            return []
    w.current_job_id = jobs[-1].id
    w.status = WorkerStatus.BUSY.value if _running(db, w.id) >= lc.max_concurrent_jobs else WorkerStatus.ONLINE.value
    db.commit()
    for job in jobs:
        if job.phase:
            coordinator.on_assigned(job, w)
    return [JobAssignment(job_id=str(job.id), type=job.type, params=job.params or {},
                          timeout_seconds=job.timeout_seconds, priority=job.priority) for job in jobs]


@router.get("/{worker_id}/next-job", response_model=Optional[JobAssignment])
async def get_next_job(worker_id: str, request: Request, x_worker_token: Optional[str] = Header(None),
                       wait: float = Query(0.0, ge=0.0, le=30.0), db: Session = Depends(get_db)):
    """The next job for this worker, or null (``wait``: long-poll seconds, see ``_claim``)."""
    jobs = await _claim(db, request, worker_id, x_worker_token, 1, wait)
    return jobs[0] if jobs else None


@router.get("/{worker_id}/next-jobs", response_model=List[JobAssignment])
async def get_next_jobs(worker_id: str, request: Request, x_worker_token: Optional[str] = Header(None),
                        max_jobs: int = Query(8, ge=1, le=64, alias="max"),
                        wait: float = Query(0.0, ge=0.0, le=30.0), db: Session = Depends(get_db)):
    """Up to ``max`` jobs at once (a burst of queued jobs in one round trip and one commit);
    [] when none.  Not in the reference: its workers use ``next-job``."""
    return await _claim(db, request, worker_id, x_worker_token, max_jobs, wait)


@router.post("/{worker_id}/jobs/{job_id}/complete")
async def complete_job(worker_id: str, job_id: str, payload: JobCompleteRequest, request: Request,
                       x_worker_token: Optional[str] = Header(None), db: Session = Depends(get_db)):
    w = authenticate_worker(db, worker_id, x_worker_token, _ip(request))
    await check_signature(request, db, w)
    job = db.get(Job, job_id)
    if job is None:
        raise HTTPException(404, "Job not found")
    if str(job.worker_id) != str(worker_id):
        raise HTTPException(403, "Not authorized to complete this job")
    if job.status != JobStatus.RUNNING.value:
        return {"status": "ignored", "job_id": job_id, "job_status": job.status}
    if job.phase == "prefill" and payload.success:
        # P/D: the prefill phase is done -> the scheduler places the decode phase
        live = {str(x) for x in db.execute(select(Worker.id).where(Worker.status.in_(
            [WorkerStatus.ONLINE.value, WorkerStatus.BUSY.value]))).scalars()}
        nxt = coordinator.on_prefill_done(job, w, payload.result, live=live | {str(w.id)})
        job.phase, job.target_worker_id, job.params = "decode", nxt["target_worker_id"], nxt["params"]
        job.status, job.worker_id, job.started_at = JobStatus.QUEUED.value, None, None
        if w.current_job_id == job.id:
            w.current_job_id = None
        ReliabilityService(db).update_score(w, "job_completed", commit=False, latency_ms=payload.processing_time_ms)
        db.commit()
        job_queued.notify()
        return {"status": "ok", "job_id": job_id, "next_phase": "decode", "decode_worker": nxt["target_worker_id"]}
    if job.phase:
        if payload.success:
            coordinator.on_decode_done(job, float(payload.processing_time_ms or 0))
        else:
            coordinator.on_failed(job)
    job.status = JobStatus.COMPLETED.value if payload.success else JobStatus.FAILED.value
    job.result, job.error = payload.result, payload.error
    job.completed_at = datetime.utcnow()
    if payload.processing_time_ms:
        job.actual_duration_ms = payload.processing_time_ms
    if w.current_job_id == job.id:
        w.current_job_id = None
    ReliabilityService(db).update_score(w, "job_completed" if payload.success else "job_failed", commit=False,
                                        latency_ms=payload.processing_time_ms)
    db.commit()
    if w.status == WorkerStatus.GOING_OFFLINE.value and _running(db, w.id) == 0:
        TaskGuaranteeService(db).handle_worker_offline(w.id, graceful=True)
    elif w.status == WorkerStatus.BUSY.value and _running(db, w.id) < _load_control(w).max_concurrent_jobs:
        w.status = WorkerStatus.ONLINE.value
        db.commit()
    if payload.success and job.enterprise_id:
        UsageService.record_usage(db, job, worker=w, enterprise=db.get(Enterprise, job.enterprise_id),
                                  usage_details=payload.usage or {})
    notify_job_done(job.id)
    return {"status": "ok", "job_id": job_id}


@router.post("/{worker_id}/going-offline")
def notify_going_offline(worker_id: str, request: Request, finish_current: bool = Query(True),
                         x_worker_token: Optional[str] = Header(None), db: Session = Depends(get_db)):
    w = authenticate_worker(db, worker_id, x_worker_token, _ip(request))
    busy = _running(db, w.id) > 0
    if finish_current and busy:
        w.status = WorkerStatus.GOING_OFFLINE.value
        db.commit()
    else:
        TaskGuaranteeService(db).handle_worker_offline(w.id, graceful=True)
    return {"status": "ok", "message": "Worker marked as going offline", "will_finish_current": finish_current and busy}


@router.post("/{worker_id}/offline")
def notify_offline(worker_id: str, request: Request, x_worker_token: Optional[str] = Header(None),
                   db: Session = Depends(get_db)):
    w = authenticate_worker(db, worker_id, x_worker_token, _ip(request))
    out = TaskGuaranteeService(db).handle_worker_offline(w.id, graceful=True)
    return {"status": "ok", "message": "Worker offline recorded", **out}


@router.post("/{worker_id}/verify")
def verify_credentials(worker_id: str, request: Request, x_worker_token: Optional[str] = Header(None),
                       db: Session = Depends(get_db)):
    try:
        w = authenticate_worker(db, worker_id, x_worker_token, _ip(request))
    except HTTPException:
        return {"valid": False}
    return {"valid": True, "worker_id": str(w.id)}


@router.post("/{worker_id}/refresh-token")
def refresh_token(worker_id: str, payload: RefreshTokenRequest, db: Session = Depends(get_db)):
    w = db.get(Worker, worker_id)
    if w is None:
        raise HTTPException(404, "Worker not found")
    if not w.refresh_token_hash:
        raise HTTPException(400, "No refresh token set")
    toks = SecurityService(db).refresh_tokens(w, payload.refresh_token)
    if toks is None:
        raise HTTPException(401, "Invalid refresh token")
    db.commit()
    return {"token": toks[0], "refresh_token": toks[1], "token_expires_at": w.token_expires_at.isoformat()}


def config_response(db: Session, w: Worker) -> Dict[str, Any]:
    cfg = WorkerConfigService(db).get_worker_config(w)
    return {"version": w.config_version or 0, "load_control": cfg.load_control.model_dump(),
            "model_configs": {k: v.model_dump() for k, v in cfg.model_configs.items()},
            "security": {"require_signature": bool((w.config_override or {}).get("require_signature", False)),
                         **cfg.security.model_dump()},
            "server_message": cfg.server_message}


def merge_config(db: Session, w: Worker, update: Dict[str, Any]) -> int:
    """Merge a config update; flat load-control keys (reference shape) go under ``load_control``."""
    cur = dict(w.config_override or {})
    lc = dict(cur.get("load_control") or {})
    for k, v in update.items():
        if k == "load_control" and isinstance(v, dict):
            lc.update(v)
        elif k in LoadControlConfig.model_fields:
            lc.update({k: v})
        else:
            cur[k] = v
    LoadControlConfig(**lc)   # validate
    cur["load_control"] = lc
    w.config_override = cur
    w.config_version = (w.config_version or 0) + 1
    db.commit()
    return w.config_version


@router.get("/{worker_id}/config")
def get_worker_config(worker_id: str, request: Request, x_worker_token: Optional[str] = Header(None),
                      db: Session = Depends(get_db)):
    w = authenticate_worker(db, worker_id, x_worker_token, _ip(request))
    return config_response(db, w)


@router.put("/{worker_id}/config")
def update_worker_config(worker_id: str, config: Dict[str, Any], request: Request,
                         x_worker_token: Optional[str] = Header(None), db: Session = Depends(get_db)):
    w = authenticate_worker(db, worker_id, x_worker_token, _ip(request))
    try:
        v = merge_config(db, w, config)
    except Exception as e:
        raise HTTPException(422, f"invalid config: {e}")
    return {"status": "ok", "config_version": v}


@router.get("", response_model=List[WorkerInfo])
def list_workers(region: Optional[str] = None, status: Optional[str] = None, db: Session = Depends(get_db)):
    q = select(Worker)
    if region:
        q = q.where(Worker.region == region)
    if status:
        q = q.where(Worker.status == status)
    ws = db.execute(q.order_by(Worker.reliability_score.desc())).scalars().all()
    return [WorkerInfo(id=str(w.id), name=w.name, status=w.status, region=w.region, gpu_model=w.gpu_model,
                       gpu_memory_gb=w.gpu_memory_gb, supported_types=w.supported_types or [],
                       reliability_score=w.reliability_score, success_rate=w.success_rate,
                       total_jobs=w.total_jobs or 0, supports_direct=bool(w.supports_direct),
                       direct_url=w.direct_url, last_heartbeat=w.last_heartbeat) for w in ws]


def worker_detail(db: Session, w: Worker) -> Dict[str, Any]:
    rel = ReliabilityService(db)
    return {
        "id": str(w.id), "name": w.name, "machine_id": w.machine_id, "status": w.status, "region": w.region,
        "country": w.country, "city": w.city, "gpu_model": w.gpu_model, "gpu_memory_gb": w.gpu_memory_gb,
        "gpu_count": w.gpu_count, "role": w.role, "supported_types": w.supported_types,
        "loaded_models": w.loaded_models, "reliability_score": w.reliability_score, "success_rate": w.success_rate,
        "unexpected_offline_count": w.unexpected_offline_count,
        "total_online_hours": (w.total_online_seconds or 0) / 3600, "avg_session_minutes": w.avg_session_minutes,
        "total_sessions": w.total_sessions, "online_pattern": w.online_pattern, "total_jobs": w.total_jobs,
        "completed_jobs": w.completed_jobs, "failed_jobs": w.failed_jobs, "avg_latency_ms": w.avg_latency_ms,
        "running_jobs": _running(db, w.id), "supports_direct": w.supports_direct, "direct_url": w.direct_url,
        "predicted_online_1h": rel.predict_online_probability(w, 1),
        "predicted_online_4h": rel.predict_online_probability(w, 4),
        "predicted_remaining_minutes": rel.predict_remaining_online_time(w),
        "last_heartbeat": w.last_heartbeat, "registered_at": w.registered_at,
        "engine_stats": (w.extra_caps or {}).get("engine_stats"),
    }


@router.get("/{worker_id}")
def get_worker(worker_id: str, db: Session = Depends(get_db)):
    w = db.get(Worker, worker_id)
    if w is None:
        raise HTTPException(404, "Worker not found")
    return worker_detail(db, w)
