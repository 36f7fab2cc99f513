"""Job API (reference server/app/api/jobs.py:76-352).

Submit / sync-wait / get / cancel / direct-connect lookup / queue stats.
``/sync`` waits on the task-guarantee completion event set by the worker's
complete call (no 0.5 s DB polling loop).  Optional ``X-API-Key``
(enterprise key) tags the job for usage metering.
"""
from __future__ import annotations

from datetime import datetime
from typing import Any, Optional

from fastapi import APIRouter, Depends, Header, HTTPException, Query, Request
from pydantic import BaseModel, Field
from sqlalchemy import select
from sqlalchemy.orm import Session

from app.api.deps import lookup_api_key
from app.db.database import get_db
from app.models.models import Job, JobStatus, Worker, WorkerStatus
from app.services.geo import detect_client_region
from app.services.job_signal import job_queued
from app.services.pd_runtime import coordinator
from app.services.scheduler import SmartScheduler, get_region_distance
from app.services.task_guarantee import TaskGuaranteeService

router = APIRouter(prefix="/api/v1/jobs", tags=["jobs"])


class JobCreateRequest(BaseModel):
    type: str = Field(..., description="llm | image_gen | vision | whisper | embedding")
    params: dict
    priority: int = 0
    region: Optional[str] = None
    allow_cross_region: bool = True
    prefer_direct: bool = False
    timeout_seconds: int = 300


class JobResponse(BaseModel):
    job_id: str
    status: str
    result: Optional[Any] = None
    error: Optional[str] = None
    region: Optional[str] = None
    worker_id: Optional[str] = None
    direct_url: Optional[str] = None
    created_at: datetime
    started_at: Optional[datetime] = None
    completed_at: Optional[datetime] = None
    queue_position: Optional[int] = None
    estimated_wait_seconds: Optional[int] = None


class DirectConnectionInfo(BaseModel):
    worker_id: str
    direct_url: str
    region: str
    gpu_model: Optional[str] = None
    reliability_score: float


def _to_response(job: Job, **extra) -> JobResponse:
    return JobResponse(job_id=str(job.id), status=job.status, result=job.result, error=job.error,
                       region=job.actual_region, worker_id=str(job.worker_id) if job.worker_id else None,
                       created_at=job.created_at, started_at=job.started_at, completed_at=job.completed_at, **extra)


def _new_job(db: Session, payload: JobCreateRequest, client_ip, client_region, api_key, priority_boost=0,
             timeout=None) -> Job:
    key = lookup_api_key(db, api_key)
    if key is not None and key.allowed_types and payload.type not in key.allowed_types:
        raise HTTPException(403, f"API key not allowed for job type {payload.type}")
    job = Job(type=payload.type, params=payload.params, priority=payload.priority + priority_boost,
              preferred_region=payload.region if not priority_boost else (payload.region or client_region),
              allow_cross_region=payload.allow_cross_region,
              timeout_seconds=min(payload.timeout_seconds, timeout) if timeout else payload.timeout_seconds,
              client_ip=client_ip, client_region=client_region,
              enterprise_id=key.enterprise_id if key else None, api_key_id=key.id if key else None,
              status=JobStatus.QUEUED.value, created_at=datetime.utcnow())
    pd = payload.type == "llm" and coordinator.wants_pd(payload.params)
    if pd:
        job.phase = "prefill"        # P/D job path (services/pd_runtime.py)
    db.add(job)
    db.commit()
    db.refresh(job)
    if pd:
        coordinator.on_created(job)
    job_queued.notify()          # long-polling workers (GET next-job?wait=) try to claim it now
    return job


@router.post("", response_model=JobResponse)
async def create_job(request: Request, payload: JobCreateRequest, db: Session = Depends(get_db),
                     x_api_key: Optional[str] = Header(None)):
    ip = request.client.host if request.client else None
    region = await detect_client_region(ip)
    job = _new_job(db, payload, ip, region, x_api_key)
    st = SmartScheduler(db).get_queue_stats(region=payload.region)
    return _to_response(job, queue_position=st["total_queued"], estimated_wait_seconds=st["estimated_wait_seconds"])


@router.post("/sync", response_model=JobResponse)
async def create_job_sync(request: Request, payload: JobCreateRequest, timeout: int = Query(60),
                          wait_for_worker: bool = Query(True), db: Session = Depends(get_db),
                          x_api_key: Optional[str] = Header(None)):
    ip = request.client.host if request.client else None
    region = await detect_client_region(ip)
    st = SmartScheduler(db).get_queue_stats(region=payload.region)
    if st["available_workers"] == 0 and not wait_for_worker:
        raise HTTPException(503, detail={"error": "no_workers_available", "message": "no GPU worker is online",
                                         "suggestion": "retry later or set wait_for_worker=true",
                                         "client_region": region})
    job = _new_job(db, payload, ip, region, x_api_key, priority_boost=10, timeout=timeout)
    try:
        done = await TaskGuaranteeService(db).get_job_with_fallback(job.id, True, float(timeout))
    except TimeoutError:
        raise HTTPException(408, detail={"error": "timeout", "message": f"job not finished within {timeout}s",
                                         "job_id": str(job.id)})
    return _to_response(done)


@router.get("/stats/queue")
def get_queue_stats(region: Optional[str] = None, db: Session = Depends(get_db)):
    return SmartScheduler(db).get_queue_stats(region=region)


@router.get("/direct/nearest")
async def get_nearest_worker(request: Request, job_type: str = Query(...), db: Session = Depends(get_db)):
    ip = request.client.host if request.client else None
    region = await detect_client_region(ip)
    ws = [w for w in db.execute(select(Worker).where(Worker.status == WorkerStatus.ONLINE.value,
                                                     Worker.supports_direct.is_(True),
                                                     Worker.direct_url.is_not(None))).scalars()
          if job_type in (w.supported_types or [])]
    if not ws:
        raise HTTPException(503, detail={"error": "no_direct_workers", "message": "no direct-capable worker online"})
    best = min(ws, key=lambda w: (get_region_distance(w.region, region), -(w.reliability_score or 0)))
    return {"worker_id": str(best.id), "direct_url": best.direct_url, "region": best.region,
            "client_region": region, "gpu_model": best.gpu_model, "reliability_score": best.reliability_score}


@router.get("/{job_id}", response_model=JobResponse)
def get_job(job_id: str, db: Session = Depends(get_db)):
    job = db.get(Job, job_id)
    if job is None:
        raise HTTPException(404, "Job not found")
    return _to_response(job)


@router.delete("/{job_id}")
def cancel_job(job_id: str, db: Session = Depends(get_db)):
    job = db.get(Job, job_id)
    if job is None:
        raise HTTPException(404, "Job not found")
    if job.status != JobStatus.QUEUED.value:
        raise HTTPException(400, "only queued jobs can be cancelled")
    job.status = JobStatus.CANCELLED.value
    job.completed_at = datetime.utcnow()
    db.commit()
    from app.services.task_guarantee import notify_job_done
    notify_job_done(job.id)
    return {"message": "Job cancelled", "job_id": job_id}


@router.get("/{job_id}/direct", response_model=DirectConnectionInfo)
def get_direct_connection(job_id: str, db: Session = Depends(get_db)):
    job = db.get(Job, job_id)
    if job is None:
        raise HTTPException(404, "Job not found")
    if not job.worker_id:
        raise HTTPException(400, "job has no worker yet")
    w = db.get(Worker, job.worker_id)
    if w is None:
        raise HTTPException(404, "Worker not found")
    if not w.supports_direct or not w.direct_url:
        raise HTTPException(400, "worker does not support direct connections")
    return DirectConnectionInfo(worker_id=str(w.id), direct_url=w.direct_url, region=w.region,
                                gpu_model=w.gpu_model, reliability_score=w.reliability_score)
