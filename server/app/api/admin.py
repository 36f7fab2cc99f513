"""Admin API (reference server/app/api/admin.py:74-988).

Dashboard, realtime view, detailed health, worker management, enterprises
and API keys (``ent_`` prefix, sha256 at rest), usage records / grouped
summaries, bills, and the privacy endpoints (settings, compliance,
retention, cleanup, export, right-to-be-forgotten delete, scheduled
cleanup).  Guarded by ``X-Admin-Token`` when ``ADMIN_TOKEN`` is set.
"""
from __future__ import annotations

import secrets
from collections import defaultdict
from datetime import datetime, timedelta
from typing import Any, Dict, List, Optional

from fastapi import APIRouter, Depends, HTTPException, Query
from pydantic import BaseModel, Field
from sqlalchemy import func, select, text
from sqlalchemy.orm import Session

from app.api.deps import hash_api_key, require_admin
from app.api.workers import config_response, merge_config, worker_detail
from app.db.database import get_db
from app.models.models import Job, JobStatus, Worker, WorkerStatus
from app.models.usage import Bill, Enterprise, EnterpriseAPIKey, UsageRecord
from app.services.privacy import EnterprisePrivacyService
from app.services.usage import UsageService

router = APIRouter(prefix="/api/v1/admin", tags=["admin"], dependencies=[Depends(require_admin)])


class EnterpriseCreate(BaseModel):
    name: str
    code: str
    contact_name: Optional[str] = None
    contact_email: Optional[str] = None
    contact_phone: Optional[str] = None
    billing_email: Optional[str] = None
    billing_period: str = "monthly"
    monthly_budget: Optional[float] = None
    data_retention_days: int = 30
    allow_logging: bool = True
    anonymize_data: bool = False


class EnterpriseUpdate(BaseModel):
    name: Optional[str] = None
    contact_name: Optional[str] = None
    contact_email: Optional[str] = None
    monthly_budget: Optional[float] = None
    credit_balance: Optional[float] = None
    is_active: Optional[bool] = None
    allow_logging: Optional[bool] = None
    anonymize_data: Optional[bool] = None
    custom_pricing: Optional[Dict[str, float]] = None
    price_plan_id: Optional[str] = None


class APIKeyCreate(BaseModel):
    name: str
    allowed_types: List[str] = []
    allowed_models: List[str] = []
    rate_limit_per_minute: int = 60
    daily_limit: Optional[int] = None
    ip_whitelist: List[str] = []
    expires_days: Optional[int] = None


class DashboardStats(BaseModel):
    workers: dict
    enterprises: dict
    today: dict
    this_month: dict
    timestamp: str


class PrivacySettingsUpdate(BaseModel):
    data_retention_days: Optional[int] = Field(None, ge=7, le=365)
    allow_logging: Optional[bool] = None
    anonymize_data: Optional[bool] = None
    private_deployment: Optional[bool] = None


def _iso(d: Optional[datetime]) -> Optional[str]:
    return d.isoformat() if d else None


def _enterprise_or_404(db: Session, enterprise_id: str) -> Enterprise:
    e = db.get(Enterprise, enterprise_id)
    if e is None:
        raise HTTPException(404, "Enterprise not found")
    return e


# ---------------------------------------------------------------- dashboard
@router.get("/dashboard", response_model=DashboardStats)
def get_dashboard_stats(db: Session = Depends(get_db)):
    return UsageService.get_platform_stats(db)


@router.get("/dashboard/realtime")
def get_realtime_stats(db: Session = Depends(get_db)):
    ws = db.execute(select(Worker).where(Worker.status.in_(["online", "busy"]))).scalars().all()
    running = db.execute(select(Job).where(Job.status == JobStatus.RUNNING.value)).scalars().all()
    queued = db.execute(select(func.count(Job.id)).where(Job.status == JobStatus.QUEUED.value)).scalar() or 0
    now = datetime.utcnow()
    return {
        "timestamp": now.isoformat(),
        "workers": {"online": sum(w.status == "online" for w in ws), "busy": sum(w.status == "busy" for w in ws),
                    "details": [{"id": str(w.id), "name": w.name, "machine_id": w.machine_id, "status": w.status,
                                 "region": w.region, "gpu_model": w.gpu_model, "gpu_memory_gb": w.gpu_memory_gb,
                                 "gpu_memory_used_gb": w.gpu_memory_used_gb,
                                 "current_job": str(w.current_job_id) if w.current_job_id else None,
                                 "reliability_score": w.reliability_score,
                                 "last_heartbeat": _iso(w.last_heartbeat)} for w in ws]},
        "jobs": {"running": len(running), "queued": int(queued),
                 "details": [{"id": str(j.id), "type": j.type, "worker_id": j.worker_id,
                              "started_at": _iso(j.started_at),
                              "duration_seconds": (now - j.started_at).total_seconds() if j.started_at else 0}
                             for j in running]},
    }


@router.get("/health/detailed")
def get_admin_health_detailed(db: Session = Depends(get_db)):
    try:
        db.execute(text("SELECT 1"))
        db_ok = True
    except Exception:
        db_ok = False
    cutoff = datetime.utcnow() - timedelta(minutes=5)
    stale = db.execute(select(func.count(Worker.id)).where(Worker.status.in_(["online", "busy"]),
                                                           Worker.last_heartbeat < cutoff)).scalar() or 0
    stuck = db.execute(select(func.count(Job.id)).where(Job.status == JobStatus.RUNNING.value,
                                                        Job.started_at < datetime.utcnow() - timedelta(hours=1))
                       ).scalar() or 0
    issues = []
    if not db_ok:
        issues.append("database_unreachable")
    if stale:
        issues.append(f"{stale} workers with stale heartbeat")
    if stuck:
        issues.append(f"{stuck} jobs running > 1h")
    return {"status": "healthy" if not issues else "degraded", "database": db_ok, "stale_workers": int(stale),
            "stuck_jobs": int(stuck), "issues": issues, "timestamp": datetime.utcnow().isoformat()}


# ---------------------------------------------------------------- P/D scheduler
@router.get("/pd/stats")
def get_pd_stats():
    """Cluster P/D scheduler state (services/pd_runtime.py): queues, workers per role,
    migrations; also exported as the ``queue_size{phase}`` gauges."""
    from app.services.observability import MetricsCollector
    from app.services.pd_runtime import coordinator
    st = coordinator.stats()
    mc = MetricsCollector(worker_id="control-plane")
    mc.record_queue("prefill", st["prefill_queue_size"])
    mc.record_queue("decode", st["decode_queue_size"])
    return st


# ---------------------------------------------------------------- workers
@router.get("/workers")
def list_workers(status: Optional[str] = None, region: Optional[str] = None, page: int = Query(1, ge=1),
                 page_size: int = Query(20, ge=1, le=200), db: Session = Depends(get_db)):
    q = select(Worker)
    if status:
        q = q.where(Worker.status == status)
    if region:
        q = q.where(Worker.region == region)
    total = db.execute(select(func.count()).select_from(q.subquery())).scalar() or 0
    ws = db.execute(q.order_by(Worker.registered_at.desc()).offset((page - 1) * page_size).limit(page_size)
                    ).scalars().all()
    return {"total": int(total), "page": page, "page_size": page_size,
            "items": [{"id": str(w.id), "name": w.name, "machine_id": w.machine_id, "status": w.status,
                       "region": w.region, "gpu_model": w.gpu_model, "gpu_memory_gb": w.gpu_memory_gb,
                       "gpu_count": w.gpu_count, "role": w.role, "supported_types": w.supported_types,
                       "reliability_score": w.reliability_score, "total_jobs": w.total_jobs,
                       "success_rate": w.success_rate, "last_heartbeat": _iso(w.last_heartbeat),
                       "registered_at": _iso(w.registered_at)} for w in ws]}


@router.get("/workers/{worker_id}")
def get_worker_detail(worker_id: str, db: Session = Depends(get_db)):
    w = db.get(Worker, worker_id)
    if w is None:
        raise HTTPException(404, "Worker not found")
    out = worker_detail(db, w)
    out["recent_jobs"] = [{"id": j.id, "type": j.type, "status": j.status, "created_at": _iso(j.created_at),
                           "duration_ms": j.actual_duration_ms}
                          for j in db.execute(select(Job).where(Job.worker_id == w.id)
                                              .order_by(Job.created_at.desc()).limit(20)).scalars()]
    out["config"] = config_response(db, w)
    return out


@router.get("/workers/{worker_id}/usage")
def get_worker_usage(worker_id: str, days: int = Query(30, ge=1, le=365), db: Session = Depends(get_db)):
    if db.get(Worker, worker_id) is None:
        raise HTTPException(404, "Worker not found")
    return UsageService.get_worker_usage(db, worker_id, datetime.utcnow() - timedelta(days=days))


@router.put("/workers/{worker_id}/config")
def update_worker_config(worker_id: str, config: Dict[str, Any], db: Session = Depends(get_db)):
    w = db.get(Worker, worker_id)
    if w is None:
        raise HTTPException(404, "Worker not found")
    try:
        v = merge_config(db, w, config)
    except Exception as e:
        raise HTTPException(422, f"invalid config: {e}")
    return {"status": "ok", "config_version": v}


# ---------------------------------------------------------------- enterprises
def _enterprise_dict(e: Enterprise) -> Dict[str, Any]:
    return {"id": str(e.id), "name": e.name, "code": e.code, "contact_name": e.contact_name,
            "contact_email": e.contact_email, "contact_phone": e.contact_phone, "billing_email": e.billing_email,
            "billing_period": e.billing_period, "currency": e.currency, "credit_balance": e.credit_balance,
            "monthly_budget": e.monthly_budget, "price_plan_id": e.price_plan_id,
            "custom_pricing": e.custom_pricing or {}, "data_retention_days": e.data_retention_days,
            "allow_logging": e.allow_logging, "anonymize_data": e.anonymize_data,
            "private_deployment": e.private_deployment, "is_active": e.is_active, "is_verified": e.is_verified,
            "created_at": _iso(e.created_at)}


@router.get("/enterprises")
def list_enterprises(is_active: Optional[bool] = None, search: Optional[str] = None, page: int = Query(1, ge=1),
                     page_size: int = Query(20, ge=1, le=200), db: Session = Depends(get_db)):
    q = select(Enterprise)
    if is_active is not None:
        q = q.where(Enterprise.is_active.is_(is_active))
    if search:
        q = q.where(Enterprise.name.contains(search) | Enterprise.code.contains(search))
    total = db.execute(select(func.count()).select_from(q.subquery())).scalar() or 0
    es = db.execute(q.order_by(Enterprise.created_at.desc()).offset((page - 1) * page_size).limit(page_size)
                    ).scalars().all()
    return {"total": int(total), "page": page, "page_size": page_size, "items": [_enterprise_dict(e) for e in es]}


@router.post("/enterprises")
def create_enterprise(payload: EnterpriseCreate, db: Session = Depends(get_db)):
    if db.execute(select(Enterprise).where(Enterprise.code == payload.code)).scalar_one_or_none() is not None:
        raise HTTPException(400, "Enterprise code already exists")
    e = Enterprise(**payload.model_dump(), created_at=datetime.utcnow())
    db.add(e)
    db.commit()
    db.refresh(e)
    return {"id": str(e.id), "code": e.code, "message": "Enterprise created"}


@router.get("/enterprises/{enterprise_id}")
def get_enterprise_detail(enterprise_id: str, db: Session = Depends(get_db)):
    e = _enterprise_or_404(db, enterprise_id)
    out = _enterprise_dict(e)
    out["api_keys_count"] = db.execute(select(func.count(EnterpriseAPIKey.id)).where(
        EnterpriseAPIKey.enterprise_id == e.id)).scalar() or 0
    out["usage_30d"] = UsageService.get_enterprise_usage(db, e.id)
    return out


@router.put("/enterprises/{enterprise_id}")
def update_enterprise(enterprise_id: str, payload: EnterpriseUpdate, db: Session = Depends(get_db)):
    e = _enterprise_or_404(db, enterprise_id)
    for k, v in payload.model_dump(exclude_none=True).items():
        setattr(e, k, v)
    db.commit()
    return {"status": "ok", "id": str(e.id)}


@router.get("/enterprises/{enterprise_id}/usage")
def get_enterprise_usage(enterprise_id: str, start_date: Optional[datetime] = None,
                         end_date: Optional[datetime] = None, db: Session = Depends(get_db)):
    _enterprise_or_404(db, enterprise_id)
    return UsageService.get_enterprise_usage(db, enterprise_id, start_date, end_date)


@router.post("/enterprises/{enterprise_id}/api-keys")
def create_api_key(enterprise_id: str, payload: APIKeyCreate, db: Session = Depends(get_db)):
    _enterprise_or_404(db, enterprise_id)
    raw = "ent_" + secrets.token_urlsafe(32)
    k = EnterpriseAPIKey(enterprise_id=enterprise_id, name=payload.name, key_hash=hash_api_key(raw),
                         key_prefix=raw[:12], allowed_types=payload.allowed_types,
                         allowed_models=payload.allowed_models, rate_limit_per_minute=payload.rate_limit_per_minute,
                         daily_limit=payload.daily_limit, ip_whitelist=payload.ip_whitelist,
                         expires_at=(datetime.utcnow() + timedelta(days=payload.expires_days))
                         if payload.expires_days else None, created_at=datetime.utcnow())
    db.add(k)
    db.commit()
    return {"id": str(k.id), "api_key": raw, "key_prefix": k.key_prefix, "expires_at": _iso(k.expires_at),
            "message": "store this key now; it cannot be shown again"}


@router.get("/enterprises/{enterprise_id}/api-keys")
def list_api_keys(enterprise_id: str, db: Session = Depends(get_db)):
    _enterprise_or_404(db, enterprise_id)
    ks = db.execute(select(EnterpriseAPIKey).where(EnterpriseAPIKey.enterprise_id == enterprise_id)
                    .order_by(EnterpriseAPIKey.created_at.desc())).scalars().all()
    return [{"id": str(k.id), "name": k.name, "key_prefix": k.key_prefix, "allowed_types": k.allowed_types,
             "rate_limit_per_minute": k.rate_limit_per_minute, "daily_limit": k.daily_limit,
             "is_active": k.is_active, "total_requests": k.total_requests, "last_used_at": _iso(k.last_used_at),
             "expires_at": _iso(k.expires_at), "created_at": _iso(k.created_at)} for k in ks]


# ---------------------------------------------------------------- usage
def _record_dict(r: UsageRecord) -> Dict[str, Any]:
    return {"id": str(r.id), "enterprise_id": r.enterprise_id, "worker_id": r.worker_id, "job_id": r.job_id,
            "usage_type": r.usage_type, "job_type": r.job_type, "model_id": r.model_id, "quantity": r.quantity,
            "unit": r.unit, "unit_price": r.unit_price, "total_cost": r.total_cost, "gpu_seconds": r.gpu_seconds,
            "duration_ms": r.duration_ms, "worker_region": r.worker_region, "client_region": r.client_region,
            "created_at": _iso(r.created_at)}


@router.get("/usage/records")
def list_usage_records(enterprise_id: Optional[str] = None, worker_id: Optional[str] = None,
                       usage_type: Optional[str] = None, start_time: Optional[datetime] = None,
                       end_time: Optional[datetime] = None, page: int = Query(1, ge=1),
                       page_size: int = Query(50, ge=1, le=500), db: Session = Depends(get_db)):
    q = select(UsageRecord)
    for col, val in ((UsageRecord.enterprise_id, enterprise_id), (UsageRecord.worker_id, worker_id),
                     (UsageRecord.usage_type, usage_type)):
        if val:
            q = q.where(col == val)
    if start_time:
        q = q.where(UsageRecord.created_at >= start_time)
    if end_time:
        q = q.where(UsageRecord.created_at <= end_time)
    total = db.execute(select(func.count()).select_from(q.subquery())).scalar() or 0
    rs = db.execute(q.order_by(UsageRecord.created_at.desc()).offset((page - 1) * page_size).limit(page_size)
                    ).scalars().all()
    return {"total": int(total), "page": page, "page_size": page_size, "items": [_record_dict(r) for r in rs]}


@router.get("/usage/summary")
def get_usage_summary(group_by: str = Query("day", pattern="^(hour|day|week|month|worker|enterprise|region|type)$"),
                      start_time: Optional[datetime] = None, end_time: Optional[datetime] = None,
                      db: Session = Depends(get_db)):
    end = end_time or datetime.utcnow()
    start = start_time or end - timedelta(days=30)
    rs = db.execute(select(UsageRecord).where(UsageRecord.created_at >= start, UsageRecord.created_at <= end)
                    ).scalars().all()

    def key(r: UsageRecord) -> str:
        t = r.created_at
        return {"hour": lambda: t.strftime("%Y-%m-%d %H:00"), "day": lambda: t.strftime("%Y-%m-%d"),
                "week": lambda: f"{t.isocalendar()[0]}-W{t.isocalendar()[1]:02d}",
                "month": lambda: t.strftime("%Y-%m"), "worker": lambda: r.worker_id or "unknown",
                "enterprise": lambda: r.enterprise_id or "none", "region": lambda: r.worker_region or "unknown",
                "type": lambda: r.usage_type}[group_by]()
    groups: Dict[str, Dict[str, float]] = defaultdict(lambda: {"count": 0, "quantity": 0.0, "cost": 0.0,
                                                               "gpu_seconds": 0.0})
    for r in rs:
        g = groups[key(r)]
        g["count"] += 1
        g["quantity"] += r.quantity or 0.0
        g["cost"] += r.total_cost or 0.0
        g["gpu_seconds"] += r.gpu_seconds or 0.0
    items = [{"key": k, **{m: (round(v, 6) if isinstance(v, float) else v) for m, v in g.items()}}
             for k, g in sorted(groups.items())]
    return {"group_by": group_by, "start_time": start.isoformat(), "end_time": end.isoformat(), "items": items,
            "totals": {"count": len(rs), "cost": round(sum(r.total_cost or 0 for r in rs), 6),
                       "gpu_hours": round(sum(r.gpu_seconds or 0 for r in rs) / 3600, 4)}}


# ---------------------------------------------------------------- bills
def _bill_dict(b: Bill) -> Dict[str, Any]:
    return {"id": str(b.id), "enterprise_id": b.enterprise_id, "billing_period": b.billing_period,
            "period_start": _iso(b.period_start), "period_end": _iso(b.period_end), "subtotal": b.subtotal,
            "discount": b.discount, "tax": b.tax, "total": b.total, "currency": b.currency, "status": b.status,
            "paid_at": _iso(b.paid_at), "invoice_number": b.invoice_number, "created_at": _iso(b.created_at),
            "due_at": _iso(b.due_at)}


@router.get("/bills")
def list_bills(enterprise_id: Optional[str] = None, status: Optional[str] = None, page: int = Query(1, ge=1),
               page_size: int = Query(20, ge=1, le=200), db: Session = Depends(get_db)):
    q = select(Bill)
    if enterprise_id:
        q = q.where(Bill.enterprise_id == enterprise_id)
    if status:
        q = q.where(Bill.status == status)
    total = db.execute(select(func.count()).select_from(q.subquery())).scalar() or 0
    bs = db.execute(q.order_by(Bill.created_at.desc()).offset((page - 1) * page_size).limit(page_size)
                    ).scalars().all()
    return {"total": int(total), "page": page, "page_size": page_size, "items": [_bill_dict(b) for b in bs]}


@router.get("/bills/{bill_id}")
def get_bill_detail(bill_id: str, db: Session = Depends(get_db)):
    b = db.get(Bill, bill_id)
    if b is None:
        raise HTTPException(404, "Bill not found")
    out = _bill_dict(b)
    out["usage_summary"] = b.usage_summary
    e = db.get(Enterprise, b.enterprise_id)
    out["enterprise"] = {"id": e.id, "name": e.name, "code": e.code} if e else None
    return out


# ---------------------------------------------------------------- privacy
@router.get("/enterprises/{enterprise_id}/privacy")
def get_enterprise_privacy_settings(enterprise_id: str, db: Session = Depends(get_db)):
    s = EnterprisePrivacyService(db).get_enterprise_privacy_settings(enterprise_id)
    if not s:
        raise HTTPException(404, "Enterprise not found")
    return s


@router.put("/enterprises/{enterprise_id}/privacy")
def update_enterprise_privacy_settings(enterprise_id: str, payload: PrivacySettingsUpdate,
                                       changed_by: str = Query("admin"), db: Session = Depends(get_db)):
    svc = EnterprisePrivacyService(db)
    if not svc.update_privacy_settings(enterprise_id, changed_by, payload.model_dump(exclude_none=True)):
        raise HTTPException(404, "Enterprise not found")
    return {"status": "ok", "settings": svc.get_enterprise_privacy_settings(enterprise_id)}


@router.get("/enterprises/{enterprise_id}/privacy/compliance")
def get_privacy_compliance_report(enterprise_id: str, db: Session = Depends(get_db)):
    r = EnterprisePrivacyService(db).audit_service.generate_compliance_report(enterprise_id)
    if not r:
        raise HTTPException(404, "Enterprise not found")
    return r


@router.get("/enterprises/{enterprise_id}/privacy/retention-status")
def get_data_retention_status(enterprise_id: str, db: Session = Depends(get_db)):
    r = EnterprisePrivacyService(db).retention_service.get_retention_status(enterprise_id)
    if not r:
        raise HTTPException(404, "Enterprise not found")
    return r


@router.post("/enterprises/{enterprise_id}/privacy/cleanup")
def run_data_cleanup(enterprise_id: str, db: Session = Depends(get_db)):
    _enterprise_or_404(db, enterprise_id)
    return {"status": "completed",
            "stats": EnterprisePrivacyService(db).retention_service.cleanup_expired_data(enterprise_id)}


@router.post("/enterprises/{enterprise_id}/privacy/export")
def export_enterprise_data(enterprise_id: str, include_sensitive: bool = Query(False),
                           exporter_id: str = Query("admin"), db: Session = Depends(get_db)):
    _, data = EnterprisePrivacyService(db).export_enterprise_data(enterprise_id, exporter_id, "json",
                                                                 include_sensitive)
    if not data:
        raise HTTPException(404, "Enterprise not found")
    return data


@router.delete("/enterprises/{enterprise_id}/privacy/data")
def delete_enterprise_data(enterprise_id: str, confirm: bool = Query(False), requester_id: str = Query("admin"),
                           db: Session = Depends(get_db)):
    _enterprise_or_404(db, enterprise_id)
    return EnterprisePrivacyService(db).delete_enterprise_data(enterprise_id, requester_id, confirm)


@router.post("/privacy/scheduled-cleanup")
def run_scheduled_cleanup(db: Session = Depends(get_db)):
    return EnterprisePrivacyService(db).run_scheduled_cleanup()
