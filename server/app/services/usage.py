"""Usage metering and billing aggregates (reference services/usage.py:18-431).

``record_usage`` is called by ``POST /jobs/{id}/complete`` whenever the
job carries an enterprise (the reference never called it).
Pricing precedence: enterprise custom price, then its price plan, then
the defaults below.  Summaries honour the enterprise privacy flags.
"""
from __future__ import annotations

from collections import defaultdict
from datetime import datetime, timedelta
from typing import Any, Dict, List, Optional

from sqlalchemy import func, select
from sqlalchemy.orm import Session

from app.models.models import Job, JobStatus, Worker
from app.models.usage import Enterprise, PricePlan, UsageRecord, UsageType, WorkerUsageSummary

DEFAULT_PRICES = {
    UsageType.LLM_TOKENS.value: 0.002,        # per 1K tokens
    UsageType.LLM_REQUESTS.value: 0.01,
    UsageType.IMAGE_GEN.value: 0.1,           # per image
    UsageType.IMAGE_PIXELS.value: 0.00001,
    UsageType.WHISPER_SECONDS.value: 0.006,
    UsageType.EMBEDDING_TOKENS.value: 0.0001,  # per 1K tokens
    UsageType.GPU_SECONDS.value: 0.001,
}


class UsageService:
    @staticmethod
    def record_usage(db: Session, job: Job, worker: Optional[Worker] = None, enterprise: Optional[Enterprise] = None,
                     api_key_id: Optional[str] = None, usage_details: Optional[Dict[str, Any]] = None,
                     client_ip: Optional[str] = None) -> UsageRecord:
        details = usage_details or {}
        u = UsageService._calculate_usage(job, details)
        unit_price, cost = UsageService._calculate_cost(db, enterprise, u["usage_type"], u["quantity"])
        started, completed = job.started_at, job.completed_at or datetime.utcnow()
        duration = int((completed - started).total_seconds() * 1000) if started else None
        gpu_s = float(details.get("gpu_seconds") or (duration or 0) / 1000.0)
        rec = UsageRecord(
            enterprise_id=enterprise.id if enterprise else job.enterprise_id, worker_id=job.worker_id,
            job_id=job.id, api_key_id=api_key_id or job.api_key_id,
            machine_id=worker.machine_id if worker else None, usage_type=u["usage_type"], job_type=job.type,
            model_id=(job.params or {}).get("model"), quantity=u["quantity"], unit=u["unit"],
            unit_price=unit_price, total_cost=cost, gpu_seconds=gpu_s,
            gpu_memory_peak_gb=details.get("gpu_memory_peak_gb"), started_at=started, completed_at=completed,
            duration_ms=duration, request_summary=UsageService._create_request_summary(job, enterprise),
            response_summary=UsageService._create_response_summary(job, enterprise),
            worker_region=worker.region if worker else None,
            client_ip=None if (enterprise and enterprise.anonymize_data) else (client_ip or job.client_ip),
            client_region=job.client_region)
        db.add(rec)
        if enterprise is not None:
            enterprise.credit_balance = (enterprise.credit_balance or 0.0) - cost
        db.commit()
        return rec

    @staticmethod
    def _calculate_usage(job: Job, details: Dict) -> Dict[str, Any]:
        res = job.result or {}
        t = job.type
        if t == "llm":
            usage = res.get("usage") or {}
            tokens = int(details.get("total_tokens") or usage.get("total_tokens") or 0)
            return {"usage_type": UsageType.LLM_TOKENS.value, "quantity": tokens / 1000.0, "unit": "1k_tokens",
                    "tokens": tokens}
        if t == "image_gen":
            n = int(details.get("num_images") or len(res.get("images") or []) or 1)
            return {"usage_type": UsageType.IMAGE_GEN.value, "quantity": float(n), "unit": "images"}
        if t == "whisper":
            secs = float(details.get("audio_seconds") or res.get("duration") or 0.0)
            return {"usage_type": UsageType.WHISPER_SECONDS.value, "quantity": secs, "unit": "seconds"}
        if t == "embedding":
            tokens = int(details.get("total_tokens") or (res.get("usage") or {}).get("total_tokens") or 0)
            return {"usage_type": UsageType.EMBEDDING_TOKENS.value, "quantity": tokens / 1000.0,
                    "unit": "1k_tokens"}
        secs = float(details.get("gpu_seconds") or 0.0)
        return {"usage_type": UsageType.GPU_SECONDS.value, "quantity": secs, "unit": "seconds"}

    @staticmethod
    def _calculate_cost(db: Session, enterprise: Optional[Enterprise], usage_type: str, quantity: float) -> tuple:
        price = None
        if enterprise is not None and (enterprise.custom_pricing or {}).get(usage_type) is not None:
            price = float(enterprise.custom_pricing[usage_type])
        elif enterprise is not None and enterprise.price_plan_id:
            plan = db.get(PricePlan, enterprise.price_plan_id)
            price = float((plan.prices or {}).get(usage_type, 0.0)) if plan else 0.0
        if price is None:
            price = DEFAULT_PRICES.get(usage_type, 0.0)
        return price, price * quantity

    @staticmethod
    def _create_request_summary(job: Job, enterprise: Optional[Enterprise]) -> Optional[Dict]:
        if enterprise is not None and not enterprise.allow_logging:
            return None
        p = job.params or {}
        s: Dict[str, Any] = {"type": job.type, "model": p.get("model")}
        if "messages" in p:
            s["message_count"] = len(p.get("messages") or [])
        if "max_tokens" in p:
            s["max_tokens"] = p["max_tokens"]
        if not (enterprise is not None and enterprise.anonymize_data):
            prompt = p.get("prompt") or ""
            if not prompt and p.get("messages"):
                prompt = str((p["messages"][-1] or {}).get("content", ""))
            s["prompt_preview"] = prompt[:100]
        return s

    @staticmethod
    def _create_response_summary(job: Job, enterprise: Optional[Enterprise]) -> Optional[Dict]:
        if enterprise is not None and not enterprise.allow_logging:
            return None
        r = job.result or {}
        s: Dict[str, Any] = {"status": job.status, "finish_reason": r.get("finish_reason"), "usage": r.get("usage")}
        if not (enterprise is not None and enterprise.anonymize_data) and isinstance(r.get("response"), str):
            s["response_preview"] = r["response"][:100]
        return s

    @staticmethod
    def _aggregate(records: List[UsageRecord]) -> Dict[str, Any]:
        by_type: Dict[str, Dict[str, float]] = defaultdict(lambda: {"quantity": 0.0, "cost": 0.0, "count": 0})
        for r in records:
            b = by_type[r.usage_type]
            b["quantity"] += r.quantity or 0.0
            b["cost"] += r.total_cost or 0.0
            b["count"] += 1
        return {"total_records": len(records), "total_cost": round(sum(r.total_cost or 0 for r in records), 6),
                "total_gpu_seconds": round(sum(r.gpu_seconds or 0 for r in records), 3),
                "by_type": dict(by_type)}

    @staticmethod
    def get_enterprise_usage(db: Session, enterprise_id: str, start_date: Optional[datetime] = None,
                             end_date: Optional[datetime] = None) -> Dict[str, Any]:
        end = end_date or datetime.utcnow()
        start = start_date or end - timedelta(days=30)
        recs = list(db.execute(select(UsageRecord).where(
            UsageRecord.enterprise_id == enterprise_id, UsageRecord.created_at >= start,
            UsageRecord.created_at <= end)).scalars())
        out = UsageService._aggregate(recs)
        out.update(enterprise_id=enterprise_id, start_date=start.isoformat(), end_date=end.isoformat())
        return out

    @staticmethod
    def get_worker_usage(db: Session, worker_id: str, start_date: Optional[datetime] = None,
                         end_date: Optional[datetime] = None) -> Dict[str, Any]:
        end = end_date or datetime.utcnow()
        start = start_date or end - timedelta(days=30)
        recs = list(db.execute(select(UsageRecord).where(
            UsageRecord.worker_id == worker_id, UsageRecord.created_at >= start,
            UsageRecord.created_at <= end)).scalars())
        out = UsageService._aggregate(recs)
        out.update(worker_id=worker_id, start_date=start.isoformat(), end_date=end.isoformat(),
                   total_revenue=out["total_cost"])
        return out

    @staticmethod
    def aggregate_hourly_summary(db: Session, worker_id: str, hour: datetime) -> WorkerUsageSummary:
        start = hour.replace(minute=0, second=0, microsecond=0)
        end = start + timedelta(hours=1)
        recs = list(db.execute(select(UsageRecord).where(
            UsageRecord.worker_id == worker_id, UsageRecord.created_at >= start,
            UsageRecord.created_at < end)).scalars())
        jobs = list(db.execute(select(Job).where(Job.worker_id == worker_id, Job.started_at >= start,
                                                 Job.started_at < end)).scalars())
        s = db.execute(select(WorkerUsageSummary).where(
            WorkerUsageSummary.worker_id == worker_id, WorkerUsageSummary.period_type == "hourly",
            WorkerUsageSummary.period_start == start)).scalar_one_or_none()
        if s is None:
            s = WorkerUsageSummary(worker_id=worker_id, period_type="hourly", period_start=start, period_end=end)
            db.add(s)
        w = db.get(Worker, worker_id)
        s.machine_id = w.machine_id if w else None
        s.total_jobs = len(jobs)
        s.completed_jobs = sum(1 for j in jobs if j.status == JobStatus.COMPLETED.value)
        s.total_gpu_seconds = sum(r.gpu_seconds or 0 for r in recs)
        s.total_tokens = int(sum((r.quantity or 0) * 1000 for r in recs if r.usage_type == UsageType.LLM_TOKENS.value))
        s.total_images = int(sum(r.quantity or 0 for r in recs if r.usage_type == UsageType.IMAGE_GEN.value))
        s.total_revenue = sum(r.total_cost or 0 for r in recs)
        peaks = [r.gpu_memory_peak_gb for r in recs if r.gpu_memory_peak_gb]
        s.peak_gpu_memory_gb = max(peaks) if peaks else None
        db.commit()
        return s

    @staticmethod
    def get_platform_stats(db: Session) -> Dict[str, Any]:
        """Dashboard numbers (shape of reference usage.py:387-431: workers/enterprises/today/this_month)."""
        now = datetime.utcnow()
        today = now.replace(hour=0, minute=0, second=0, microsecond=0)
        month = today.replace(day=1)

        def window(since: datetime) -> Dict[str, Any]:
            n, cost, gpu_s = db.execute(select(func.count(UsageRecord.id),
                                               func.coalesce(func.sum(UsageRecord.total_cost), 0.0),
                                               func.coalesce(func.sum(UsageRecord.gpu_seconds), 0.0))
                                        .where(UsageRecord.created_at >= since)).one()
            return {"jobs": int(n or 0), "revenue": round(float(cost or 0), 2),
                    "gpu_hours": round(float(gpu_s or 0) / 3600.0, 2)}
        total_w = db.execute(select(func.count(Worker.id))).scalar() or 0
        online_w = db.execute(select(func.count(Worker.id)).where(
            Worker.status.in_(["online", "busy"]))).scalar() or 0
        n_ent = db.execute(select(func.count(Enterprise.id)).where(Enterprise.is_active.is_(True))).scalar() or 0
        return {"timestamp": now.isoformat(), "workers": {"total": int(total_w), "online": int(online_w)},
                "enterprises": {"total": int(n_ent)}, "today": window(today), "this_month": window(month)}
