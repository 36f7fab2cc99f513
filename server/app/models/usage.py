"""Enterprise / billing / usage ORM (reconstructed)."""
from __future__ import annotations

import enum
import uuid
from datetime import datetime

from sqlalchemy import JSON, Boolean, DateTime, Float, Integer, String
from sqlalchemy.orm import Mapped, mapped_column

from app.db.database import Base


def _uuid() -> str:
    return str(uuid.uuid4())


class UsageType(str, enum.Enum):
    LLM_TOKENS = "llm_tokens"
    LLM_REQUESTS = "llm_requests"
    IMAGE_GEN = "image_gen"
    IMAGE_PIXELS = "image_pixels"
    WHISPER_SECONDS = "whisper_seconds"
    EMBEDDING_TOKENS = "embedding_tokens"
    GPU_SECONDS = "gpu_seconds"


class Enterprise(Base):
    __tablename__ = "enterprises"
    id: Mapped[str] = mapped_column(String(36), primary_key=True, default=_uuid)
    name: Mapped[str] = mapped_column(String(256))
    code: Mapped[str] = mapped_column(String(64), unique=True)
    contact_name: Mapped[str | None] = mapped_column(String(128))
    contact_email: Mapped[str | None] = mapped_column(String(256))
    contact_phone: Mapped[str | None] = mapped_column(String(64))
    billing_email: Mapped[str | None] = mapped_column(String(256))
    billing_period: Mapped[str] = mapped_column(String(16), default="monthly")
    currency: Mapped[str] = mapped_column(String(8), default="CNY")
    credit_balance: Mapped[float] = mapped_column(Float, default=0.0)
    credit_limit: Mapped[float | None] = mapped_column(Float)
    monthly_budget: Mapped[float | None] = mapped_column(Float)
    price_plan_id: Mapped[str | None] = mapped_column(String(36))
    custom_pricing: Mapped[dict] = mapped_column(JSON, default=dict)
    data_retention_days: Mapped[int] = mapped_column(Integer, default=30)
    allow_logging: Mapped[bool] = mapped_column(Boolean, default=True)
    anonymize_data: Mapped[bool] = mapped_column(Boolean, default=False)
    private_deployment: Mapped[bool] = mapped_column(Boolean, default=False)
    privacy_settings: Mapped[dict | None] = mapped_column(JSON)
    is_active: Mapped[bool] = mapped_column(Boolean, default=True)
    is_verified: Mapped[bool] = mapped_column(Boolean, default=False)
    created_at: Mapped[datetime] = mapped_column(DateTime, default=datetime.utcnow)


class EnterpriseAPIKey(Base):
    __tablename__ = "enterprise_api_keys"
    id: Mapped[str] = mapped_column(String(36), primary_key=True, default=_uuid)
    enterprise_id: Mapped[str] = mapped_column(String(36), index=True)
    name: Mapped[str | None] = mapped_column(String(128))
    key_hash: Mapped[str] = mapped_column(String(128), index=True)
    key_prefix: Mapped[str] = mapped_column(String(16))
    allowed_types: Mapped[list | None] = mapped_column(JSON)
    allowed_models: Mapped[list | None] = mapped_column(JSON)
    rate_limit_per_minute: Mapped[int] = mapped_column(Integer, default=60)
    daily_limit: Mapped[int | None] = mapped_column(Integer)
    ip_whitelist: Mapped[list | None] = mapped_column(JSON)
    is_active: Mapped[bool] = mapped_column(Boolean, default=True)
    total_requests: Mapped[int] = mapped_column(Integer, default=0)
    last_used_at: Mapped[datetime | None] = mapped_column(DateTime)
    expires_at: Mapped[datetime | None] = mapped_column(DateTime)
    created_at: Mapped[datetime] = mapped_column(DateTime, default=datetime.utcnow)


class UsageRecord(Base):
    __tablename__ = "usage_records"
    id: Mapped[str] = mapped_column(String(36), primary_key=True, default=_uuid)
    enterprise_id: Mapped[str | None] = mapped_column(String(36), index=True)
    worker_id: Mapped[str | None] = mapped_column(String(36), index=True)
    job_id: Mapped[str | None] = mapped_column(String(36), index=True)
    api_key_id: Mapped[str | None] = mapped_column(String(36))
    machine_id: Mapped[str | None] = mapped_column(String(128))
    usage_type: Mapped[str] = mapped_column(String(32))
    job_type: Mapped[str | None] = mapped_column(String(32))
    model_id: Mapped[str | None] = mapped_column(String(256))
    quantity: Mapped[float] = mapped_column(Float, default=0.0)
    unit: Mapped[str | None] = mapped_column(String(32))
    unit_price: Mapped[float] = mapped_column(Float, default=0.0)
    total_cost: Mapped[float] = mapped_column(Float, default=0.0)
    gpu_seconds: Mapped[float] = mapped_column(Float, default=0.0)
    gpu_memory_peak_gb: Mapped[float | None] = mapped_column(Float)
    started_at: Mapped[datetime | None] = mapped_column(DateTime)
    completed_at: Mapped[datetime | None] = mapped_column(DateTime)
    duration_ms: Mapped[int | None] = mapped_column(Integer)
    request_summary: Mapped[dict | None] = mapped_column(JSON)
    response_summary: Mapped[dict | None] = mapped_column(JSON)
    worker_region: Mapped[str | None] = mapped_column(String(64))
    client_ip: Mapped[str | None] = mapped_column(String(64))
    client_region: Mapped[str | None] = mapped_column(String(64))
    created_at: Mapped[datetime] = mapped_column(DateTime, default=datetime.utcnow, index=True)


class Bill(Base):
    __tablename__ = "bills"
    id: Mapped[str] = mapped_column(String(36), primary_key=True, default=_uuid)
    enterprise_id: Mapped[str] = mapped_column(String(36), index=True)
    billing_period: Mapped[str] = mapped_column(String(16), default="monthly")
    period_start: Mapped[datetime | None] = mapped_column(DateTime)
    period_end: Mapped[datetime | None] = mapped_column(DateTime)
    subtotal: Mapped[float] = mapped_column(Float, default=0.0)
    discount: Mapped[float] = mapped_column(Float, default=0.0)
    tax: Mapped[float] = mapped_column(Float, default=0.0)
    total: Mapped[float] = mapped_column(Float, default=0.0)
    currency: Mapped[str] = mapped_column(String(8), default="CNY")
    usage_summary: Mapped[dict | None] = mapped_column(JSON)
    status: Mapped[str] = mapped_column(String(16), default="pending")
    paid_at: Mapped[datetime | None] = mapped_column(DateTime)
    payment_method: Mapped[str | None] = mapped_column(String(32))
    invoice_number: Mapped[str | None] = mapped_column(String(64))
    invoice_url: Mapped[str | None] = mapped_column(String(256))
    created_at: Mapped[datetime] = mapped_column(DateTime, default=datetime.utcnow)
    due_at: Mapped[datetime | None] = mapped_column(DateTime)


class PricePlan(Base):
    __tablename__ = "price_plans"
    id: Mapped[str] = mapped_column(String(36), primary_key=True, default=_uuid)
    name: Mapped[str | None] = mapped_column(String(128))
    prices: Mapped[dict] = mapped_column(JSON, default=dict)


class WorkerUsageSummary(Base):
    __tablename__ = "worker_usage_summaries"
    id: Mapped[str] = mapped_column(String(36), primary_key=True, default=_uuid)
    worker_id: Mapped[str] = mapped_column(String(36), index=True)
    machine_id: Mapped[str | None] = mapped_column(String(128))
    period_type: Mapped[str] = mapped_column(String(16), default="hourly")
    period_start: Mapped[datetime | None] = mapped_column(DateTime)
    period_end: Mapped[datetime | None] = mapped_column(DateTime)
    total_jobs: Mapped[int] = mapped_column(Integer, default=0)
    completed_jobs: Mapped[int] = mapped_column(Integer, default=0)
    total_gpu_seconds: Mapped[float] = mapped_column(Float, default=0.0)
    total_tokens: Mapped[int] = mapped_column(Integer, default=0)
    total_images: Mapped[int] = mapped_column(Integer, default=0)
    total_revenue: Mapped[float] = mapped_column(Float, default=0.0)
    peak_gpu_memory_gb: Mapped[float | None] = mapped_column(Float)
