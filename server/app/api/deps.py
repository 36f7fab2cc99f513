"""Shared request dependencies: worker-token auth, optional request signatures, enterprise API keys."""
from __future__ import annotations

import hashlib
import json
from datetime import datetime
from typing import Optional

from fastapi import Depends, Header, HTTPException, Request
from sqlalchemy import select
from sqlalchemy.orm import Session

from app.config import settings
from app.db.database import get_db
from app.models.models import Worker
from app.models.usage import EnterpriseAPIKey
from app.services.security import SecurityService

_AUTH_STATUS = {"worker_not_found": (404, "Worker not found"), "account_locked": (403, "Account locked"),
                "invalid_token": (401, "Invalid token"), "token_expired": (401, "Token expired")}


def authenticate_worker(db: Session, worker_id: str, token: Optional[str], ip: Optional[str] = None) -> Worker:
    if not token:
        raise HTTPException(401, "Missing X-Worker-Token")
    w, err = SecurityService(db).verify_worker_auth(worker_id, token, ip)
    if w is None:
        code, msg = _AUTH_STATUS.get(err, (401, err or "unauthorized"))
        raise HTTPException(code, msg)
    return w


async def check_signature(request: Request, db: Session, worker: Worker) -> None:
    """Enforce HMAC request signing when ``REQUIRE_SIGNATURE`` is on (reference left it unused)."""
    if not settings.require_signature:
        return
    ts = request.headers.get("X-Timestamp")
    sig = request.headers.get("X-Signature")
    raw = await request.body()
    try:
        body = json.loads(raw) if raw else None
    except ValueError:
        body = raw.decode(errors="replace")
    ok, err = SecurityService(db).verify_request_signature(worker, request.method, request.url.path, body,
                                                           int(ts) if ts and ts.isdigit() else None, sig)
    if not ok:
        raise HTTPException(401, f"bad signature: {err}")


def hash_api_key(key: str) -> str:
    return hashlib.sha256(key.encode()).hexdigest()


def lookup_api_key(db: Session, key: Optional[str]) -> Optional[EnterpriseAPIKey]:
    """Resolve an ``ent_`` enterprise key; raises 401/403 on invalid/expired/disabled keys."""
    if not key:
        return None
    rec = db.execute(select(EnterpriseAPIKey).where(EnterpriseAPIKey.key_hash == hash_api_key(key))
                     ).scalar_one_or_none()
    if rec is None or not rec.is_active:
        raise HTTPException(401, "Invalid API key")
    if rec.expires_at and rec.expires_at < datetime.utcnow():
        raise HTTPException(403, "API key expired")
    rec.total_requests = (rec.total_requests or 0) + 1
    rec.last_used_at = datetime.utcnow()
    return rec


def require_admin(x_admin_token: Optional[str] = Header(None)) -> None:
    """Admin routes are open unless ``ADMIN_TOKEN`` is configured (reference: no auth)."""
    if settings.admin_token and x_admin_token != settings.admin_token:
        raise HTTPException(401, "admin token required")


DB = Depends(get_db)
