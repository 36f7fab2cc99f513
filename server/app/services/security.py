"""Worker authentication, token lifecycle and request signing
(reference services/security.py:24-336).

Signatures are HMAC-SHA256 over ``METHOD:PATH:sha256(body):timestamp`` with a
300 s window; the worker API enforces them when ``settings.require_signature``
(the reference never verified them, Appendix E-20).
"""
from __future__ import annotations

import asyncio
import hashlib
import hmac
import inspect
import json
import logging
import secrets
from datetime import datetime, timedelta
from typing import Any, Optional, Tuple

from sqlalchemy.orm import Session

from app.models.models import Worker

logger = logging.getLogger(__name__)
audit_logger = logging.getLogger("security.audit")


class SecuritySettings:
    TOKEN_EXPIRY_HOURS = 24
    REFRESH_THRESHOLD_HOURS = 4
    MAX_FAILED_ATTEMPTS = 5
    LOCKOUT_MINUTES = 15
    SIGNATURE_VALIDITY_SECONDS = 300
    TOKEN_BYTES = 32


class TokenManager:
    @staticmethod
    def generate_token() -> str:
        return secrets.token_urlsafe(SecuritySettings.TOKEN_BYTES)

    @staticmethod
    def generate_signing_secret() -> str:
        return secrets.token_hex(32)

    @staticmethod
    def hash_token(token: str) -> str:
        salt = secrets.token_hex(8)
        digest = hashlib.sha256((salt + token).encode()).hexdigest()
        return f"{salt}${digest}"

    @staticmethod
    def verify_token_hash(token: str, token_hash: Optional[str]) -> bool:
        if not token or not token_hash:
            return False
        if "$" in token_hash:
            salt, digest = token_hash.split("$", 1)
            return hmac.compare_digest(hashlib.sha256((salt + token).encode()).hexdigest(), digest)
        return hmac.compare_digest(hashlib.sha256(token.encode()).hexdigest(), token_hash)

    @staticmethod
    def expiry() -> datetime:
        return datetime.utcnow() + timedelta(hours=SecuritySettings.TOKEN_EXPIRY_HOURS)


class RequestSigner:
    @staticmethod
    def _body_hash(body: Any) -> str:
        if body is None:
            b = b""
        elif isinstance(body, (bytes, bytearray)):
            b = bytes(body)
        elif isinstance(body, str):
            b = body.encode()
        else:
            b = json.dumps(body, sort_keys=True, separators=(",", ":")).encode()
        return hashlib.sha256(b).hexdigest()

    @staticmethod
    def sign_request(method: str, path: str, body: Any, timestamp: int, secret: str) -> str:
        msg = f"{method.upper()}:{path}:{RequestSigner._body_hash(body)}:{int(timestamp)}"
        return hmac.new(secret.encode(), msg.encode(), hashlib.sha256).hexdigest()

    @staticmethod
    def verify_signature(method: str, path: str, body: Any, timestamp: int, signature: str,
                         secret: str) -> Tuple[bool, str]:
        now = int(datetime.utcnow().timestamp())
        if abs(now - int(timestamp)) > SecuritySettings.SIGNATURE_VALIDITY_SECONDS:
            return False, "signature_expired"
        expect = RequestSigner.sign_request(method, path, body, timestamp, secret)
        if not hmac.compare_digest(expect, signature or ""):
            return False, "invalid_signature"
        return True, ""


class AuditLogger:
    @staticmethod
    def log_auth_event(event: str, worker_id: str, success: bool, ip: Optional[str] = None, **details) -> None:
        audit_logger.info("AUTH_EVENT %s", json.dumps({"event": event, "worker_id": worker_id, "success": success,
                                                        "ip": ip, "ts": datetime.utcnow().isoformat(), **details},
                                                       default=str))

    @staticmethod
    def log_security_event(event: str, severity: str = "info", **details) -> None:
        audit_logger.warning("SECURITY_EVENT %s", json.dumps({"event": event, "severity": severity,
                                                               "ts": datetime.utcnow().isoformat(), **details},
                                                              default=str))


class SecurityService:
    """Worker authentication over either a sync ``Session`` (this server) or an
    ``AsyncSession`` (reference API: the same methods become awaitable)."""

    def __init__(self, db):
        self.db = db
        ex = getattr(db, "execute", None)
        self._async = asyncio.iscoroutinefunction(ex) or inspect.iscoroutinefunction(ex)

    def _check(self, w, token: str, ip: Optional[str], worker_id) -> Tuple[Optional[Worker], str, bool]:
        """Pure decision: (worker or None, error, needs_commit)."""
        if w is None:
            AuditLogger.log_auth_event("verify", str(worker_id), False, ip, reason="worker_not_found")
            return None, "worker_not_found", False
        now = datetime.utcnow()
        if w.locked_until and w.locked_until > now:
            return None, "account_locked", False
        if not TokenManager.verify_token_hash(token, w.auth_token_hash):
            w.failed_auth_attempts = (w.failed_auth_attempts or 0) + 1
            w.last_failed_auth = now
            if w.failed_auth_attempts >= SecuritySettings.MAX_FAILED_ATTEMPTS:
                w.locked_until = now + timedelta(minutes=SecuritySettings.LOCKOUT_MINUTES)
                AuditLogger.log_security_event("worker_locked", "high", worker_id=str(w.id))
            AuditLogger.log_auth_event("verify", str(w.id), False, ip, reason="invalid_token")
            return None, "invalid_token", True
        if w.token_expires_at and w.token_expires_at < now:
            return None, "token_expired", False
        if w.failed_auth_attempts:
            w.failed_auth_attempts = 0
            w.locked_until = None
            return w, "", True
        return w, "", False

    def verify_worker_auth(self, worker_id: str, token: str, ip: Optional[str] = None):
        if self._async:
            return self._verify_worker_auth_async(worker_id, token, ip)
        w = self.db.get(Worker, str(worker_id)) if worker_id else None
        w, err, dirty = self._check(w, token, ip, worker_id)
        if dirty:
            self.db.commit()
        return w, err

    async def _verify_worker_auth_async(self, worker_id: str, token: str, ip: Optional[str] = None):
        from sqlalchemy import select
        w = None
        if worker_id:
            res = await self.db.execute(select(Worker).where(Worker.id == str(worker_id)))
            w = res.scalar_one_or_none()
        w, err, dirty = self._check(w, token, ip, worker_id)
        if dirty:
            await self.db.commit()
        return w, err

    def should_refresh_token(self, worker) -> bool:
        exp = getattr(worker, "token_expires_at", None)
        if exp is None:
            return False
        return exp - datetime.utcnow() < timedelta(hours=SecuritySettings.REFRESH_THRESHOLD_HOURS)

    def issue_tokens(self, worker: Worker) -> Tuple[str, str]:
        token, refresh = TokenManager.generate_token(), TokenManager.generate_token()
        worker.auth_token_hash = TokenManager.hash_token(token)
        worker.refresh_token_hash = TokenManager.hash_token(refresh)
        worker.token_expires_at = TokenManager.expiry()
        if not worker.signing_secret:
            worker.signing_secret = TokenManager.generate_signing_secret()
        return token, refresh

    def refresh_tokens(self, worker: Worker, refresh_token: str) -> Optional[Tuple[str, str]]:
        if not TokenManager.verify_token_hash(refresh_token, worker.refresh_token_hash):
            AuditLogger.log_auth_event("refresh", str(worker.id), False, reason="invalid_refresh_token")
            return None
        return self.issue_tokens(worker)

    def _signature(self, worker, method, path, body, timestamp, signature) -> Tuple[bool, str]:
        secret = getattr(worker, "signing_secret", None)
        if not secret:
            return False, "no_signing_secret"
        if timestamp is None or not signature:
            return False, "missing_signature"
        return RequestSigner.verify_signature(method, path, body, int(timestamp), signature, secret)

    def verify_request_signature(self, worker, method: str, path: str, body: Any, timestamp: Optional[int],
                                 signature: Optional[str]):
        out = self._signature(worker, method, path, body, timestamp, signature)
        if self._async:
            async def _done():
                return out
            return _done()
        return out
