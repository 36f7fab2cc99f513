"""Enterprise privacy suite (reference services/privacy.py:29-812).

* ``DataAnonymizer`` — salted hashes, format-preserving masks (e-mail keeps
  its domain, digits keep 2+2), IP truncation, PII scrubbing and recursive
  dict redaction.
* ``DataEncryptor`` — authenticated symmetric encryption keyed by a
  passphrase (PBKDF2-SHA256).  Uses ``cryptography``'s Fernet when it is
  installed; otherwise a stdlib construction (HMAC-SHA256 counter-mode
  keystream + encrypt-then-MAC tag), so the server has no hard dependency
  on ``cryptography`` (SURVEY §6 note on requirements).  A wrong key
  decrypts to ``"[DECRYPTION_FAILED]"``.
* ``DataRetentionService``, ``PrivacyAuditService`` (audit events on the
  ``audit`` logger), ``EnterprisePrivacyService`` (settings, export /
  right-to-be-forgotten delete, scheduled cleanup).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import ipaddress
import json
import logging
import os
import re
import secrets
from datetime import datetime, timedelta
from typing import Any, Dict, List, Optional, Tuple

from sqlalchemy import delete, func, select
from sqlalchemy.orm import Session

from app.models.models import Job
from app.models.usage import Bill, Enterprise, UsageRecord

logger = logging.getLogger(__name__)
audit_logger = logging.getLogger("audit")


class PrivacyConfig:
    DEFAULT_RETENTION_DAYS = 30
    MIN_RETENTION_DAYS = 7
    MAX_RETENTION_DAYS = 365
    ANONYMIZE_IP_MASK = True
    ANONYMIZE_CONTENT = True
    HASH_SALT_LENGTH = 16
    ENCRYPTION_KEY_ENV = "PRIVACY_ENCRYPTION_KEY"
    KEY_DERIVATION_ITERATIONS = 100_000
    CONTENT_FIELDS = ["prompt", "messages", "input", "output", "response"]
    SECRET_FIELDS = ["api_key", "token", "password", "secret"]
    IDENTITY_FIELDS = ["email", "phone", "address", "name"]
    SENSITIVE_FIELDS = CONTENT_FIELDS + SECRET_FIELDS + IDENTITY_FIELDS
    # order matters: long digit runs before the shorter phone pattern
    PII_PATTERNS = {
        "email": r"[A-Za-z0-9._%+-]+@[A-Za-z0-9.-]+\.[A-Za-z]{2,}",
        "credit_card": r"\b\d{4}[-\s]?\d{4}[-\s]?\d{4}[-\s]?\d{4}\b",
        "id_card_cn": r"\b\d{17}[\dXx]\b",
        "phone_cn": r"(?<!\d)1[3-9]\d{9}(?!\d)",
        "phone_intl": r"\+\d{1,3}[-.\s]?\d{4,14}",
        "ip_address": r"\b\d{1,3}\.\d{1,3}\.\d{1,3}\.\d{1,3}\b",
    }


class DataAnonymizer:
    def __init__(self, salt: Optional[str] = None):
        self.salt = salt or secrets.token_hex(PrivacyConfig.HASH_SALT_LENGTH)
        self._patterns = [(k, re.compile(p)) for k, p in PrivacyConfig.PII_PATTERNS.items()]

    def anonymize_string(self, value: str, preserve_format: bool = False) -> str:
        if not value:
            return value
        if not preserve_format:
            return self._hash_value(value)
        if "@" in value:
            local, _, domain = value.partition("@")
            return f"{local[:1]}***@{domain}"
        if any(c.isdigit() for c in value):
            return self._mask_digits(value)
        if len(value) <= 2:
            return "*" * len(value)
        return value[0] + "*" * (len(value) - 2) + value[-1]

    def anonymize_ip(self, ip: str) -> str:
        try:
            a = ipaddress.ip_address(ip)
        except ValueError:
            return "[INVALID_IP]"
        if a.version == 4:
            o = str(a).split(".")
            return f"{o[0]}.{o[1]}.xxx.xxx"
        groups = a.exploded.split(":")
        return f"{int(groups[0], 16):x}:{int(groups[1], 16):x}::xxxx"

    def anonymize_content(self, content: str, max_preview: int = 50) -> str:
        if not content:
            return content
        text = self._remove_pii(content)
        if len(text) > max_preview:
            text = text[:max_preview] + "..."
        return text

    def anonymize_dict(self, data: Any, fields_to_anonymize: Optional[List[str]] = None) -> Any:
        fields = {f.lower() for f in (fields_to_anonymize or PrivacyConfig.SENSITIVE_FIELDS)}
        if isinstance(data, list):
            return [self.anonymize_dict(x, fields_to_anonymize) for x in data]
        if not isinstance(data, dict):
            return data
        out: Dict[str, Any] = {}
        for k, v in data.items():
            key = str(k).lower()
            if key in fields:
                if key in PrivacyConfig.SECRET_FIELDS:
                    out[k] = "[REDACTED]"
                elif key in PrivacyConfig.CONTENT_FIELDS:
                    blob = v if isinstance(v, str) else json.dumps(v, sort_keys=True, default=str)
                    out[k] = f"[CONTENT:{self._hash_value(blob)[:12]}:len={len(blob)}]"
                elif isinstance(v, str):
                    out[k] = f"[{self.anonymize_string(v, preserve_format=True)}]"
                else:
                    out[k] = "[REDACTED]"
            elif isinstance(v, (dict, list)):
                out[k] = self.anonymize_dict(v, fields_to_anonymize)
            else:
                out[k] = v
        return out

    def create_pseudonym(self, identifier: str, context: str = "") -> str:
        return "anon_" + self._hash_value(f"{context}:{identifier}")[:16]

    def _hash_value(self, value: str) -> str:
        return hashlib.sha256(f"{self.salt}:{value}".encode()).hexdigest()

    @staticmethod
    def _mask_digits(value: str) -> str:
        if len(value) <= 4:
            return "*" * len(value)
        return value[:2] + "*" * (len(value) - 4) + value[-2:]

    def _remove_pii(self, text: str) -> str:
        for name, pat in self._patterns:
            text = pat.sub(f"[{name.upper()}]", text)
        return text


class DataEncryptor:
    _MAGIC = b"d1"

    def __init__(self, encryption_key: Optional[str] = None):
        key = encryption_key or os.environ.get(PrivacyConfig.ENCRYPTION_KEY_ENV)
        if not key:
            key = secrets.token_urlsafe(32)
            logger.warning("no %s set; using an ephemeral encryption key", PrivacyConfig.ENCRYPTION_KEY_ENV)
        material = hashlib.pbkdf2_hmac("sha256", key.encode(), b"dgi-privacy-v1",
                                       PrivacyConfig.KEY_DERIVATION_ITERATIONS, dklen=64)
        self._enc_key, self._mac_key = material[:32], material[32:]
        self._fernet = None
        try:
            from cryptography.fernet import Fernet  # type: ignore
            self._fernet = Fernet(base64.urlsafe_b64encode(material[:32]))
        except Exception:
            pass

    def _keystream(self, nonce: bytes, n: int) -> bytes:
        out = bytearray()
        ctr = 0
        while len(out) < n:
            out += hmac.new(self._enc_key, nonce + ctr.to_bytes(8, "big"), hashlib.sha256).digest()
            ctr += 1
        return bytes(out[:n])

    def encrypt(self, plaintext: str) -> str:
        data = plaintext.encode()
        if self._fernet is not None:
            return self._fernet.encrypt(data).decode()
        nonce = secrets.token_bytes(16)
        ct = bytes(a ^ b for a, b in zip(data, self._keystream(nonce, len(data))))
        body = self._MAGIC + nonce + ct
        tag = hmac.new(self._mac_key, body, hashlib.sha256).digest()
        return base64.urlsafe_b64encode(body + tag).decode()

    def decrypt(self, ciphertext: str) -> str:
        try:
            if self._fernet is not None:
                return self._fernet.decrypt(ciphertext.encode()).decode()
            raw = base64.urlsafe_b64decode(ciphertext.encode())
            body, tag = raw[:-32], raw[-32:]
            if not body.startswith(self._MAGIC) or not hmac.compare_digest(
                    tag, hmac.new(self._mac_key, body, hashlib.sha256).digest()):
                raise ValueError("bad tag")
            nonce, ct = body[2:18], body[18:]
            return bytes(a ^ b for a, b in zip(ct, self._keystream(nonce, len(ct)))).decode()
        except Exception:
            return "[DECRYPTION_FAILED]"

    def encrypt_dict(self, data: Dict, fields_to_encrypt: List[str]) -> Dict:
        out = dict(data)
        enc = []
        for f in fields_to_encrypt:
            if f in out and out[f] is not None:
                v = out[f]
                out[f] = self.encrypt(v if isinstance(v, str) else json.dumps(v, default=str))
                enc.append(f)
        if enc:
            out["_encrypted_fields"] = enc
        return out

    def decrypt_dict(self, data: Dict) -> Dict:
        out = dict(data)
        for f in out.pop("_encrypted_fields", []) or []:
            if f in out:
                v = self.decrypt(out[f])
                try:
                    out[f] = json.loads(v)
                except (ValueError, TypeError):
                    out[f] = v
        return out


class DataRetentionService:
    def __init__(self, db: Session):
        self.db = db

    def cleanup_expired_data(self, enterprise_id: Optional[str] = None) -> Dict[str, int]:
        stats = {"usage_records_deleted": 0, "jobs_anonymized": 0, "enterprises_processed": 0}
        q = select(Enterprise).where(Enterprise.is_active.is_(True))
        if enterprise_id:
            q = q.where(Enterprise.id == enterprise_id)
        for ent in self.db.execute(q).scalars():
            days = ent.data_retention_days or PrivacyConfig.DEFAULT_RETENTION_DAYS
            days = max(PrivacyConfig.MIN_RETENTION_DAYS, min(PrivacyConfig.MAX_RETENTION_DAYS, days))
            cutoff = datetime.utcnow() - timedelta(days=days)
            stats["jobs_anonymized"] += self._anonymize_expired_jobs(ent.id, cutoff)
            stats["usage_records_deleted"] += self._delete_expired_usage_records(ent.id, cutoff)
            stats["enterprises_processed"] += 1
        self.db.commit()
        return stats

    def _delete_expired_usage_records(self, enterprise_id: str, cutoff_date: datetime) -> int:
        r = self.db.execute(delete(UsageRecord).where(UsageRecord.enterprise_id == enterprise_id,
                                                      UsageRecord.created_at < cutoff_date))
        return int(r.rowcount or 0)

    def _anonymize_expired_jobs(self, enterprise_id: str, cutoff_date: datetime) -> int:
        jobs = self.db.execute(select(Job).where(Job.enterprise_id == enterprise_id, Job.created_at < cutoff_date)
                               ).scalars().all()
        a = DataAnonymizer()
        n = 0
        for job in jobs:
            if (job.params or {}).get("_anonymized"):
                continue
            job.params = {**a.anonymize_dict(job.params or {}), "_anonymized": True}
            if job.result:
                job.result = a.anonymize_dict(job.result)
            n += 1
        return n

    def get_retention_status(self, enterprise_id: str) -> Dict[str, Any]:
        ent = self.db.get(Enterprise, enterprise_id)
        if ent is None:
            return {}
        days = ent.data_retention_days or PrivacyConfig.DEFAULT_RETENTION_DAYS
        cutoff = datetime.utcnow() - timedelta(days=days)
        total = self.db.execute(select(func.count(UsageRecord.id)).where(
            UsageRecord.enterprise_id == enterprise_id)).scalar() or 0
        expired = self.db.execute(select(func.count(UsageRecord.id)).where(
            UsageRecord.enterprise_id == enterprise_id, UsageRecord.created_at < cutoff)).scalar() or 0
        return {"enterprise_id": str(enterprise_id), "retention_days": days, "cutoff_date": cutoff.isoformat(),
                "total_records": int(total), "expired_records": int(expired),
                "retention_compliance": expired == 0}


class PrivacyAuditService:
    def __init__(self, db: Session):
        self.db = db
        self.events: List[Dict[str, Any]] = []

    def _emit(self, event: str, **fields) -> Dict[str, Any]:
        rec = {"event": event, "timestamp": datetime.utcnow().isoformat(), **fields}
        self.events.append(rec)
        audit_logger.info(json.dumps(rec, ensure_ascii=False, default=str))
        return rec

    def log_data_access(self, enterprise_id: str, accessor_id: str, accessor_type: str, data_type: str,
                        action: str, record_count: int = 1, details: Optional[Dict] = None) -> Dict[str, Any]:
        return self._emit("PRIVACY_AUDIT", enterprise_id=str(enterprise_id), accessor_id=accessor_id,
                          accessor_type=accessor_type, data_type=data_type, action=action,
                          record_count=record_count, details=details or {})

    def log_privacy_setting_change(self, enterprise_id: str, changed_by: str, setting_name: str,
                                   old_value: Any, new_value: Any) -> Dict[str, Any]:
        return self._emit("PRIVACY_SETTING_CHANGE", enterprise_id=str(enterprise_id), changed_by=changed_by,
                          setting=setting_name, old_value=old_value, new_value=new_value)

    def log_data_export(self, enterprise_id: str, exporter_id: str, export_format: str, record_count: int,
                        destination: str) -> Dict[str, Any]:
        return self._emit("DATA_EXPORT", enterprise_id=str(enterprise_id), exporter_id=exporter_id,
                          format=export_format, record_count=record_count, destination=destination)

    def generate_compliance_report(self, enterprise_id: str) -> Dict[str, Any]:
        ent = self.db.get(Enterprise, enterprise_id)
        if ent is None:
            return {}
        ret = DataRetentionService(self.db).get_retention_status(enterprise_id)
        return {
            "enterprise_id": str(enterprise_id), "enterprise_name": ent.name,
            "generated_at": datetime.utcnow().isoformat(),
            "privacy_settings": {"data_retention_days": ent.data_retention_days, "allow_logging": ent.allow_logging,
                                 "anonymize_data": ent.anonymize_data, "private_deployment": ent.private_deployment},
            "data_retention": ret,
            "compliance_status": {"retention_policy_configured": ent.data_retention_days is not None,
                                  "retention_policy_enforced": ret.get("retention_compliance", False),
                                  "logging_controlled": True, "anonymization_enabled": bool(ent.anonymize_data)},
            "recommendations": self._generate_recommendations(ent),
        }

    @staticmethod
    def _generate_recommendations(ent: Enterprise) -> List[str]:
        rec = []
        if ent.data_retention_days is None:
            rec.append("Configure a data-retention policy")
        elif ent.data_retention_days > 90:
            rec.append("Retention period exceeds 90 days; consider shortening it")
        if ent.allow_logging and not ent.anonymize_data:
            rec.append("Logging is enabled without anonymization; enable anonymize_data")
        if not ent.private_deployment:
            rec.append("Consider private deployment for highly sensitive workloads")
        return rec


class EnterprisePrivacyService:
    SETTINGS = ("data_retention_days", "allow_logging", "anonymize_data", "private_deployment")

    def __init__(self, db: Session, encryption_key: Optional[str] = None):
        self.db = db
        self.anonymizer = DataAnonymizer()
        self.encryptor = DataEncryptor(encryption_key) if encryption_key else None
        self.retention_service = DataRetentionService(db)
        self.audit_service = PrivacyAuditService(db)

    def get_enterprise_privacy_settings(self, enterprise_id: str) -> Dict[str, Any]:
        ent = self.db.get(Enterprise, enterprise_id)
        if ent is None:
            return {}
        return {"enterprise_id": str(enterprise_id),
                "data_retention_days": ent.data_retention_days or PrivacyConfig.DEFAULT_RETENTION_DAYS,
                "allow_logging": ent.allow_logging, "anonymize_data": ent.anonymize_data,
                "private_deployment": ent.private_deployment}

    def update_privacy_settings(self, enterprise_id: str, changed_by: str, settings: Dict[str, Any]) -> bool:
        ent = self.db.get(Enterprise, enterprise_id)
        if ent is None:
            return False
        for k, v in settings.items():
            if k not in self.SETTINGS or v is None:
                continue
            if k == "data_retention_days":
                v = max(PrivacyConfig.MIN_RETENTION_DAYS, min(PrivacyConfig.MAX_RETENTION_DAYS, int(v)))
            old = getattr(ent, k)
            if old != v:
                self.audit_service.log_privacy_setting_change(enterprise_id, changed_by, k, old, v)
                setattr(ent, k, v)
        self.db.commit()
        return True

    def process_data_for_storage(self, enterprise_id: str, data: Dict, data_type: str) -> Dict:
        s = self.get_enterprise_privacy_settings(enterprise_id)
        if not s:
            return data
        out = dict(data)
        if not s["allow_logging"]:
            out = self._remove_sensitive_content(out)
        if s["anonymize_data"]:
            out = self.anonymizer.anonymize_dict(out)
        if self.encryptor is not None:
            out = self.encryptor.encrypt_dict(out, PrivacyConfig.SENSITIVE_FIELDS)
        return out

    def process_data_for_retrieval(self, enterprise_id: str, data: Dict, accessor_id: str) -> Dict:
        self.audit_service.log_data_access(enterprise_id, accessor_id, "api_key", "usage_data", "read")
        return self.encryptor.decrypt_dict(data) if self.encryptor is not None else data

    def export_enterprise_data(self, enterprise_id: str, exporter_id: str, export_format: str = "json",
                               include_sensitive: bool = False) -> Tuple[str, Dict]:
        ent = self.db.get(Enterprise, enterprise_id)
        if ent is None:
            return "", {}
        recs = self.db.execute(select(UsageRecord).where(UsageRecord.enterprise_id == enterprise_id)).scalars().all()
        bills = self.db.execute(select(Bill).where(Bill.enterprise_id == enterprise_id)).scalars().all()
        iso = lambda d: d.isoformat() if d else None  # noqa: E731
        data = {
            "enterprise": {"id": str(ent.id), "name": ent.name, "code": ent.code, "created_at": iso(ent.created_at)},
            "usage_records": [{"id": str(r.id), "job_type": r.job_type, "usage_type": r.usage_type,
                               "quantity": r.quantity, "total_cost": r.total_cost, "created_at": iso(r.created_at)}
                              for r in recs],
            "bills": [{"id": str(b.id), "period_start": iso(b.period_start), "period_end": iso(b.period_end),
                       "total": b.total, "status": b.status} for b in bills],
            "export_metadata": {"exported_at": datetime.utcnow().isoformat(), "exporter_id": exporter_id,
                                "include_sensitive": include_sensitive},
        }
        if not include_sensitive:
            data = self.anonymizer.anonymize_dict(data)
        self.audit_service.log_data_export(enterprise_id, exporter_id, export_format, len(recs) + len(bills),
                                           "user_download")
        return json.dumps(data, indent=2, ensure_ascii=False), data

    def delete_enterprise_data(self, enterprise_id: str, requester_id: str, confirm: bool = False) -> Dict[str, Any]:
        n_use = self.db.execute(select(func.count(UsageRecord.id)).where(
            UsageRecord.enterprise_id == enterprise_id)).scalar() or 0
        n_bill = self.db.execute(select(func.count(Bill.id)).where(Bill.enterprise_id == enterprise_id)).scalar() or 0
        if not confirm:
            return {"status": "preview", "data_to_delete": {"usage_records": int(n_use), "bills": int(n_bill)},
                    "message": "Set confirm=true to delete"}
        self.db.execute(delete(UsageRecord).where(UsageRecord.enterprise_id == enterprise_id))
        self.db.execute(delete(Bill).where(Bill.enterprise_id == enterprise_id))
        self.db.commit()
        self.audit_service.log_data_access(enterprise_id, requester_id, "user", "all", "delete",
                                           record_count=int(n_use + n_bill),
                                           details={"reason": "right_to_be_forgotten"})
        logger.warning("enterprise data deleted: %s usage_records=%d bills=%d", enterprise_id, n_use, n_bill)
        return {"status": "deleted", "deleted": {"usage_records": int(n_use), "bills": int(n_bill)},
                "deleted_at": datetime.utcnow().isoformat()}

    def run_scheduled_cleanup(self) -> Dict[str, Any]:
        stats = self.retention_service.cleanup_expired_data()
        logger.info("scheduled privacy cleanup: %s", stats)
        return {"status": "completed", "stats": stats, "completed_at": datetime.utcnow().isoformat()}

    @staticmethod
    def _remove_sensitive_content(data: Dict) -> Dict:
        out = dict(data)
        for f in PrivacyConfig.CONTENT_FIELDS:
            if f in out:
                out[f] = "[NOT_LOGGED]"
        return out
