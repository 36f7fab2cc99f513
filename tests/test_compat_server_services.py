"""Control-plane services: geo, privacy, security, reliability, task guarantee,
scheduler and usage.

Behavioural parity with the reference's tests/test_server_{geo,privacy,
security}.py (offline region detection, anonymisation / PII / encryption,
token hashing, request signatures, auth branches against an AsyncSession
mock) plus the service logic the reference never tested (reliability score
deltas, offline requeue / retry exhaustion, stale-job and dead-worker
sweeps, atomic job assignment, pricing) on a private in-memory SQLite DB.
"""
import asyncio
from datetime import datetime, timedelta
from unittest.mock import AsyncMock

import pytest
from sqlalchemy.orm import sessionmaker

from app.db.database import Base, make_engine
from app.models.models import Job, JobStatus, Worker, WorkerStatus
from app.services.geo import detect_client_region, get_region_info, get_region_name
from app.services.privacy import DataAnonymizer, DataEncryptor
from app.services.reliability import ReliabilityService
from app.services.security import RequestSigner, SecurityService, SecuritySettings, TokenManager
from app.services.task_guarantee import TaskGuaranteeService


@pytest.fixture
def db():
    from app.models import models, usage  # noqa: F401  (register tables)
    eng = make_engine("sqlite:///:memory:")
    Base.metadata.create_all(bind=eng)
    s = sessionmaker(bind=eng, expire_on_commit=False)()
    yield s
    s.close()
    eng.dispose()


def _worker(db, **kw):
    w = Worker(name=kw.pop("name", "w"), status=kw.pop("status", WorkerStatus.ONLINE.value),
               supported_types=kw.pop("supported_types", ["llm"]), **kw)
    db.add(w)
    db.commit()
    return w


def _job(db, **kw):
    j = Job(type=kw.pop("type", "llm"), params=kw.pop("params", {"prompt": "x"}), **kw)
    db.add(j)
    db.commit()
    return j


# ----------------------------------------------------------------------------- geo

@pytest.mark.parametrize("ip", [None, "10.0.0.1", "192.168.1.4", "127.0.0.1", "localhost", "172.16.0.9"])
def test_geo_private_and_missing_default_to_asia_east(ip):
    assert asyncio.run(detect_client_region(ip)) == "asia-east"


@pytest.mark.parametrize("ip,region", [("2.1.1.1", "europe-west"), ("3.9.9.9", "america-north")])
def test_geo_prefix_table(ip, region):
    assert asyncio.run(detect_client_region(ip)) == region


def test_geo_region_names():
    assert "东亚" in get_region_name("asia-east")
    assert get_region_name("unknown") == "unknown"
    assert isinstance(get_region_info("europe-west"), dict)


# ----------------------------------------------------------------------------- privacy

@pytest.fixture
def anon():
    return DataAnonymizer(salt="s")


def test_email_keeps_domain(anon):
    out = anon.anonymize_string("user@example.com", preserve_format=True)
    assert out.endswith("@example.com") and "***@" in out


@pytest.mark.parametrize("raw,check", [("1234", lambda m: m == "****"),
                                       ("1234567890", lambda m: m[:2] == "12" and m[-2:] == "90" and "*" in m)])
def test_digit_masking(anon, raw, check):
    assert check(anon.anonymize_string(raw, preserve_format=True))


def test_hash_mode_is_stable_and_salted(anon):
    a = anon.anonymize_string("secret")
    assert a == anon.anonymize_string("secret") and "secret" not in a
    assert DataAnonymizer(salt="other").anonymize_string("secret") != a


def test_ip_truncation(anon):
    assert anon.anonymize_ip("1.2.3.4") == "1.2.xxx.xxx"
    assert anon.anonymize_ip("2001:db8:abcd:0012::1").startswith("2001:db8::")


def test_pii_removed_from_preview(anon):
    out = anon.anonymize_content("mail test@example.com or call 13800138000", max_preview=200)
    assert "[EMAIL]" in out and "[PHONE_CN]" in out and "test@example.com" not in out


def test_recursive_dict_redaction(anon):
    out = anon.anonymize_dict({"prompt": "secret text", "nested": {"token": "abc", "keep": 1},
                               "items": [{"password": "p"}]})
    assert out["prompt"].startswith("[") and out["nested"]["keep"] == 1
    assert out["nested"]["token"] == "[REDACTED]" and out["items"][0]["password"] == "[REDACTED]"


def test_encryption_roundtrip_wrong_key_and_tamper():
    e = DataEncryptor(encryption_key="k1")
    ct = e.encrypt("hello")
    assert ct != "hello" and e.decrypt(ct) == "hello"
    assert DataEncryptor(encryption_key="k2").decrypt(ct) == "[DECRYPTION_FAILED]"
    assert e.decrypt(ct[:-4] + "AAAA") == "[DECRYPTION_FAILED]"
    assert e.encrypt("hello") != ct   # fresh nonce per message


def test_encrypt_dict_fields():
    e = DataEncryptor(encryption_key="k")
    d = e.encrypt_dict({"prompt": {"a": 1}, "keep": 2}, ["prompt"])
    assert d["keep"] == 2 and d["prompt"] != {"a": 1}
    assert e.decrypt_dict(d)["prompt"] == {"a": 1}


# ----------------------------------------------------------------------------- security

def test_token_hash_roundtrip():
    h = TokenManager.hash_token("t")
    assert TokenManager.verify_token_hash("t", h) and not TokenManager.verify_token_hash("wrong", h)
    assert not TokenManager.verify_token_hash("t", None)
    assert TokenManager.hash_token("t") != TokenManager.hash_token("t")   # salted


def test_signature_ok_tampered_and_expired():
    ts = int(datetime.utcnow().timestamp())
    sig = RequestSigner.sign_request("POST", "/x", '{"a":1}', ts, "secret")
    assert RequestSigner.verify_signature("POST", "/x", '{"a":1}', ts, sig, "secret") == (True, "")
    assert RequestSigner.verify_signature("POST", "/x", '{"a":2}', ts, sig, "secret") == (False, "invalid_signature")
    old = ts - (SecuritySettings.SIGNATURE_VALIDITY_SECONDS + 1)
    sig = RequestSigner.sign_request("GET", "/x", None, old, "secret")
    assert RequestSigner.verify_signature("GET", "/x", None, old, sig, "secret") == (False, "signature_expired")


def test_refresh_threshold():
    svc = SecurityService(AsyncMock())

    class W:
        token_expires_at = None
    w = W()
    assert svc.should_refresh_token(w) is False
    w.token_expires_at = datetime.utcnow()
    assert svc.should_refresh_token(w) is True
    w.token_expires_at = datetime.utcnow() + timedelta(days=2)
    assert svc.should_refresh_token(w) is False


def test_signature_requires_secret_async_api():
    svc = SecurityService(AsyncMock())

    class W:
        signing_secret = None
    ok, err = asyncio.run(svc.verify_request_signature(W(), "GET", "/x", None, 1, "sig"))
    assert (ok, err) == (False, "no_signing_secret")


class _Res:
    def __init__(self, w):
        self.w = w

    def scalar_one_or_none(self):
        return self.w


class _W:
    def __init__(self, **kw):
        self.id = "00000000-0000-0000-0000-000000000000"
        self.locked_until = None
        self.auth_token_hash = TokenManager.hash_token("good")
        self.refresh_token_hash = None
        self.token_expires_at = None
        self.failed_auth_attempts = 1
        self.last_failed_auth = None
        self.__dict__.update(kw)


@pytest.mark.parametrize("worker,token,err", [
    (None, "x", "worker_not_found"),
    (_W(locked_until=datetime.utcnow() + timedelta(days=1)), "good", "account_locked"),
    (_W(), "bad", "invalid_token"),
    (_W(token_expires_at=datetime.utcnow() - timedelta(seconds=1)), "good", "token_expired"),
    (_W(failed_auth_attempts=2), "good", ""),
])
def test_auth_branches_async_session(worker, token, err):
    db = AsyncMock()
    db.execute.return_value = _Res(worker)
    w, e = asyncio.run(SecurityService(db).verify_worker_auth("00000000-0000-0000-0000-000000000000", token))
    assert e == err
    if err == "":
        assert w is worker and worker.failed_auth_attempts == 0


def test_auth_lockout_after_repeated_failures_sync_session(db):
    w = _worker(db, auth_token_hash=TokenManager.hash_token("good"))
    svc = SecurityService(db)
    for _ in range(SecuritySettings.MAX_FAILED_ATTEMPTS):
        assert svc.verify_worker_auth(w.id, "bad")[1] == "invalid_token"
    assert svc.verify_worker_auth(w.id, "good")[1] == "account_locked"


def test_issue_and_refresh_tokens(db):
    w = _worker(db)
    svc = SecurityService(db)
    tok, ref = svc.issue_tokens(w)
    db.commit()
    assert svc.verify_worker_auth(w.id, tok) == (w, "")
    assert svc.refresh_tokens(w, "nope") is None
    tok2, _ = svc.refresh_tokens(w, ref)
    assert svc.verify_worker_auth(w.id, tok2)[1] == "" and svc.verify_worker_auth(w.id, tok)[1] == "invalid_token"


# ----------------------------------------------------------------------------- reliability

@pytest.mark.parametrize("event,delta", [("job_completed", 0.02), ("job_failed", -0.05),
                                         ("unexpected_offline", -0.15), ("graceful_offline", -0.02),
                                         ("long_session", 0.05)])
def test_reliability_deltas(event, delta):
    w = Worker(reliability_score=0.5, total_jobs=0, completed_jobs=0, failed_jobs=0, unexpected_offline_count=0)
    ReliabilityService().update_score(w, event, commit=False)
    assert w.reliability_score == pytest.approx(0.5 + delta)


def test_reliability_bounds_success_rate_and_latency():
    w = Worker(reliability_score=0.99, total_jobs=0, completed_jobs=0, failed_jobs=0)
    svc = ReliabilityService()
    svc.update_score(w, "job_completed", commit=False, latency_ms=50)
    assert w.reliability_score == 1.0 and w.avg_latency_ms == 50
    for _ in range(30):
        svc.update_score(w, "job_failed", commit=False)
    assert w.reliability_score == pytest.approx(0.1) and w.success_rate == pytest.approx(1 / 31)


def test_online_prediction_uses_hourly_pattern():
    w = Worker(reliability_score=1.0)
    svc = ReliabilityService()
    assert svc.predict_online_probability(w) == 0.5
    for _ in range(20):
        svc.update_score(w, "heartbeat", commit=False)
    assert svc.predict_online_probability(w, hours_ahead=0) > 0.8
    svc.start_session(w, commit=False)
    assert svc.predict_remaining_online_time(w) > 0


# ----------------------------------------------------------------------------- task guarantee

def test_offline_worker_jobs_requeue_then_fail(db):
    w = _worker(db)
    j1 = _job(db, status=JobStatus.RUNNING.value, worker_id=w.id, retry_count=0)
    j2 = _job(db, status=JobStatus.RUNNING.value, worker_id=w.id, retry_count=3, max_retries=3)
    out = TaskGuaranteeService(db).handle_worker_offline(w.id)
    assert out == {"requeued": 1, "failed": 1}
    db.refresh(j1)
    db.refresh(j2)
    assert (j1.status, j1.worker_id, j1.retry_count) == (JobStatus.QUEUED.value, None, 1)
    assert j2.status == JobStatus.FAILED.value
    db.refresh(w)
    assert w.status == WorkerStatus.OFFLINE.value and w.reliability_score < 1.0


def test_stale_job_and_dead_worker_sweeps(db):
    w = _worker(db, last_heartbeat=datetime.utcnow() - timedelta(hours=1))
    alive = _worker(db, name="alive", last_heartbeat=datetime.utcnow())
    stale = _job(db, status=JobStatus.RUNNING.value, worker_id=alive.id,
                 started_at=datetime.utcnow() - timedelta(hours=2), retry_count=5, max_retries=3)
    svc = TaskGuaranteeService(db)
    assert svc.check_stale_jobs() == 1
    db.refresh(stale)
    assert stale.status == JobStatus.TIMEOUT.value
    assert svc.check_dead_workers(timeout_seconds=90) == 1
    db.refresh(w)
    db.refresh(alive)
    assert w.status == WorkerStatus.OFFLINE.value and alive.status == WorkerStatus.ONLINE.value


def test_job_fallback_returns_terminal_or_times_out(db):
    j = _job(db, status=JobStatus.COMPLETED.value)
    svc = TaskGuaranteeService(db)
    assert asyncio.run(svc.get_job_with_fallback(j.id)).status == JobStatus.COMPLETED.value
    q = _job(db)
    with pytest.raises(TimeoutError):
        asyncio.run(svc.get_job_with_fallback(q.id, max_wait_seconds=0.2))


# ----------------------------------------------------------------------------- smart scheduler

def test_atomic_assignment_respects_type_priority_and_order(db):
    from app.services.scheduler import SmartScheduler
    w = _worker(db, supported_types=["llm"])
    _job(db, type="image_gen", priority=100)
    low = _job(db, priority=1)
    high = _job(db, priority=5)
    sched = SmartScheduler(db)
    first = sched.atomic_assign_job(w.id, w.supported_types, worker=w)
    assert first.id == high.id and first.status == JobStatus.RUNNING.value and first.worker_id == w.id
    assert sched.atomic_assign_job(w.id, ["llm"], worker=w).id == low.id
    assert sched.atomic_assign_job(w.id, ["llm"], worker=w) is None   # only the image job is left
    assert sched.atomic_assign_job(w.id, [], worker=w) is None


def test_role_aware_assignment_prefers_matching_phase(db):
    from app.services.scheduler import SmartScheduler
    w = _worker(db, supported_types=["llm"], role="decode")
    _job(db, phase="prefill")
    dec = _job(db, phase="decode")
    assert SmartScheduler(db).atomic_assign_job(w.id, ["llm"], worker=w).id == dec.id


def test_queue_stats_and_wait_estimate(db):
    from app.services.scheduler import SmartScheduler
    _worker(db)
    for _ in range(3):
        _job(db)
    _job(db, type="image_gen")
    st = SmartScheduler(db).get_queue_stats()
    assert st["total_queued"] == 4 and st["by_type"] == {"llm": 3, "image_gen": 1}
    assert st["available_workers"] == 1 and st["estimated_wait_seconds"] == 120
