"""Control-plane tests: services (geo, privacy, observability, security, worker config,
P/D scheduler) and an end-to-end FastAPI flow with simulated workers.

Mirrors the reference's server unit tests (tests/test_server_{geo,privacy,
observability,security,pd_scheduler}.py) and adds the API flow the
reference never tested (register → submit → pull → complete → usage → admin).
"""
import asyncio
import importlib.util
import sys
import threading
import time
from datetime import datetime, timedelta
from pathlib import Path
from unittest.mock import MagicMock, patch

import pytest

ROOT = Path(__file__).resolve().parents[1]


# ----------------------------------------------------------------- geo
def test_geo_offline_defaults_and_prefixes():
    from app.services.geo import detect_client_region, get_region_name
    assert asyncio.run(detect_client_region(None)) == "asia-east"
    assert asyncio.run(detect_client_region("10.0.0.1")) == "asia-east"
    assert asyncio.run(detect_client_region("localhost")) == "asia-east"
    assert asyncio.run(detect_client_region("2.1.1.1")) == "europe-west"
    assert asyncio.run(detect_client_region("3.9.9.9")) == "america-north"
    assert "东亚" in get_region_name("asia-east")
    assert get_region_name("unknown") == "unknown"


# ----------------------------------------------------------------- privacy
def test_privacy_anonymizer():
    from app.services.privacy import DataAnonymizer
    a = DataAnonymizer(salt="s")
    out = a.anonymize_string("user@example.com", preserve_format=True)
    assert out.endswith("@example.com") and "***@" in out
    assert a.anonymize_string("1234", preserve_format=True) == "****"
    m = a.anonymize_string("1234567890", preserve_format=True)
    assert m.startswith("12") and m.endswith("90") and "*" in m
    assert a.anonymize_ip("1.2.3.4") == "1.2.xxx.xxx"
    assert a.anonymize_ip("2001:db8:abcd:0012::1").startswith("2001:db8::")
    c = a.anonymize_content("contact me at test@example.com and call 13800138000", max_preview=200)
    assert "[EMAIL]" in c and "[PHONE_CN]" in c
    d = a.anonymize_dict({"prompt": "secret text", "nested": {"token": "abc", "keep": 1}, "items": [{"password": "p"}]})
    assert d["prompt"].startswith("[") and d["nested"]["token"] == "[REDACTED]" and d["nested"]["keep"] == 1
    assert d["items"][0]["password"] == "[REDACTED]"
    assert a.create_pseudonym("x") == a.create_pseudonym("x") != a.create_pseudonym("y")


def test_privacy_encryptor_roundtrip_wrong_key_and_tamper():
    from app.services.privacy import DataEncryptor
    e1 = DataEncryptor(encryption_key="k1")
    ct = e1.encrypt("hello")
    assert e1.decrypt(ct) == "hello"
    assert DataEncryptor(encryption_key="k2").decrypt(ct) == "[DECRYPTION_FAILED]"
    assert e1.decrypt(ct[:-4] + "AAAA") == "[DECRYPTION_FAILED]"
    d = e1.encrypt_dict({"prompt": {"a": 1}, "keep": 2}, ["prompt"])
    assert d["prompt"] != {"a": 1} and e1.decrypt_dict(d) == {"prompt": {"a": 1}, "keep": 2}


# ----------------------------------------------------------------- observability
def _load_observability_with_mocks():
    class _Metric:
        def __init__(self, name, desc, labels, buckets=None):
            self.values = {}

        def labels(self, **kw):
            return self.values.setdefault(tuple(sorted(kw.items())), MagicMock())
    prom = MagicMock()
    prom.Counter = prom.Gauge = prom.Histogram = _Metric
    prom.generate_latest = MagicMock(return_value=b"# metrics")
    prom.CONTENT_TYPE_LATEST = "text/plain"
    with patch.dict(sys.modules, {"prometheus_client": prom, "opentelemetry": MagicMock(),
                                  "opentelemetry.trace": MagicMock()}):
        spec = importlib.util.spec_from_file_location(
            "obs_under_test", ROOT / "server" / "app" / "services" / "observability.py")
        mod = importlib.util.module_from_spec(spec)
        sys.modules["obs_under_test"] = mod
        spec.loader.exec_module(mod)
    return mod


def test_observability_collector_and_logger():
    obs = _load_observability_with_mocks()
    t = obs.TracingManager("svc")
    assert t._tracer is None and t._enabled is False
    with t.span("x") as sp:
        assert sp is None
    c = obs.MetricsCollector(worker_id="w1", model_name="m", worker_role="hybrid")
    for i in range(3):
        c.record_request("decode", 0.1 * (i + 1), tokens=10, success=i != 1)
    c.record_batch("prefill", 8)
    c.record_kv_cache_stats("gpu", 0.9, 100, 2)
    c.record_gpu_stats(0, 1, 2, 50.0)
    c.record_speculative_stats(0.7, 1.5)
    s = c.get_summary()
    assert s["total_requests"] == 3 and s["error_count"] == 1
    assert s["avg_latency_ms"] == pytest.approx(200, rel=1e-3)
    c.update_tokens_per_second()
    assert c._token_count == 0
    app = MagicMock()
    obs.setup_metrics_routes(app)
    app.include_router.assert_called_once()
    lg = obs.StructuredLogger("t")
    lg.set_context(session_id="abc")
    with patch.object(lg.logger, "info") as mi:
        lg.info("m", request_id="r1")
        extra = mi.call_args.kwargs["extra"]
        assert extra["session_id"] == "abc" and extra["request_id"] == "r1"
    with patch.object(obs, "HAS_PROMETHEUS", False):
        assert "error" in asyncio.run(obs.create_metrics_endpoint()())


# ----------------------------------------------------------------- security / config
def test_security_signer_and_tokens():
    from app.services.security import RequestSigner, TokenManager
    tok = TokenManager.generate_token()
    h = TokenManager.hash_token(tok)
    assert TokenManager.verify_token_hash(tok, h) and not TokenManager.verify_token_hash(tok + "x", h)
    ts = int(time.time())
    sig = RequestSigner.sign_request("POST", "/p", {"a": 1}, ts, "sec")
    ok, _ = RequestSigner.verify_signature("POST", "/p", {"a": 1}, ts, sig, "sec")
    assert ok
    ok, _ = RequestSigner.verify_signature("POST", "/p", {"a": 2}, ts, sig, "sec")
    assert not ok
    ok, err = RequestSigner.verify_signature("POST", "/p", {"a": 1}, ts - 3600, sig, "sec")
    assert not ok


def test_worker_config_should_accept():
    import random
    from app.services.worker_config import LoadControlConfig, WorkerConfigService as S
    assert S.should_accept_job(LoadControlConfig(), "llm")[0]
    assert S.should_accept_job(LoadControlConfig(max_jobs_per_hour=2), "llm", 2) == (False, "hourly_limit_reached")
    lc = LoadControlConfig(working_hours_start=22, working_hours_end=6)
    assert S.should_accept_job(lc, "llm", now=datetime(2025, 1, 1, 23))[0]
    assert not S.should_accept_job(lc, "llm", now=datetime(2025, 1, 1, 12))[0]
    assert S.should_accept_job(LoadControlConfig(type_weights={"llm": 0.0}), "llm")[1] == "job_type_disabled"
    rng = random.Random(0)
    n = sum(S.should_accept_job(LoadControlConfig(acceptance_rate=0.3), "llm", rng=rng)[0] for _ in range(2000))
    assert 450 < n < 750


def test_pd_scheduler_tracks_load():
    from app.services.pd_scheduler import JobPhase, PrefillDecodeScheduler, WorkerCapability, WorkerRole
    s = PrefillDecodeScheduler()
    s.register_worker("p", WorkerCapability(worker_id="p", role=WorkerRole.PREFILL, compute_flops=2500))
    s.register_worker("d", WorkerCapability(worker_id="d", role=WorkerRole.DECODE,
                                                 memory_bandwidth_gbps=8000))

    async def flow():
        await s.submit_job("j1", prompt_tokens=100, max_tokens=10)
        [(job, a)] = await s.get_batch(JobPhase.PREFILL)
        assert a.worker_id == "p" and s._workers["p"].active_prefill_jobs == 1
        await s.transition_to_decode("j1", "kv1", "p")
        assert s._workers["p"].active_prefill_jobs == 0
        [(job, a)] = await s.get_batch(JobPhase.DECODE)
        assert a.worker_id == "d" and a.kv_migration_needed and a.migration_source == "p" and s._workers["d"].active_decode_jobs == 1
        await s.complete_job("j1", JobPhase.DECODE, latency_ms=5.0)
        assert s._workers["d"].active_decode_jobs == 0
    asyncio.run(flow())
    st = s.get_stats()
    assert st["prefill_jobs"] == 1 and st["decode_jobs"] == 1 and st["kv_cache_entries"] == 1


# ----------------------------------------------------------------- end-to-end API
@pytest.fixture()
def client():
    from fastapi.testclient import TestClient
    from app.db.database import Base, engine
    from app.main import app
    Base.metadata.drop_all(bind=engine)
    with TestClient(app) as c:
        yield c
    Base.metadata.drop_all(bind=engine)


def _register(c, **kw):
    body = {"name": "mi355x-node", "region": "asia-east", "gpu_model": "AMD Instinct MI355X", "gpu_memory_gb": 288,
            "gpu_count": 8, "supported_types": ["llm"], **kw}
    r = c.post("/api/v1/workers/register", json=body)
    assert r.status_code == 200, r.text
    d = r.json()
    return d["worker_id"], {"X-Worker-Token": d["token"]}, d


def test_api_job_lifecycle_with_usage(client):
    c = client
    assert c.get("/health").json()["status"] == "healthy"
    assert len(c.get("/regions").json()["available_regions"]) == 7
    ent = c.post("/api/v1/admin/enterprises", json={"name": "Acme", "code": "acme"}).json()
    key = c.post(f"/api/v1/admin/enterprises/{ent['id']}/api-keys", json={"name": "k"}).json()["api_key"]
    assert key.startswith("ent_")
    wid, hdr, _ = _register(c)
    assert c.post(f"/api/v1/workers/{wid}/heartbeat", json={"status": "online"}, headers=hdr).json()["status"] == "ok"
    assert c.post(f"/api/v1/workers/{wid}/heartbeat", json={"status": "online"},
                  headers={"X-Worker-Token": "bad"}).status_code == 401
    r = c.post("/api/v1/jobs", json={"type": "llm", "params": {"messages": [{"role": "user", "content": "hi"}],
                                                                "max_tokens": 8}}, headers={"X-API-Key": key})
    assert r.status_code == 200, r.text
    job_id = r.json()["job_id"]
    assert r.json()["status"] == "queued"
    assert c.get("/api/v1/jobs/stats/queue").json()["total_queued"] == 1
    a = c.get(f"/api/v1/workers/{wid}/next-job", headers=hdr).json()
    assert a["job_id"] == job_id and a["params"]["max_tokens"] == 8
    assert c.get(f"/api/v1/workers/{wid}/next-job", headers=hdr).json() is None
    res = {"response": "hello", "usage": {"prompt_tokens": 3, "completion_tokens": 5, "total_tokens": 8},
           "finish_reason": "length"}
    r = c.post(f"/api/v1/workers/{wid}/jobs/{job_id}/complete", json={"success": True, "result": res,
                                                                       "processing_time_ms": 40}, headers=hdr)
    assert r.status_code == 200, r.text
    j = c.get(f"/api/v1/jobs/{job_id}").json()
    assert j["status"] == "completed" and j["result"]["response"] == "hello" and j["worker_id"] == wid
    recs = c.get("/api/v1/admin/usage/records").json()
    assert recs["total"] == 1 and recs["items"][0]["usage_type"] == "llm_tokens"
    assert recs["items"][0]["total_cost"] == pytest.approx(0.002 * 8 / 1000)
    assert c.get("/api/v1/admin/dashboard").json()["today"]["jobs"] == 1
    assert c.get("/api/v1/admin/usage/summary?group_by=type").json()["items"][0]["key"] == "llm_tokens"
    w = c.get(f"/api/v1/workers/{wid}").json()
    assert w["completed_jobs"] == 1 and w["success_rate"] == 1.0
    assert c.get("/api/v1/admin/dashboard/realtime").json()["workers"]["online"] == 1
    assert c.get("/api/v1/admin/health/detailed").json()["database"] is True
    # privacy endpoints
    p = c.get(f"/api/v1/admin/enterprises/{ent['id']}/privacy").json()
    assert p["data_retention_days"] == 30
    c.put(f"/api/v1/admin/enterprises/{ent['id']}/privacy", json={"anonymize_data": True})
    assert c.get(f"/api/v1/admin/enterprises/{ent['id']}/privacy/compliance").json()["compliance_status"][
        "anonymization_enabled"] is True
    exp = c.post(f"/api/v1/admin/enterprises/{ent['id']}/privacy/export").json()
    assert len(exp["usage_records"]) == 1
    prev = c.delete(f"/api/v1/admin/enterprises/{ent['id']}/privacy/data").json()
    assert prev["status"] == "preview" and prev["data_to_delete"]["usage_records"] == 1
    assert c.delete(f"/api/v1/admin/enterprises/{ent['id']}/privacy/data?confirm=true").json()["status"] == "deleted"
    assert c.get("/api/v1/admin/usage/records").json()["total"] == 0
    assert c.get("/metrics").status_code == 200 and c.get("/ready").json()["status"] == "ready"


def test_api_cancel_offline_requeue_and_concurrency(client):
    c = client
    wid, hdr, _ = _register(c)
    c.put(f"/api/v1/workers/{wid}/config", json={"max_concurrent_jobs": 2}, headers=hdr)
    cfg = c.get(f"/api/v1/workers/{wid}/config", headers=hdr).json()
    assert cfg["load_control"]["max_concurrent_jobs"] == 2 and cfg["version"] == 1
    ids = [c.post("/api/v1/jobs", json={"type": "llm", "params": {"prompt": str(i)}}).json()["job_id"]
           for i in range(4)]
    assert c.delete(f"/api/v1/jobs/{ids[3]}").json()["job_id"] == ids[3]
    got = [c.get(f"/api/v1/workers/{wid}/next-job", headers=hdr).json() for _ in range(3)]
    assert got[0] and got[1] and got[2] is None          # capped at 2 concurrent
    assert c.get(f"/api/v1/workers/{wid}").json()["status"] == "busy"
    assert c.delete(f"/api/v1/jobs/{got[0]['job_id']}").status_code == 400
    r = c.post(f"/api/v1/workers/{wid}/offline", headers=hdr).json()
    assert r["requeued"] == 2
    assert all(c.get(f"/api/v1/jobs/{g['job_id']}").json()["status"] == "queued" for g in got[:2])
    # a second worker picks the requeued work up
    wid2, hdr2, _ = _register(c, region="europe-west")
    assert c.get(f"/api/v1/workers/{wid2}/next-job", headers=hdr2).json()["job_id"] in ids
    # token refresh
    _, _, reg = _register(c)
    r = c.post(f"/api/v1/workers/{reg['worker_id']}/refresh-token", json={"refresh_token": reg["refresh_token"]})
    assert r.status_code == 200
    new = {"X-Worker-Token": r.json()["token"]}
    assert c.post(f"/api/v1/workers/{reg['worker_id']}/verify", headers=new).json()["valid"] is True
    assert c.post(f"/api/v1/workers/{reg['worker_id']}/verify",
                  headers={"X-Worker-Token": reg["token"]}).json()["valid"] is False


def test_advertised_worker_concurrency_is_honoured(client):
    """A continuous-batching worker advertises how many jobs it runs at once
    (``capabilities.max_concurrent_jobs``): the pull API hands it that many and its remote
    config says so (the worker applies the remote load control, so a default of 1 there
    serialised every job of a batching engine).  An admin override still wins, and a worker
    that advertises nothing keeps one job at a time."""
    c = client
    wid, hdr, _ = _register(c, capabilities={"max_concurrent_jobs": 3, "continuous_batching": True})
    legacy, lhdr, _ = _register(c, region="europe-west")
    assert c.get(f"/api/v1/workers/{wid}/config", headers=hdr).json()["load_control"]["max_concurrent_jobs"] == 3
    assert c.get(f"/api/v1/workers/{legacy}/config", headers=lhdr).json()["load_control"]["max_concurrent_jobs"] == 1
    for i in range(5):
        c.post("/api/v1/jobs", json={"type": "llm", "params": {"prompt": str(i)}, "region": "asia-east"})
    got = [c.get(f"/api/v1/workers/{wid}/next-job", headers=hdr).json() for _ in range(4)]
    assert all(got[:3]) and got[3] is None
    assert c.get(f"/api/v1/workers/{legacy}/next-job", headers=lhdr).json() is not None
    assert c.get(f"/api/v1/workers/{legacy}/next-job", headers=lhdr).json() is None
    c.put(f"/api/v1/workers/{wid}/config", json={"max_concurrent_jobs": 2}, headers=hdr)     # admin override
    assert c.get(f"/api/v1/workers/{wid}/config", headers=hdr).json()["load_control"]["max_concurrent_jobs"] == 2


def test_api_sync_job_completed_by_worker_thread(client):
    c = client
    wid, hdr, _ = _register(c)
    stop = threading.Event()

    def worker_loop():
        from fastapi.testclient import TestClient
        from app.main import app
        wc = TestClient(app)
        while not stop.is_set():
            a = wc.get(f"/api/v1/workers/{wid}/next-job", headers=hdr).json()
            if a:
                wc.post(f"/api/v1/workers/{wid}/jobs/{a['job_id']}/complete",
                        json={"success": True, "result": {"echo": a["params"]["prompt"]}}, headers=hdr)
                return
            time.sleep(0.05)
    t = threading.Thread(target=worker_loop, daemon=True)
    t.start()
    r = c.post("/api/v1/jobs/sync?timeout=20", json={"type": "llm", "params": {"prompt": "ping"}})
    stop.set()
    t.join(5)
    assert r.status_code == 200, r.text
    assert r.json()["status"] == "completed" and r.json()["result"] == {"echo": "ping"}
    r = c.post("/api/v1/jobs/sync?timeout=1&wait_for_worker=true", json={"type": "image_gen", "params": {}})
    assert r.status_code == 408


def test_next_job_long_poll_wakes_on_a_new_job(client):
    """GET next-job?wait=S keeps the request open and hands over a job queued while it waits (the
    reference's workers only see it at their next poll, 2 s by default); with nothing queued it
    returns null after ``wait``; without ``wait`` it answers at once as before."""
    c = client
    wid, hdr, _ = _register(c)
    t0 = time.perf_counter()
    assert c.get(f"/api/v1/workers/{wid}/next-job", headers=hdr).json() is None
    assert time.perf_counter() - t0 < 0.2
    t0 = time.perf_counter()
    assert c.get(f"/api/v1/workers/{wid}/next-job?wait=0.3", headers=hdr).json() is None
    assert time.perf_counter() - t0 >= 0.3
    got = {}

    def poll():
        from fastapi.testclient import TestClient
        from app.main import app
        wc = TestClient(app)
        t = time.perf_counter()
        got["a"] = wc.get(f"/api/v1/workers/{wid}/next-job?wait=10", headers=hdr).json()
        got["t"] = time.perf_counter() - t
    th = threading.Thread(target=poll, daemon=True)
    th.start()
    time.sleep(0.4)
    t_sub = time.perf_counter()
    job_id = c.post("/api/v1/jobs", json={"type": "llm", "params": {"prompt": "p"}}).json()["job_id"]
    th.join(10)
    assert got["a"] and got["a"]["job_id"] == job_id
    assert got["t"] < 2.0                                  # not the 10 s wait
    assert time.perf_counter() - t_sub < 1.0


def test_next_jobs_claims_a_burst_in_one_request(client):
    """GET next-jobs?max=N claims up to N queued jobs (bounded by the worker's free job slots) in
    one transaction; each job goes to exactly one claimer; [] when the queue is empty."""
    c = client
    wid, hdr, _ = _register(c)
    c.put(f"/api/v1/workers/{wid}/config", json={"max_concurrent_jobs": 6}, headers=hdr)
    ids = [c.post("/api/v1/jobs", json={"type": "llm", "params": {"prompt": str(i)}}).json()["job_id"]
           for i in range(7)]
    a = c.get(f"/api/v1/workers/{wid}/next-jobs?max=3", headers=hdr).json()
    assert len(a) == 3 and len({x["job_id"] for x in a}) == 3
    b = c.get(f"/api/v1/workers/{wid}/next-jobs?max=8", headers=hdr).json()
    assert len(b) == 3                                        # 6 job slots: 3 + 3, two stay queued
    assert len({x["job_id"] for x in a} | {x["job_id"] for x in b}) == 6
    assert c.get(f"/api/v1/workers/{wid}/next-jobs?max=8", headers=hdr).json() == []
    wid2, hdr2, _ = _register(c)
    c.put(f"/api/v1/workers/{wid2}/config", json={"max_concurrent_jobs": 8}, headers=hdr2)
    rest = c.get(f"/api/v1/workers/{wid2}/next-jobs?max=8", headers=hdr2).json()
    assert {x["job_id"] for x in a + b + rest} == set(ids) and len(rest) == 1
    for x in a + b:
        assert c.get(f"/api/v1/jobs/{x['job_id']}").json()["status"] == "running"
    t0 = time.perf_counter()
    assert c.get(f"/api/v1/workers/{wid2}/next-jobs?max=2&wait=0.2", headers=hdr2).json() == []
    assert time.perf_counter() - t0 >= 0.2


def test_job_signal_wakes_waiters_across_threads():
    from app.services.job_signal import JobSignal
    sig = JobSignal()

    async def main():
        assert await sig.wait(0.05) is False                  # timeout
        loop = asyncio.get_running_loop()
        loop.call_later(0.05, sig.notify)                     # same loop
        assert await sig.wait(5.0) is True
        threading.Timer(0.05, sig.notify).start()             # another thread
        t = time.perf_counter()
        assert await sig.wait(5.0) is True
        assert time.perf_counter() - t < 2.0
    asyncio.run(main())
    sig.notify()                                              # no waiter: a no-op


def test_api_no_worker_503_and_direct(client):
    c = client
    r = c.post("/api/v1/jobs/sync?wait_for_worker=false", json={"type": "llm", "params": {}})
    assert r.status_code == 503
    assert c.get("/api/v1/jobs/direct/nearest?job_type=llm").status_code == 503
    wid, hdr, _ = _register(c, supports_direct=True, direct_url="http://10.0.0.5:8001")
    d = c.get("/api/v1/jobs/direct/nearest?job_type=llm").json()
    assert d["worker_id"] == wid and d["direct_url"].endswith(":8001")


def test_api_pd_job_path_places_decode_by_scheduler(client):
    """The cluster P/D path (reference pd_scheduler API, wired by services/pd_runtime):
    a ``pd`` job is pulled by a prefill worker, its completion hands it to the
    scheduler's decode placement, it is requeued pinned to the chosen decode
    worker (with the KV source), only that worker can pull it, and the stats
    endpoint reports the whole lifecycle."""
    c = client
    pre, hp, _ = _register(c, role="prefill", capabilities={"compute_flops": 2500.0})
    dec1, hd1, _ = _register(c, role="decode", capabilities={"memory_bandwidth_gbps": 8000.0})
    dec2, hd2, _ = _register(c, role="decode", capabilities={"memory_bandwidth_gbps": 2000.0})
    # dec2 reports a nearly full KV cache: the scheduler must prefer dec1
    c.post(f"/api/v1/workers/{dec2}/heartbeat", json={"status": "online",
                                                       "engine_stats": {"num_blocks": 100, "used_blocks": 95}},
           headers=hd2)
    st0 = c.get("/api/v1/admin/pd/stats").json()
    job_id = c.post("/api/v1/jobs", json={"type": "llm", "params": {"prompt": "hello", "max_tokens": 8,
                                                                     "pd": True}}).json()["job_id"]
    assert c.get("/api/v1/admin/pd/stats").json()["prefill_queue_size"] == st0["prefill_queue_size"] + 1
    # decode workers do not take the prefill phase; the prefill worker does
    assert c.get(f"/api/v1/workers/{dec1}/next-job", headers=hd1).json() is None
    a = c.get(f"/api/v1/workers/{pre}/next-job", headers=hp).json()
    assert a["job_id"] == job_id
    r = c.post(f"/api/v1/workers/{pre}/jobs/{job_id}/complete",
               json={"success": True, "result": {"response": "W", "first_token": "W", "kv_cache_key": "kv-1",
                                                 "kv_url": "http://10.0.0.9:8080/kv/kv-1"},
                     "processing_time_ms": 12}, headers=hp).json()
    assert r["next_phase"] == "decode" and r["decode_worker"] == dec1
    assert c.get(f"/api/v1/jobs/{job_id}").json()["status"] == "queued"
    # pinned: the other decode worker cannot take it
    assert c.get(f"/api/v1/workers/{dec2}/next-job", headers=hd2).json() is None
    b = c.get(f"/api/v1/workers/{dec1}/next-job", headers=hd1).json()
    assert b["job_id"] == job_id and b["params"]["pd_phase"] == "decode" and b["params"]["kv_source"] == pre
    assert b["params"]["kv_url"] == "http://10.0.0.9:8080/kv/kv-1"      # where the decode worker pulls the KV
    c.post(f"/api/v1/workers/{dec1}/jobs/{job_id}/complete",
           json={"success": True, "result": {"response": "World", "usage": {"completion_tokens": 8}},
                 "processing_time_ms": 30}, headers=hd1)
    assert c.get(f"/api/v1/jobs/{job_id}").json()["status"] == "completed"
    st = c.get("/api/v1/admin/pd/stats").json()
    assert st["transitions"] == st0["transitions"] + 1 and st["decode_completed"] == st0["decode_completed"] + 1
    assert st["migrations"] == st0["migrations"] + 1
    assert st["prefill_workers"] >= 1 and st["decode_workers"] >= 2


def test_worker_daemon_runs_pd_phases():
    from worker.main import Worker as Daemon
    d = Daemon.__new__(Daemon)
    d.worker_id = "w1"
    calls = []

    def fake(job_type, params, job_id="direct"):
        calls.append(dict(params))
        return {"response": "tok" if params.get("max_tokens") == 1 else "full text", "usage": {}}
    d._execute = fake
    out = d.execute("llm", {"prompt": "x", "max_tokens": 16, "pd": True}, "j1")
    assert out["phase"] == "prefill" and out["kv_cache_key"] == "w1:j1" and calls[-1]["max_tokens"] == 1
    out = d.execute("llm", {"prompt": "x", "max_tokens": 16, "pd": True, "pd_phase": "decode", "kv_source": "p"},
                    "j1")
    assert out["phase"] == "decode" and out["response"] == "full text" and calls[-1]["max_tokens"] == 16


# ----------------------------------------------------------------- admin console
def _spa_calls():
    """(method, path template) of every admin API call in the SPA's script."""
    import re
    s = (ROOT / "server/static/admin/index.html").read_text()
    calls = [("GET", m) for m in re.findall(r'get\(\s*[`"](/[^`"?]*)', s)]
    calls += re.findall(r'call\("(GET|POST|PUT|DELETE)",\s*[`"](/[^`"?]*)', s)
    norm = (lambda p: re.sub(r"\$\{[^}]*\}", "{x}", p) + ("{x}" if p.endswith("/") else ""))
    return s, sorted(set((m, norm(p)) for m, p in calls))


def test_admin_console_is_served_and_calls_only_real_routes(client):
    import re
    s, calls = _spa_calls()
    r = client.get("/admin")
    assert r.status_code == 200 and "MI355X Inference" in r.text
    assert "cdn" not in s.lower() and "<script src" not in s          # self-contained, works offline
    spec = client.get("/openapi.json").json()["paths"]
    routes = [(m.upper(), path) for path, ops in spec.items() for m in ops if path.startswith("/api/v1/admin")]
    assert routes

    def known(method, path):
        for m, tpl in routes:
            rx = "^" + re.sub(r"\{[^}]+\}", "[^/]+", tpl) + "$"
            if m == method and re.match(rx, "/api/v1/admin" + path.replace("{x}", "X")):
                return True
        return False
    missing = [c for c in calls if not known(*c)]
    assert not missing, missing
    # the console covers every admin area: privacy, enterprises + keys, worker config, bills, usage, P/D
    paths = {p for _, p in calls}
    for need in ("/enterprises/{x}/privacy", "/enterprises/{x}/privacy/compliance",
                 "/enterprises/{x}/privacy/retention-status", "/enterprises/{x}/privacy/cleanup",
                 "/enterprises/{x}/privacy/export", "/enterprises/{x}/privacy/data", "/privacy/scheduled-cleanup",
                 "/enterprises", "/enterprises/{x}/api-keys", "/workers/{x}/config", "/workers/{x}/usage",
                 "/bills", "/bills/{x}", "/usage/records", "/pd/stats", "/health/detailed", "/dashboard/realtime"):
        assert any(p == need or p.startswith(need) for p in paths), need
    assert ("PUT", "/workers/{x}/config") in calls and ("DELETE", "/enterprises/{x}/privacy/data") in calls


def test_admin_console_script_parses_and_reads_real_fields(client):
    import re
    import shutil
    import subprocess
    s, _ = _spa_calls()
    js = re.search(r"<script>(.*)</script>", s, re.S).group(1)
    if shutil.which("node"):
        p = ROOT / "server/static/admin/.check.js"
        try:
            p.write_text(js)
            out = subprocess.run(["node", "--check", str(p)], capture_output=True, text=True)
            assert out.returncode == 0, out.stderr
        finally:
            p.unlink(missing_ok=True)
    # the response fields the dashboard / worker / usage pages read
    c = client
    wid, hdr, _ = _register(c)
    d = c.get("/api/v1/admin/dashboard").json()
    assert {"online", "total"} <= set(d["workers"]) and {"jobs", "revenue", "gpu_hours"} <= set(d["today"])
    rt = c.get("/api/v1/admin/dashboard/realtime").json()
    assert {"busy", "details"} <= set(rt["workers"]) and {"running", "queued", "details"} <= set(rt["jobs"])
    w = c.get(f"/api/v1/admin/workers/{wid}").json()
    assert "load_control" in w["config"] and "version" in w["config"]
    assert c.put(f"/api/v1/admin/workers/{wid}/config", json={"load_control": {"max_concurrent_jobs": 64}}
                 ).json()["status"] == "ok"
    assert c.get(f"/api/v1/admin/workers/{wid}").json()["config"]["load_control"]["max_concurrent_jobs"] == 64
    u = c.get(f"/api/v1/admin/workers/{wid}/usage?days=30").json()
    assert {"total_cost", "total_gpu_seconds"} <= set(u)
    su = c.get("/api/v1/admin/usage/summary?group_by=day").json()
    assert {"count", "cost", "gpu_hours"} <= set(su["totals"])
    pd = c.get("/api/v1/admin/pd/stats").json()
    assert {"prefill_queue_size", "decode_queue_size", "transitions", "migrations"} <= set(pd)
    ent = c.post("/api/v1/admin/enterprises", json={"name": "Acme", "code": "acme"}).json()
    c.post(f"/api/v1/admin/enterprises/{ent['id']}/api-keys", json={"name": "k"})
    keys = c.get(f"/api/v1/admin/enterprises/{ent['id']}/api-keys").json()
    assert isinstance(keys, list) and {"name", "key_prefix", "total_requests"} <= set(keys[0])
    h = c.get("/api/v1/admin/health/detailed").json()
    assert {"status", "database", "stale_workers", "stuck_jobs", "issues"} <= set(h)
