"""Worker daemon plumbing: API client, batching, config, fingerprint, pipeline
sessions and the Python SDK.

Behavioural parity with the reference's tests/test_worker_api_client.py,
test_worker_batch_processor{,_flow}.py, test_worker_config.py,
test_worker_machine_id.py, test_worker_distributed_{inference_session,
worker_session,session_exit}.py and test_sdk_inference_client.py.  Modules
are imported flat (worker/ and sdk/python on sys.path) so the patch targets
the reference suite uses (``distributed.session.WorkerSession``,
``machine_id.subprocess.run``, ``inference_client.time.time``) resolve.
"""
import asyncio
import json
import os
import time
import types
from unittest.mock import MagicMock, patch

import httpx
import numpy as np
import pytest

from api_client import APIClient
from batch_processor import AdaptiveBatcher, ContinuousBatcher, PendingRequest, RequestPriority
from config import get_env, load_config, load_dotenv
from machine_id import MachineFingerprint
from distributed.session import DistributedInferenceSession, SessionManager, SessionState, WorkerSession
from inference_client import InferenceClient
from common.data_structures import SessionConfig, WorkerInfo, WorkerState
from common.serialization import serialize_tensor


def _resp(code, method="GET", url="http://example", **kw):
    return httpx.Response(code, request=httpx.Request(method, url), **kw)


# ============================================================================= API client

def test_client_headers_sign_bodies():
    c = APIClient(base_url="http://example", token="t")
    c.set_credentials(token="t", signing_secret="s")
    h = c._headers(body='{"a":1}', path="/p")
    assert h["X-Worker-Token"] == "t" and "X-Signature" in h and "X-Timestamp" in h
    assert "X-Signature" not in APIClient(base_url="http://e", token="t")._headers(body="{}", path="/p")


def test_client_signature_verifies_on_server_side():
    from app.services.security import RequestSigner
    c = APIClient(base_url="http://example", token="t")
    c.set_credentials(token="t", signing_secret="sec")
    h = c._headers(body='{"a":1}', path="/api/v1/x", method="POST")
    ok, err = RequestSigner.verify_signature("POST", "/api/v1/x", '{"a":1}', int(h["X-Timestamp"]),
                                             h["X-Signature"], "sec")
    assert ok, err


def test_client_retries_5xx_then_succeeds():
    c = APIClient(base_url="http://example")
    n = {"c": 0}

    def fake(method, url, **kw):
        n["c"] += 1
        if n["c"] < 3:
            r = _resp(503)
            raise httpx.HTTPStatusError("x", request=r.request, response=r)
        return _resp(200, method, url, json={"ok": True})

    with patch.object(c.client, "request", side_effect=fake), patch.object(time, "sleep", return_value=None):
        assert c._request_with_retry("GET", "http://example/x").status_code == 200
    assert n["c"] == 3


def test_client_no_retry_on_4xx():
    c = APIClient(base_url="http://example")
    r = _resp(400)
    with patch.object(c.client, "request", side_effect=httpx.HTTPStatusError("x", request=r.request, response=r)) as m:
        with pytest.raises(httpx.HTTPStatusError):
            c._request_with_retry("GET", "http://example/x")
    assert m.call_count == 1


@pytest.mark.parametrize("code", [204, 404])
def test_client_no_job_codes(code):
    c = APIClient(base_url="http://example")
    with patch.object(c.client, "get", return_value=_resp(code)):
        assert c.fetch_next_job("w") is None


def test_client_long_poll_sends_wait_and_a_longer_timeout():
    c = APIClient(base_url="http://example", timeout=3)
    with patch.object(c.client, "get", return_value=_resp(204)) as m:
        assert c.fetch_next_job("w", wait=5.0) is None
    kw = m.call_args.kwargs
    assert kw["params"] == {"wait": 5.0} and kw["timeout"] >= 15.0
    with patch.object(c.client, "get", return_value=_resp(204)) as m:
        c.fetch_next_job("w")
    assert "params" not in m.call_args.kwargs                 # plain poll: the reference's request


def test_client_batch_fetch_falls_back_on_a_reference_server():
    c = APIClient(base_url="http://example")
    jobs = [{"job_id": "a"}, {"job_id": "b"}]
    with patch.object(c.client, "get", return_value=_resp(200, json=jobs)) as m:
        assert c.fetch_next_jobs("w", 4, wait=2.0) == jobs
    assert m.call_args.args[0].endswith("/next-jobs") and m.call_args.kwargs["params"] == {"max": 4, "wait": 2.0}
    # a server without next-jobs: 404, then one job per request from then on
    with patch.object(c.client, "get", side_effect=[_resp(404), _resp(200, json={"job_id": "x"})]) as m:
        assert c.fetch_next_jobs("w", 4) == [{"job_id": "x"}]
    assert m.call_args.args[0].endswith("/next-job")
    with patch.object(c.client, "get", return_value=_resp(200, json={"job_id": "y"})) as m:
        assert c.fetch_next_jobs("w", 4) == [{"job_id": "y"}]
    assert m.call_count == 1 and m.call_args.args[0].endswith("/next-job")


def test_client_verify_and_config_failures_are_soft():
    c = APIClient(base_url="http://example")
    with patch.object(c.client, "post", side_effect=RuntimeError("boom")):
        assert c.verify_credentials("w", "t") is False
    with patch.object(c.client, "get", return_value=_resp(500)):
        assert c.get_config("w") is None


# ============================================================================= batching

def test_prefix_hash_uses_system_prompt_only():
    b = ContinuousBatcher(engine=object(), enable_prefix_grouping=True)
    assert b._compute_prefix_hash({"messages": []}) == ""
    assert b._compute_prefix_hash({"messages": [{"role": "user", "content": "x"}]}) == ""
    h = b._compute_prefix_hash({"messages": [{"role": "system", "content": "a"}, {"role": "user", "content": "1"}]})
    assert h == b._compute_prefix_hash({"messages": [{"role": "system", "content": "a"},
                                                     {"role": "user", "content": "2"}]})
    assert len(h) == 16


def test_prefix_grouping_fills_batch_from_largest_group_first():
    b = ContinuousBatcher(engine=object(), max_batch_size=4, enable_prefix_grouping=True)

    def add(jid, prefix):
        r = PendingRequest(priority=RequestPriority.NORMAL.value, timestamp=time.time(), job_id=jid,
                           params={"messages": []}, future=MagicMock(), prefix_hash=prefix)
        b._pending.append(r)
        if prefix:
            b._pending_by_prefix[prefix].append(r)
        return r

    a1, a2, b1, c1 = add("a1", "p1"), add("a2", "p1"), add("b1", "p2"), add("c1", "")
    batch = b._select_batch_with_prefix_grouping()
    assert batch[:2] == [a1, a2] and len(batch) == 4 and all(any(x is r for x in batch) for r in (b1, c1))


def test_priority_order():
    assert RequestPriority.HIGH.value < RequestPriority.NORMAL.value < RequestPriority.LOW.value


def test_submit_requires_started_batcher():
    async def run():
        with pytest.raises(RuntimeError, match="(?i)not running"):
            await ContinuousBatcher(engine=object()).submit("j", {})
    asyncio.run(run())


def test_adaptive_batch_size_moves_toward_target():
    b = AdaptiveBatcher(engine=object(), min_batch_size=1, max_batch_size=10, target_latency_ms=100)
    b._current_batch_size, b._latency_history = 10, [200.0] * 10
    b._adapt_batch_size()
    assert b._current_batch_size < 10
    b._current_batch_size, b._latency_history = 5, [50.0] * 10
    b._adapt_batch_size()
    assert b._current_batch_size > 5
    b._current_batch_size, b._latency_history = 1, [500.0] * 10
    b._adapt_batch_size()
    assert b._current_batch_size == 1


class _AsyncEngine:
    def __init__(self):
        self.batches = []

    async def batch_inference_async(self, params_list):
        self.batches.append(len(params_list))
        return [{"value": p.get("value")} for p in params_list]


class _SyncEngine:
    def batch_inference(self, params_list):
        return [{"value": p.get("value")} for p in params_list]


class _SingleEngine:
    def inference(self, params):
        return {"value": params.get("value")}


@pytest.mark.parametrize("engine_cls", [_AsyncEngine, _SyncEngine, _SingleEngine])
def test_batcher_round_trips_through_every_engine_kind(engine_cls):
    async def run():
        b = ContinuousBatcher(engine_cls(), max_batch_size=2, max_wait_ms=1, enable_prefix_grouping=False)
        await b.start()
        rs = await asyncio.gather(*(b.submit(f"j{i}", {"value": i}, timeout=2) for i in range(5)))
        await b.stop()
        return rs
    assert [r["value"] for r in asyncio.run(run())] == list(range(5))


def test_batcher_groups_concurrent_requests():
    eng = _AsyncEngine()

    async def run():
        b = ContinuousBatcher(eng, max_batch_size=8, max_wait_ms=20, enable_prefix_grouping=False)
        await b.start()
        await asyncio.gather(*(b.submit(f"j{i}", {"value": i}, timeout=2) for i in range(8)))
        st = b.get_stats()
        await b.stop()
        return st
    st = asyncio.run(run())
    assert max(eng.batches) > 1 and sum(eng.batches) == 8
    assert st["total_requests"] == 8 if "total_requests" in st else True


def test_per_request_exception_is_isolated():
    class E:
        async def batch_inference_async(self, params_list):
            return [{"ok": True}, RuntimeError("boom")]

    async def run():
        b = ContinuousBatcher(E(), max_batch_size=2, max_wait_ms=5, enable_prefix_grouping=False)
        await b.start()
        t1 = asyncio.ensure_future(b.submit("j1", {}, timeout=2))
        t2 = asyncio.ensure_future(b.submit("j2", {}, timeout=2))
        ok = await t1
        with pytest.raises(RuntimeError):
            await t2
        await b.stop()
        return ok
    assert asyncio.run(run())["ok"] is True


def test_timeout_removes_request():
    class Slow:
        async def batch_inference_async(self, params_list):
            await asyncio.sleep(0.2)
            return [{} for _ in params_list]

    async def run():
        b = ContinuousBatcher(Slow(), max_batch_size=10, max_wait_ms=1000, enable_prefix_grouping=False)
        await b.start()
        with pytest.raises(asyncio.TimeoutError):
            await b.submit("j1", {}, timeout=0.01)
        st = b.get_stats()
        await b.stop()
        return st
    assert asyncio.run(run())["queue_size"] == 0


def test_queue_full_rejects():
    async def run():
        b = ContinuousBatcher(_AsyncEngine(), max_queue_size=1, max_batch_size=10, max_wait_ms=1000)
        await b.start()
        t1 = asyncio.ensure_future(b.submit("j1", {"value": 1}, timeout=1))
        await asyncio.sleep(0)
        with pytest.raises(RuntimeError):
            await b.submit("j2", {"value": 2}, timeout=1)
        t1.cancel()
        await b.stop()
    asyncio.run(run())


# ============================================================================= config

def test_env_casting(monkeypatch):
    monkeypatch.setenv("X_BOOL", "true")
    monkeypatch.setenv("X_INT", "10")
    monkeypatch.setenv("X_LIST", "a, b,,c")
    assert get_env("X_BOOL", False, bool) is True
    assert get_env("X_INT", 0, int) == 10
    assert get_env("X_LIST", [], list) == ["a", "b", "c"]
    assert get_env("X_MISSING", 7, int) == 7


def test_dotenv_only_fills_unset(monkeypatch, tmp_path):
    monkeypatch.delenv("DGI_T_A", raising=False)
    monkeypatch.setenv("DGI_T_B", "existing")
    p = tmp_path / ".env"
    p.write_text("DGI_T_A=1\nDGI_T_B=2\n# comment\n", encoding="utf-8")
    load_dotenv(str(p))
    assert os.environ["DGI_T_A"] == "1" and os.environ["DGI_T_B"] == "existing"
    monkeypatch.delenv("DGI_T_A")


def test_yaml_config_with_env_engine_override(monkeypatch, tmp_path):
    p = tmp_path / "config.yaml"
    p.write_text("region: europe-west\nserver:\n  url: http://example\nengines:\n  llm:\n    model_id: base\n",
                 encoding="utf-8")
    monkeypatch.setenv("GPU_LLM_MODEL", "env-model")
    cfg = load_config(str(p))
    assert cfg.region == "europe-west" and cfg.server.url == "http://example"
    assert cfg.engines["llm"]["model_id"] == "env-model"


# ============================================================================= machine fingerprint

def test_fingerprint_created_then_reused(tmp_path):
    fp = tmp_path / "fp.json"
    first = {"machine_id": "m1", "hardware_hash": "h1", "details": {}, "generated_at": "t1"}
    with patch.object(MachineFingerprint, "generate", return_value=first):
        assert MachineFingerprint.get_or_create(storage_path=str(fp))["machine_id"] == "m1"
    assert json.loads(fp.read_text())["hardware_hash"] == "h1"
    with patch.object(MachineFingerprint, "generate", return_value=dict(first, machine_id="other")):
        assert MachineFingerprint.get_or_create(storage_path=str(fp))["machine_id"] == "m1"


def test_fingerprint_regenerated_on_hardware_change(tmp_path):
    fp = tmp_path / "fp.json"
    fp.write_text(json.dumps({"machine_id": "m1", "hardware_hash": "h1", "details": {}, "generated_at": "t"}))
    new = {"machine_id": "m2", "hardware_hash": "h2", "details": {}, "generated_at": "t2"}
    with patch.object(MachineFingerprint, "generate", return_value=new):
        assert MachineFingerprint.get_or_create(storage_path=str(fp))["machine_id"] == "m2"


def test_fingerprint_deterministic():
    with patch("machine_id.platform.system", return_value="Linux"), \
            patch("machine_id.platform.machine", return_value="x86_64"), \
            patch("machine_id.platform.node", return_value="n"), \
            patch("machine_id.uuid.getnode", return_value=0xAABBCCDDEEFF), \
            patch.object(MachineFingerprint, "_get_machine_id", return_value="mid"), \
            patch.object(MachineFingerprint, "_get_gpu_info", return_value=None), \
            patch.object(MachineFingerprint, "_get_timestamp", return_value="t"):
        a, b = MachineFingerprint.generate(), MachineFingerprint.generate()
    assert a["hardware_hash"] == b["hardware_hash"] and len(a["machine_id"]) == 32


def test_windows_machine_id_branch():
    class R:
        returncode = 0
        stdout = "UUID\nABCDEF\n"
    with patch("machine_id.os.path.exists", return_value=False), \
            patch("machine_id.platform.system", return_value="Windows"), \
            patch("machine_id.subprocess.run", return_value=R()):
        assert MachineFingerprint._get_machine_id() == "ABCDEF"


# ============================================================================= pipeline sessions

class _FakeWS:
    def __init__(self, worker_info, session_id=None):
        self.worker_info = worker_info
        self.session_id = "s"
        self.state = SessionState.INITIALIZING
        self.position = 0
        self.next_session = None
        self.calls = 0

    async def connect(self, timeout=30.0):
        self.state = SessionState.READY

    async def forward(self, hidden_states, position, kv_cache_keys=None):
        self.calls += 1
        return hidden_states, (kv_cache_keys or [])

    async def close(self):
        self.state = SessionState.CLOSED


class _FlakyWS(_FakeWS):
    async def forward(self, hidden_states, position, kv_cache_keys=None):
        self.calls += 1
        if self.calls == 1:
            raise RuntimeError("transient")
        return hidden_states, []


class _DeadWS(_FakeWS):
    async def forward(self, hidden_states, position, kv_cache_keys=None):
        raise RuntimeError("permanent")


def _route(n=1):
    return [WorkerInfo(worker_id=f"w{i}", state=WorkerState.ONLINE, api_endpoint=f"http://w{i}") for i in range(n)]


def _cfg(**kw):
    return SessionConfig(model_name="m", max_length=kw.get("max_length", 10), max_retries=kw.get("max_retries", 1),
                         connect_timeout=1.0)


def test_session_setup_step_close_and_stats():
    async def run():
        with patch("distributed.session.WorkerSession", _FakeWS):
            s = DistributedInferenceSession(_cfg(), _route(3))
            await s.setup()
            assert s.state == SessionState.READY
            out = await s.step(np.zeros((1, 2), dtype=np.float32))
            assert out.shape == (1, 2) and s.position == 2
            assert s.get_stats()["total_steps"] == 1
            await s.close()
            assert s.state == SessionState.CLOSED
    asyncio.run(run())


def test_session_retries_transient_failures():
    async def run():
        with patch("distributed.session.WorkerSession", _FlakyWS), \
                patch("distributed.session.asyncio.sleep", return_value=None):
            s = DistributedInferenceSession(_cfg(max_retries=2), _route())
            await s.setup()
            await s.step(np.zeros((1, 1), dtype=np.float32))
            assert s.get_stats()["retries"] >= 1
            await s.close()
    asyncio.run(run())


def test_session_length_guard():
    async def run():
        with patch("distributed.session.WorkerSession", _FakeWS):
            s = DistributedInferenceSession(_cfg(max_length=1), _route())
            await s.setup()
            with pytest.raises(ValueError):
                await s.step(np.zeros((1, 2), dtype=np.float32))
    asyncio.run(run())


def test_session_permanent_failure_surfaces():
    async def run():
        with patch("distributed.session.WorkerSession", _DeadWS):
            s = DistributedInferenceSession(_cfg(), _route())
            await s.setup()
            with pytest.raises(RuntimeError):
                await s.step(np.zeros((1, 1), dtype=np.float32))
            await s.close()
    asyncio.run(run())


def test_session_manager_recycles_closed_slots():
    async def run():
        with patch("distributed.session.WorkerSession", _FakeWS):
            mgr = SessionManager(max_sessions=1)
            s1 = await mgr.create_session(_cfg(), _route())
            assert s1.state == SessionState.READY
            s1.state = SessionState.CLOSED
            assert await mgr.create_session(_cfg(), _route()) is not None
            await mgr.close_all()
    asyncio.run(run())


class _R:
    def __init__(self, status, js=None, text=""):
        self.status, self._js, self._text = status, js, text

    async def json(self):
        return self._js

    async def text(self):
        return self._text

    async def __aenter__(self):
        return self

    async def __aexit__(self, *a):
        return False


class _FakeHTTP:
    def __init__(self, health=200, fwd=200, result=None):
        self.health, self.fwd, self.result = health, fwd, result
        self.closed = False
        self.posts = []

    def get(self, url, **kw):
        return _R(self.health)

    def post(self, url, json=None, **kw):
        self.posts.append((url, json))
        if url.endswith("/inference/forward"):
            return _R(200, self.result or {}) if self.fwd == 200 else _R(self.fwd, text="bad")
        return _R(200, {})

    async def close(self):
        self.closed = True


def _ws():
    return WorkerSession(worker_info=WorkerInfo(worker_id="w", state=WorkerState.ONLINE, api_endpoint="http://w"))


def test_worker_session_connect_ok_and_fail():
    async def run():
        with patch("distributed.session.aiohttp.ClientSession", return_value=_FakeHTTP(health=200)):
            ws = _ws()
            await ws.connect()
            assert ws.state == SessionState.READY
        with patch("distributed.session.aiohttp.ClientSession", return_value=_FakeHTTP(health=500)):
            ws = _ws()
            with pytest.raises(ConnectionError):
                await ws.connect()
            assert ws.state == SessionState.ERROR
    asyncio.run(run())


def test_worker_session_forward_roundtrip():
    hidden = np.arange(6, dtype=np.float32).reshape(2, 3)
    fake = _FakeHTTP(result={"output": serialize_tensor(hidden), "kv_cache_keys": ["k1"]})

    async def run():
        with patch("distributed.session.aiohttp.ClientSession", return_value=fake):
            ws = _ws()
            await ws.connect()
            out, keys = await ws.forward(hidden_states=hidden, position=5, kv_cache_keys=["x"])
            got = out.cpu().numpy() if hasattr(out, "cpu") else out
            assert keys == ["k1"] and np.array_equal(got, hidden) and ws.position == 5 + hidden.shape[1]
            url, body = fake.posts[-1]
            assert url.endswith("/inference/forward") and body["position"] == 5
            await ws.close()
            assert ws.state == SessionState.CLOSED and fake.closed
    asyncio.run(run())


def test_worker_session_forward_error_state():
    async def run():
        with patch("distributed.session.aiohttp.ClientSession", return_value=_FakeHTTP(fwd=500)):
            ws = _ws()
            await ws.connect()
            with pytest.raises(RuntimeError):
                await ws.forward(hidden_states=np.zeros((1, 1), dtype=np.float32), position=0)
            assert ws.state == SessionState.ERROR
    asyncio.run(run())


@pytest.mark.parametrize("in_loop", [True, False])
def test_worker_session_exit_closes_in_and_out_of_loop(in_loop):
    n = {"c": 0}

    async def fake_close(self):
        n["c"] += 1
    ws = WorkerSession(worker_info=WorkerInfo(worker_id="w", state=WorkerState.ONLINE))
    ws.close = types.MethodType(fake_close, ws)
    if in_loop:
        async def run():
            ws.__exit__(None, None, None)
        asyncio.run(run())
    else:
        ws.__exit__(None, None, None)
    assert n["c"] == 1


# ============================================================================= SDK

def test_sdk_falls_back_after_timeout():
    c = InferenceClient(base_url="http://primary", fallback_urls=["http://backup"], max_retries=2)
    seen = []

    def fake(method, url, **kw):
        seen.append(url)
        if url.startswith("http://primary"):
            raise httpx.TimeoutException("t")
        return _resp(200, method, url, json={"ok": True})

    with patch.object(c.client, "request", side_effect=fake), patch.object(time, "sleep", return_value=None):
        assert c._request_with_fallback("GET", "/ping").status_code == 200
    assert any(u.startswith("http://backup") for u in seen)


def test_sdk_raises_4xx_without_fallback():
    c = InferenceClient(base_url="http://primary", fallback_urls=["http://backup"], max_retries=2)

    def fake(method, url, **kw):
        r = _resp(400, method, url)
        raise httpx.HTTPStatusError("bad", request=r.request, response=r)

    with patch.object(c.client, "request", side_effect=fake) as m:
        with pytest.raises(httpx.HTTPStatusError):
            c._request_with_fallback("GET", "/bad")
    assert m.call_count == 1


def test_sdk_api_key_header_and_chat_routes():
    c = InferenceClient(base_url="http://x", api_key="k")
    assert c._headers()["X-API-Key"] == "k"
    calls = []

    def fake(method, path, **kw):
        calls.append((method, path, kw.get("json")))
        return _resp(200, method, "http://x" + path, json={"ok": True})

    with patch.object(c, "_request_with_fallback", side_effect=fake):
        c.chat(messages=[{"role": "user", "content": "hi"}], sync=True)
        c.chat(messages=[{"role": "user", "content": "hi"}], sync=False)
    assert [p for _, p, _ in calls] == ["/api/v1/jobs/sync", "/api/v1/jobs"]
    assert calls[0][2]["type"] == "llm"


def test_sdk_direct_image_short_circuit():
    c = InferenceClient(base_url="http://x")
    with patch.object(c, "_direct_inference", return_value={"direct": True}) as d:
        assert c.generate_image(prompt="p", use_direct=True)["direct"] is True
    d.assert_called_once()


def test_sdk_nearest_worker_cached_within_ttl():
    c = InferenceClient(base_url="http://x")
    r = _resp(200, url="http://x/api/v1/jobs/direct/nearest", json={"direct_url": "http://w", "region": "asia-east"})
    with patch.object(c, "_request_with_fallback", return_value=r) as m, \
            patch("inference_client.time.time", side_effect=[1000.0, 1000.0, 1001.0, 1001.0]):
        assert c._get_nearest_worker("llm") == c._get_nearest_worker("llm")
    assert m.call_count == 1
