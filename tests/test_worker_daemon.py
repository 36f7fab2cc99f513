"""Worker daemon, API client, machine fingerprint, SDK, and an end-to-end run:
control plane (uvicorn thread) + worker daemon (dgi engine on CPU) + SDK client.

Unit tests mirror the reference's tests/test_worker_{api_client,config,machine_id}.py
and tests/test_sdk_inference_client.py.
"""
import json
import os
import socket
import threading
import time
from unittest.mock import patch

import httpx
import pytest


# ----------------------------------------------------------------- config
def test_get_env_casting(monkeypatch):
    from config import get_env
    monkeypatch.setenv("X_BOOL", "true")
    monkeypatch.setenv("X_INT", "10")
    monkeypatch.setenv("X_LIST", "a, b,,c")
    assert get_env("X_BOOL", False, bool) is True
    assert get_env("X_INT", 0, int) == 10
    assert get_env("X_LIST", [], list) == ["a", "b", "c"]
    assert get_env("X_MISSING", 5, int) == 5


def test_load_dotenv_and_yaml_with_env_override(monkeypatch, tmp_path):
    from config import load_config, load_dotenv
    env = tmp_path / ".env"
    env.write_text("DGI_T_A=1\nDGI_T_B=2\n", encoding="utf-8")
    monkeypatch.setenv("DGI_T_B", "existing")
    load_dotenv(str(env))
    assert os.environ["DGI_T_A"] == "1" and os.environ["DGI_T_B"] == "existing"
    monkeypatch.delenv("DGI_T_A")
    cfg = tmp_path / "config.yaml"
    cfg.write_text("region: europe-west\nserver:\n  url: http://example\nengines:\n  llm:\n    model_id: base\n",
                   encoding="utf-8")
    monkeypatch.setenv("GPU_LLM_MODEL", "env-model")
    c = load_config(str(cfg))
    assert c.region == "europe-west" and c.server.url == "http://example"
    assert c.engines["llm"]["model_id"] == "env-model"
    assert c.engine_config("llm")["backend"] == "mi355x"
    c.save(str(tmp_path / "out.yaml"))
    assert load_config(str(tmp_path / "out.yaml")).region == "europe-west"


# ----------------------------------------------------------------- machine id
def test_machine_fingerprint_reuse_and_regen(tmp_path):
    from machine_id import MachineFingerprint
    fp = tmp_path / "fp.json"
    first = {"machine_id": "m1", "hardware_hash": "h1", "details": {}, "generated_at": "t1"}
    with patch.object(MachineFingerprint, "generate", return_value=first):
        assert MachineFingerprint.get_or_create(str(fp))["machine_id"] == "m1"
        assert MachineFingerprint.get_or_create(str(fp))["machine_id"] == "m1"
    new = {"machine_id": "m2", "hardware_hash": "h2", "details": {}, "generated_at": "t2"}
    with patch.object(MachineFingerprint, "generate", return_value=new):
        assert MachineFingerprint.get_or_create(str(fp))["machine_id"] == "m2"


def test_machine_fingerprint_deterministic_and_windows_branch():
    from machine_id import MachineFingerprint
    with patch("machine_id.platform.node", return_value="n"), \
            patch("machine_id.uuid.getnode", return_value=0xAABBCCDDEEFF), \
            patch.object(MachineFingerprint, "_get_machine_id", return_value="mid"), \
            patch.object(MachineFingerprint, "_get_gpu_info", return_value=None), \
            patch.object(MachineFingerprint, "_get_timestamp", return_value="t"):
        a, b = MachineFingerprint.generate(), MachineFingerprint.generate()
    assert a["hardware_hash"] == b["hardware_hash"] and len(a["machine_id"]) == 32
    assert a["details"]["mac_address"] == "AA:BB:CC:DD:EE:FF"

    class _R:
        returncode = 0
        stdout = "UUID\nABCDEF\n"
    with patch("machine_id.os.path.exists", return_value=False), \
            patch("machine_id.platform.system", return_value="Windows"), \
            patch("machine_id.subprocess.run", return_value=_R()):
        assert MachineFingerprint._get_machine_id() == "ABCDEF"


# ----------------------------------------------------------------- api client
def _resp(code, **kw):
    return httpx.Response(code, request=httpx.Request("GET", "http://example"), **kw)


def test_api_client_signing_retry_and_errors():
    from api_client import APIClient
    c = APIClient("http://example", token="t")
    c.set_credentials("t", "s")
    h = c._headers(body='{"a":1}', path="/p")
    assert h["X-Worker-Token"] == "t" and "X-Signature" in h and "X-Timestamp" in h
    # server-side verification of the same signature scheme
    from app.services.security import RequestSigner
    ok, _ = RequestSigner.verify_signature("POST", "/p", {"a": 1}, int(h["X-Timestamp"]), h["X-Signature"], "s")
    assert ok
    n = {"i": 0}

    def flaky(method, url, **kw):
        n["i"] += 1
        if n["i"] < 3:
            r = _resp(503)
            raise httpx.HTTPStatusError("x", request=r.request, response=r)
        return _resp(200, json={"ok": True})
    with patch.object(c.client, "request", side_effect=flaky), patch("api_client.time.sleep"):
        assert c._request_with_retry("GET", "http://example/x").status_code == 200 and n["i"] == 3
    r400 = _resp(400)
    with patch.object(c.client, "request", side_effect=httpx.HTTPStatusError("x", request=r400.request,
                                                                             response=r400)):
        with pytest.raises(httpx.HTTPStatusError):
            c._request_with_retry("GET", "http://example/x")
    for code in (204, 404):
        with patch.object(c.client, "get", return_value=_resp(code)):
            assert c.fetch_next_job("w") is None
    with patch.object(c.client, "post", side_effect=RuntimeError("boom")):
        assert c.verify_credentials("w", "t") is False
    with patch.object(c.client, "get", return_value=_resp(500)):
        assert c.get_config("w") is None


# ----------------------------------------------------------------- SDK
def test_sdk_fallback_headers_endpoints_and_cache():
    from inference_client import InferenceClient
    c = InferenceClient("http://primary", fallback_urls=["http://backup"], max_retries=2, api_key="k")
    assert c._headers()["X-API-Key"] == "k"
    seen = []

    def req(method, url, **kw):
        seen.append(url)
        if url.startswith("http://primary"):
            raise httpx.TimeoutException("t")
        return httpx.Response(200, request=httpx.Request(method, url), json={"ok": True})
    with patch.object(c.client, "request", side_effect=req), patch("inference_client.time.sleep"):
        assert c._request_with_fallback("GET", "/ping").status_code == 200
    assert any(u.startswith("http://backup") for u in seen)
    calls = []

    def fake(method, path, **kw):
        calls.append(path)
        return httpx.Response(200, request=httpx.Request(method, "http://x" + path), json={"ok": True})
    with patch.object(c, "_request_with_fallback", side_effect=fake):
        c.chat([{"role": "user", "content": "hi"}], sync=True)
        c.chat([{"role": "user", "content": "hi"}], sync=False)
    assert calls == ["/api/v1/jobs/sync", "/api/v1/jobs"]
    with patch.object(c, "_direct_inference", return_value={"direct": True}) as d:
        assert c.generate_image("p", use_direct=True)["direct"] is True
        d.assert_called_once()
    resp = httpx.Response(200, request=httpx.Request("GET", "http://x"), json={"direct_url": "http://w"})
    with patch.object(c, "_request_with_fallback", return_value=resp) as rf:
        assert c._get_nearest_worker("llm") == c._get_nearest_worker("llm")
        assert rf.call_count == 1


# ----------------------------------------------------------------- end to end
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _wait_http(url, timeout=60):
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            if httpx.get(url, timeout=2).status_code == 200:
                return
        except httpx.HTTPError:
            time.sleep(0.2)
    raise TimeoutError(url)


def _e2e(tmp_path, engine_cfg: dict, name: str, n_sync: int = 4, max_tokens: int = 6):
    """Control plane (uvicorn thread, SQLite) + worker daemon (``llm_native``) + SDK: concurrent
    sync jobs, a direct call and an SSE stream.  Returns (sync outputs, direct output, stream
    pieces, worker list, the worker's NativeLLMEngine, timings)."""
    import uvicorn
    from app.db.database import Base, engine
    from app.main import app
    from config import WorkerConfig
    from inference_client import InferenceClient
    from main import Worker

    Base.metadata.drop_all(bind=engine)
    sport, dport = _free_port(), _free_port()
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=sport, log_level="warning"))
    st = threading.Thread(target=server.run, daemon=True)
    st.start()
    base = f"http://127.0.0.1:{sport}"
    _wait_http(base + "/health")

    cfg = WorkerConfig(name=name, region="asia-east", supported_types=["llm"], engines={"llm": engine_cfg},
                       heartbeat_interval=1, poll_interval=0.05)
    cfg.server.url = base
    cfg.direct.enabled, cfg.direct.host, cfg.direct.port = True, "127.0.0.1", dport
    cfg.direct.public_url = f"http://127.0.0.1:{dport}"
    cfg.load_control.max_concurrent_jobs = 8
    w = Worker(cfg, config_path=str(tmp_path / "worker.yaml"))
    timings = {}
    with patch("machine_id.Path.home", return_value=tmp_path):
        wt = threading.Thread(target=w.start, kwargs={"install_signals": False}, daemon=True)
        wt.start()
        try:
            t0 = time.time()
            while w.worker_id is None or not w.running:
                assert time.time() - t0 < 240, "worker did not start"
                time.sleep(0.1)
            _wait_http(f"http://127.0.0.1:{dport}/health")
            sdk = InferenceClient(base, timeout=120)
            msgs = [{"role": "user", "content": "hello mi355x"}]
            # several concurrent sync jobs batch inside the engine
            outs = [None] * n_sync

            def one(i):
                outs[i] = sdk.chat(msgs, max_tokens=max_tokens, temperature=0.0, sync=True, timeout=120)
            ts = [threading.Thread(target=one, args=(i,)) for i in range(n_sync)]
            t1 = time.time()
            [t.start() for t in ts]
            [t.join(180) for t in ts]
            timings["sync_batch_s"] = time.time() - t1
            t1 = time.time()
            d = sdk.chat(msgs, max_tokens=max_tokens, temperature=0.0, use_direct=True)
            timings["direct_s"] = time.time() - t1
            t1 = time.time()
            pieces = list(sdk.stream_chat(msgs, max_tokens=max_tokens, temperature=0.0))
            timings["stream_s"] = time.time() - t1
            info = sdk.list_workers()
            # the engine's state before shutdown unloads it
            ne = w.engines["llm"]
            inner = getattr(ne, "engine", None)
            g = getattr(getattr(inner, "runner", None), "graphs", None)
            timings["device"] = getattr(ne, "device", "")
            timings["graphs_captured"] = bool(g is not None and g.captured)
            return outs, d, pieces, info, ne, timings
        finally:
            w.request_shutdown(graceful=True)
            wt.join(60)
            server.should_exit = True
            st.join(30)
            assert not wt.is_alive()


def test_end_to_end_server_worker_sdk(tmp_path):
    outs, d, pieces, info, _eng, _t = _e2e(
        tmp_path, {"model_id": "llama-tiny", "backend": "mi355x", "max_num_seqs": 16,
                   "max_num_batched_tokens": 512, "max_model_len": 512}, "cpu-worker")
    for o in outs:
        assert o is not None and o["status"] == "completed", o
        assert o["result"]["usage"]["completion_tokens"] == 6
    assert len({o["result"]["response"] for o in outs}) == 1      # greedy: identical
    assert d["success"] and d["result"]["response"] == outs[0]["result"]["response"]
    assert len(pieces) >= 1
    assert info[0]["total_jobs"] == 4 and saved_yaml_has_token(tmp_path / "worker.yaml")


@pytest.mark.gpu
def test_end_to_end_served_path_on_gpu(tmp_path):
    """the reference's live path — SDK -> control plane -> worker
    daemon pull -> engine (reference worker/main.py:313-376) — with the ``llm_native`` engine
    on cuda:0 (hipGraph decode, warm-up, prefix cache).  Sync, direct and SSE jobs return the
    greedy continuation the in-process engine computes for the same prompt ids."""
    import torch
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.sched.request import SamplingParams
    from dgi.utils.tokenizer import chat_prompt_ids
    ecfg = {"model_id": "llama-tiny-hd128", "backend": "mi355x", "device": "cuda:0", "max_num_seqs": 16,
            "max_num_batched_tokens": 512, "max_model_len": 512, "warmup": True, "seed": 0}
    outs, d, pieces, info, eng, timings = _e2e(tmp_path, ecfg, "gpu-worker", n_sync=6, max_tokens=12)
    for o in outs:
        assert o is not None and o["status"] == "completed", o
    texts = {o["result"]["response"] for o in outs}
    assert len(texts) == 1 and d["success"] and d["result"]["response"] in texts
    assert "".join(pieces) in texts
    assert timings["device"].startswith("cuda") and timings["graphs_captured"], timings
    # the in-process engine on the same (seeded random-init) weights, same prompt ids
    ref = LLMEngine(EngineConfig(model="llama-tiny-hd128", device="cuda:0", max_num_seqs=16,
                                 max_num_batched_tokens=512, max_model_len=512, seed=0, use_graphs=False))
    ids = chat_prompt_ids(eng.tokenizer, [{"role": "user", "content": "hello mi355x"}])
    want = ref.generate([ids], SamplingParams(max_tokens=12, temperature=0.0))[0].output
    assert eng.tokenizer.decode(want, skip_special_tokens=True) in texts
    assert {o["result"]["usage"]["completion_tokens"] for o in outs} == {len(want)}
    torch.cuda.synchronize()
    assert info[0]["total_jobs"] == 6


def saved_yaml_has_token(path) -> bool:
    import yaml
    return bool((yaml.safe_load(open(path)) or {}).get("token"))
