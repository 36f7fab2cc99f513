"""Worker v2.0 config sections and their wiring.

The reference README documents ``inference`` / ``distributed`` /
``speculative`` / ``observability`` sections (README.md:815-910) that its
``WorkerConfig`` never parses.  Here they are typed, merged
with the ``DGI_*`` runtime env knobs, and feed the engines, the job-level
batcher and the worker's metrics / tracing.
"""
import threading
import time

import pytest
import yaml


def _yaml(tmp_path, data):
    p = tmp_path / "config.yaml"
    p.write_text(yaml.safe_dump(data), encoding="utf-8")
    return str(p)


def test_sections_parse_and_reach_llm_engine_config(tmp_path, monkeypatch):
    from config import load_config
    monkeypatch.delenv("GPU_LLM_MODEL", raising=False)
    monkeypatch.setenv("DGI_MAX_NUM_SEQS", "384")
    monkeypatch.setenv("DGI_CPU_TIER_GB", "64")
    monkeypatch.setenv("DGI_GRAPH_BATCH_BUCKETS", "1,8,64")
    cfg = load_config(_yaml(tmp_path, {
        "inference": {"engine": "llm_native", "batch": {"max_batch_size": 16, "max_wait_ms": 20},
                      "sglang": {"mem_fraction_static": 0.8}},
        "distributed": {"enabled": True, "role": "decode",
                        "model_shard": {"model_id": "llama3-70b", "start_layer": 40, "end_layer": 80},
                        "kv_cache": {"cpu_cache_size_gb": 32}},
        "speculative": {"enabled": True, "tree_width": 2, "tree_depth": 4},
        "observability": {"metrics": {"port": 9191}, "tracing": {"enabled": True, "exporter": "console"}},
    }))
    assert cfg.inference.batch.max_batch_size == 16 and cfg.inference.batch.max_wait_ms == 20
    assert cfg.distributed.model_shard.start_layer == 40 and cfg.distributed.kv_cache.cpu_cache_size_gb == 32
    assert cfg.observability.metrics.port == 9191 and cfg.observability.tracing.exporter == "console"
    e = cfg.engine_config("llm")
    assert e["backend"] == "mi355x"
    assert e["native"]["max_num_seqs"] == 384 and e["native"]["host_kv_gb"] == 64.0
    assert e["native"]["graph_batch_buckets"] == [1, 8, 64]
    assert e["speculative"]["depth"] == 4 and e["speculative"]["width"] == 2
    assert e["sglang"]["mem_fraction_static"] == 0.8
    assert e["distributed"]["role"] == "decode"


def test_engine_section_does_not_override_explicit_backend(tmp_path, monkeypatch):
    from config import load_config
    monkeypatch.delenv("GPU_LLM_BACKEND", raising=False)
    cfg = load_config(_yaml(tmp_path, {"inference": {"engine": "llm_vllm"},
                                       "engines": {"llm": {"backend": "sglang"}}}))
    assert cfg.engine_config("llm")["backend"] == "sglang"
    cfg = load_config(_yaml(tmp_path, {"inference": {"engine": "llm_vllm"}}))
    assert cfg.engine_config("llm")["backend"] == "vllm"


@pytest.mark.parametrize("pd,pp,layout,prefill", [("6:2", 2, "pdpp", 6), ("3:1", 1, "pd", 3), (None, 4, "pp", None)])
def test_dgi_layout_knobs(monkeypatch, pd, pp, layout, prefill):
    from config import WorkerConfig
    if pd:
        monkeypatch.setenv("DGI_PD", pd)
    else:
        monkeypatch.delenv("DGI_PD", raising=False)
    monkeypatch.setenv("DGI_PP", str(pp))
    monkeypatch.setenv("GPU_LAYOUT", "auto")
    c = WorkerConfig().engine_config("llm")
    assert c["layout"] in (layout, "auto")
    if prefill:
        assert c["prefill_ranks"] == prefill


def test_native_engine_receives_runtime_knobs():
    from engines.llm_native import NativeLLMEngine
    e = NativeLLMEngine({"model_id": "llama-tiny", "device": "cpu", "max_model_len": 256,
                         "native": {"block_size": 16, "graph_batch_buckets": [1, 2], "host_kv_gb": 0.0,
                                    "max_num_seqs": 4, "max_num_batched_tokens": 128}})
    e.load_model()
    try:
        assert e.engine.cfg.max_num_seqs == 4 and e.engine.cfg.graph_buckets == (1, 2)
        assert e.engine.cfg.max_num_batched_tokens == 128
    finally:
        e.unload_model()


class _BatchEngine:
    """An HF-style engine that only batches whole requests."""

    def __init__(self):
        self.calls = []

    async def batch_inference_async(self, params_list):
        self.calls.append(len(params_list))
        return [{"response": p["prompt"].upper(), "usage": {"completion_tokens": 1}} for p in params_list]

    def inference(self, params):  # pragma: no cover - must not be used when batching
        raise AssertionError("per-request path used")


def test_worker_routes_batchable_engines_through_job_batcher():
    from config import WorkerConfig
    from main import Worker
    cfg = WorkerConfig(supported_types=["llm"])
    cfg.inference.batch.max_batch_size = 8
    cfg.inference.batch.max_wait_ms = 30
    w = Worker(cfg, config_path="/tmp/unused-worker.yaml")
    eng = _BatchEngine()
    w.engines["llm"] = eng
    w._maybe_batcher("llm", eng)
    assert "llm" in w._batchers
    outs = [None] * 6

    def one(i):
        outs[i] = w.execute("llm", {"prompt": f"p{i}"}, job_id=f"j{i}")
    ts = [threading.Thread(target=one, args=(i,)) for i in range(6)]
    [t.start() for t in ts]
    [t.join(timeout=10) for t in ts]
    assert [o["response"] for o in outs] == [f"P{i}" for i in range(6)]
    assert max(eng.calls) > 1                      # requests were grouped
    if w.metrics is not None:
        assert w.metrics.get_summary()["total_requests"] == 6
    for b in w._batchers.values():
        b.close()


def test_native_engines_bypass_job_batcher():
    from config import WorkerConfig
    from engines.llm_native import NativeLLMEngine
    from main import Worker
    w = Worker(WorkerConfig(supported_types=["llm"]), config_path="/tmp/unused-worker.yaml")
    w._maybe_batcher("llm", NativeLLMEngine({"model_id": "llama-tiny"}))
    assert w._batchers == {}


def test_direct_server_mounts_metrics_routes():
    from fastapi.testclient import TestClient
    from config import WorkerConfig
    from direct_server import DirectServer
    from main import Worker
    w = Worker(WorkerConfig(supported_types=["llm"]), config_path="/tmp/unused-worker.yaml")
    ds = DirectServer(w, "127.0.0.1", 0)
    c = TestClient(ds.app)
    assert c.get("/metrics").status_code == 200
    assert c.get("/ready").json()["status"] == "not_ready"   # no engine loaded yet
    w.engines["llm"] = object()
    assert c.get("/ready").json()["status"] == "ready"
    time.sleep(0)


@pytest.mark.parametrize("name,layout,backend,prefill", [
    ("config.example.yaml", "pdpp", "mi355x", 5),
    ("config.8gb.yaml", "single", "mi355x", None),
    ("config.2gb.yaml", "single", "native", None),
])
def test_shipped_example_configs_load(monkeypatch, name, layout, backend, prefill):
    """The example configs shipped next to the worker (reference worker/config*.yaml) parse and wire up."""
    import os
    from worker.config import load_config
    for k in list(os.environ):
        if k.startswith(("GPU_", "DGI_")):
            monkeypatch.delenv(k, raising=False)
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "worker")
    cfg = load_config(os.path.join(root, name))
    llm = cfg.engine_config("llm")
    assert llm["layout"] == layout
    assert llm["backend"] == backend
    assert llm.get("prefill_ranks") == prefill
