"""Metrics, tracing and structured logging (server/app/services/observability.py).

Behavioural parity with the reference's tests/test_server_observability.py:
TracingManager (disabled spans, decorator), MetricsCollector counters and
summary, StructuredLogger context, the /metrics endpoint factory and route
mounting, and the with/without-Prometheus paths.  prometheus_client is
installed here, so the exported series are checked against the real
registry instead of a mock.
"""
import asyncio
import time
from unittest.mock import MagicMock, patch

import pytest

from server.app.services import observability as obs
from server.app.services.observability import (MetricsCollector, StructuredLogger, TracingManager,
                                                create_metrics_endpoint, setup_metrics_routes)

prom = pytest.importorskip("prometheus_client")


def _sample(name, **labels):
    return prom.REGISTRY.get_sample_value(name, labels) or 0.0


@pytest.fixture
def col():
    return MetricsCollector(worker_id=f"w-{time.monotonic_ns()}", model_name="m-test", worker_role="hybrid")


# ----------------------------------------------------------------------------- tracing

def test_tracer_defaults_and_disabled_span():
    t = TracingManager(service_name="svc")
    assert (t.service_name, t._tracer, t._enabled) == ("svc", None, False)
    with t.span("x") as sp:
        assert sp is None


def test_trace_decorator_keeps_coroutine_and_result():
    t = TracingManager()

    @t.trace_inference
    async def infer(x=1):
        return {"y": x + 1}

    assert asyncio.iscoroutinefunction(infer) and infer.__name__ == "infer"
    assert asyncio.run(infer(x=4)) == {"y": 5}


def test_span_with_fake_tracer_sets_attributes_and_error_status():
    t = TracingManager()
    span = MagicMock()
    span.__enter__ = MagicMock(return_value=span)
    span.__exit__ = MagicMock(return_value=None)
    t._tracer = MagicMock()
    t._tracer.start_as_current_span.return_value = span
    t._enabled = True
    with t.span("s", {"tokens": 3}) as sp:
        assert sp is span
    span.set_attribute.assert_called_with("tokens", 3)
    if obs.HAS_OTEL:
        with pytest.raises(ValueError):
            with t.span("bad"):
                raise ValueError("boom")
        assert span.set_status.called


def test_setup_without_otel_stays_disabled():
    with patch.object(obs, "HAS_OTEL", False):
        t = TracingManager("svc")
        assert t.setup() is False and not t._enabled


# ----------------------------------------------------------------------------- collector

def test_collector_initial_state(col):
    assert (col.model_name, col.worker_role) == ("m-test", "hybrid")
    assert (col._request_count, col._token_count, col._error_count) == (0, 0, 0)


def test_record_success_and_error(col):
    col.record_request(phase="prefill", latency_seconds=0.5, tokens=100, success=True)
    col.record_request(phase="decode", latency_seconds=1.0, tokens=0, success=False)
    assert (col._request_count, col._token_count, col._latency_sum, col._error_count) == (2, 100, 1.5, 1)


def test_record_many_counts_errors(col):
    for i in range(10):
        col.record_request("prefill", 0.1 * (i + 1), 10, success=i % 3 != 0)
    assert (col._request_count, col._token_count, col._error_count) == (10, 100, 4)


def test_prometheus_series_move(col):
    before = _sample("inference_requests_total", model="m-test", worker_id=col.worker_id, status="success")
    col.record_request("prefill", 0.02, 7, True)
    col.record_request("prefill", 0.02, 0, False)
    assert _sample("inference_requests_total", model="m-test", worker_id=col.worker_id, status="success") == before + 1
    assert _sample("inference_requests_total", model="m-test", worker_id=col.worker_id, status="error") == 1
    assert _sample("tokens_generated_total", model="m-test", worker_id=col.worker_id) == 7
    assert _sample("inference_latency_seconds_count", model="m-test", phase="prefill", worker_role="hybrid") >= 2


def test_batch_kv_gpu_spec_migration_series(col):
    n0 = _sample("batch_size_count", phase="decode")
    col.record_batch(phase="decode", batch_size=32)
    assert _sample("batch_size_count", phase="decode") == n0 + 1
    col.record_kv_cache_stats(level="gpu", hit_rate=0.85, size_bytes=100 << 20, evictions=10)
    assert _sample("kv_cache_hit_rate", level="gpu") == pytest.approx(0.85)
    assert _sample("kv_cache_evictions_total", level="gpu", worker_id=col.worker_id) == 10
    col.record_gpu_stats(gpu_id=0, memory_used=8 << 30, memory_total=288 << 30, utilization=75.5)
    assert _sample("gpu_memory_total_bytes", worker_id=col.worker_id, gpu_id="0") == float(288 << 30)
    col.record_speculative_stats(accept_rate=0.8, speedup=2.5)
    assert _sample("speculative_speedup", worker_id=col.worker_id) == 2.5
    col.record_migration("p0", "d0", 0.004)
    assert _sample("kv_migration_latency_seconds_count", source_worker="p0", target_worker="d0") >= 1
    col.record_queue("prefill", 5)
    assert _sample("queue_size", phase="prefill") == 5


def test_tokens_per_second_resets_window(col):
    col._token_count = 1000
    col._last_update = time.time() - 1.0
    col.update_tokens_per_second()
    assert col._token_count == 0 and 500 < col._tps <= 1000
    assert _sample("tokens_per_second", model="m-test", worker_id=col.worker_id) == pytest.approx(col._tps)


def test_summary_and_empty_summary(col):
    assert col.get_summary()["error_rate"] == 0.0 and col.get_summary()["avg_latency_ms"] == 0.0
    col.record_request("prefill", 0.1, 50, True)
    col.record_request("prefill", 0.2, 60, True)
    col.record_request("decode", 0.3, 70, False)
    s = col.get_summary()
    assert (s["worker_id"], s["model_name"], s["total_requests"], s["error_count"]) == \
        (col.worker_id, "m-test", 3, 1)
    assert s["error_rate"] == pytest.approx(1 / 3) and s["avg_latency_ms"] == pytest.approx(200.0)


def test_engine_stats_feed(col):
    col.record_engine_stats({"waiting": 3, "running": 40, "prefix_hit_rate": 0.5})
    assert _sample("queue_size", phase="decode") == 40
    col.record_engine_stats({})


def test_without_prometheus_nothing_breaks(col):
    with patch.object(obs, "HAS_PROMETHEUS", False):
        col.record_request("decode", 0.2, 20, True)
        col.record_batch("prefill", 8)
        col.record_kv_cache_stats("gpu", 0.9)
        col.record_gpu_stats(0, 1000, 2000, 50.0)
        col.record_speculative_stats(0.7, 1.5)
        col.update_tokens_per_second()
    assert col._request_count == 1


@pytest.mark.parametrize("n_err,total,rate", [(0, 5, 0.0), (100, 100, 1.0), (1, 4, 0.25)])
def test_error_rate_edges(n_err, total, rate):
    c = MetricsCollector(worker_id="edge")
    for i in range(total):
        c.record_request("decode", 0.0, 1_000_000 if i == 0 else 1, success=i >= n_err)
    s = c.get_summary()
    assert s["error_rate"] == pytest.approx(rate) and s["avg_latency_ms"] == 0.0


def test_full_workflow_counts():
    c = MetricsCollector(worker_id="wf", model_name="llama", worker_role="hybrid")
    for i in range(5):
        c.record_request("prefill", 0.1 + i * 0.02, 512, True)
        c.record_batch("prefill", 4)
        for _ in range(10):
            c.record_request("decode", 0.01, 1, True)
    s = c.get_summary()
    assert (s["total_requests"], s["error_count"], s["total_tokens"]) == (55, 0, 5 * 512 + 50)


# ----------------------------------------------------------------------------- logging

def test_logger_context_lifecycle():
    lg = StructuredLogger(name="t")
    assert lg.logger is not None and lg._context == {}
    lg.set_context(worker_id="w1", model="m")
    assert lg._format_extra({"k": "v"}) == {"worker_id": "w1", "model": "m", "k": "v"}
    lg.clear_context()
    assert lg._context == {}


@pytest.mark.parametrize("level", ["info", "warning", "error", "debug"])
def test_logger_levels_carry_context(level):
    lg = StructuredLogger(name="t2")
    lg.set_context(session_id="abc")
    with patch.object(lg.logger, level) as m:
        getattr(lg, level)("msg", request_id="r1")
    m.assert_called_once()
    extra = m.call_args.kwargs["extra"]
    assert extra["session_id"] == "abc" and extra["request_id"] == "r1"


def test_logger_reserved_names_are_renamed_not_fatal(caplog):
    lg = StructuredLogger(name="t3")
    with caplog.at_level("INFO", logger="t3"):
        lg.info("hello", name="clash", lineno="clash2")
    assert caplog.records and caplog.records[0].x_name == "clash"


# ----------------------------------------------------------------------------- HTTP surface

def test_metrics_endpoint_variants():
    ep = create_metrics_endpoint()
    assert asyncio.iscoroutinefunction(ep)
    resp = asyncio.run(ep())
    assert b"inference_requests_total" in resp.body
    with patch.object(obs, "HAS_PROMETHEUS", False):
        assert "error" in asyncio.run(create_metrics_endpoint()())


def test_setup_routes_includes_one_router():
    app = MagicMock()
    setup_metrics_routes(app)
    app.include_router.assert_called_once()


def test_routes_serve_metrics_live_ready():
    from fastapi import FastAPI
    from fastapi.testclient import TestClient
    app = FastAPI()
    state = {"ok": False}
    setup_metrics_routes(app, ready_check=lambda: state["ok"])
    c = TestClient(app)
    assert c.get("/metrics").status_code == 200
    assert c.get("/live").json()["status"] == "healthy"
    assert c.get("/ready").json()["status"] == "not_ready"
    state["ok"] = True
    assert c.get("/ready").json()["status"] == "ready"
