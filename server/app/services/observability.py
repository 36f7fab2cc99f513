"""Metrics, tracing and structured logs (reference services/observability.py:20-488).

Same metric names/labels.  Mounted on the server and the
worker direct server (``setup_metrics_routes``) and fed by the dgi engine
(batch sizes, prefill/decode latency, TTFT/TPOT, KV hit rates, migration
latency, speculative accept rate).  prometheus_client and OpenTelemetry
are optional: without them the collectors keep in-process counters only.
"""
from __future__ import annotations

import functools
import logging
import time
from contextlib import contextmanager
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Optional

logger = logging.getLogger(__name__)

try:
    from prometheus_client import CONTENT_TYPE_LATEST, Counter, Gauge, Histogram, generate_latest
    HAS_PROMETHEUS = True
except Exception:  # pragma: no cover
    HAS_PROMETHEUS = False

try:
    from opentelemetry import trace
    HAS_OTEL = True
except Exception:  # pragma: no cover
    trace = None
    HAS_OTEL = False

LAT_BUCKETS = (0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0)

if HAS_PROMETHEUS:
    def _mk(kind, name, desc, labels, **kw):
        try:
            return kind(name, desc, labels, **kw)
        except ValueError:  # already registered (module reloaded)
            from prometheus_client import REGISTRY
            return REGISTRY._names_to_collectors.get(name) or kind(name, desc, labels, registry=None, **kw)

    INFERENCE_REQUESTS_TOTAL = _mk(Counter, "inference_requests_total", "Inference requests", ["model", "worker_id", "status"])
    INFERENCE_LATENCY = _mk(Histogram, "inference_latency_seconds", "Inference latency", ["model", "phase", "worker_role"],
                            buckets=LAT_BUCKETS)
    TOKENS_GENERATED = _mk(Counter, "tokens_generated_total", "Generated tokens", ["model", "worker_id"])
    TOKENS_PER_SECOND = _mk(Gauge, "tokens_per_second", "Token throughput", ["model", "worker_id"])
    KV_CACHE_HIT_RATE = _mk(Gauge, "kv_cache_hit_rate", "KV cache hit rate", ["level"])
    KV_CACHE_SIZE_BYTES = _mk(Gauge, "kv_cache_size_bytes", "KV cache bytes", ["level", "worker_id"])
    KV_CACHE_EVICTIONS = _mk(Counter, "kv_cache_evictions_total", "KV evictions", ["level", "worker_id"])
    WORKER_STATUS = _mk(Gauge, "worker_status", "Worker status", ["worker_id", "role"])
    GPU_MEMORY_USED = _mk(Gauge, "gpu_memory_used_bytes", "GPU memory used", ["worker_id", "gpu_id"])
    GPU_MEMORY_TOTAL = _mk(Gauge, "gpu_memory_total_bytes", "GPU memory total", ["worker_id", "gpu_id"])
    GPU_UTILIZATION = _mk(Gauge, "gpu_utilization_percent", "GPU utilization", ["worker_id", "gpu_id"])
    DISTRIBUTED_HOPS = _mk(Histogram, "distributed_inference_hops", "Pipeline hops", ["model"])
    KV_MIGRATION_LATENCY = _mk(Histogram, "kv_migration_latency_seconds", "KV migration latency",
                               ["source_worker", "target_worker"], buckets=LAT_BUCKETS)
    BATCH_SIZE = _mk(Histogram, "batch_size", "Batch size", ["phase"], buckets=(1, 2, 4, 8, 16, 32, 64, 128, 256, 512))
    QUEUE_SIZE = _mk(Gauge, "queue_size", "Queue size", ["phase"])
    SPECULATIVE_ACCEPT_RATE = _mk(Gauge, "speculative_accept_rate", "Speculative accept rate", ["worker_id"])
    SPECULATIVE_SPEEDUP = _mk(Gauge, "speculative_speedup", "Speculative speedup", ["worker_id"])


class TracingManager:
    def __init__(self, service_name: str = "distributed-inference"):
        self.service_name = service_name
        self._tracer = None
        self._enabled = False
        self.sample_rate = 1.0

    def setup(self, exporter: str = "console", endpoint: Optional[str] = None, sample_rate: float = 1.0) -> bool:
        """Install an OTel tracer provider (console or OTLP exporter) when OTel is available."""
        self.sample_rate = sample_rate
        if not HAS_OTEL:
            return False
        try:
            from opentelemetry.sdk.resources import Resource
            from opentelemetry.sdk.trace import TracerProvider
            from opentelemetry.sdk.trace.export import BatchSpanProcessor, ConsoleSpanExporter
            from opentelemetry.sdk.trace.sampling import TraceIdRatioBased
            provider = TracerProvider(resource=Resource.create({"service.name": self.service_name}),
                                      sampler=TraceIdRatioBased(sample_rate))
            if exporter == "otlp" and endpoint:
                from opentelemetry.exporter.otlp.proto.grpc.trace_exporter import OTLPSpanExporter
                provider.add_span_processor(BatchSpanProcessor(OTLPSpanExporter(endpoint=endpoint)))
            else:
                provider.add_span_processor(BatchSpanProcessor(ConsoleSpanExporter()))
            trace.set_tracer_provider(provider)
            self._tracer = trace.get_tracer(self.service_name)
            self._enabled = True
        except Exception as e:
            logger.info("tracing not enabled: %s", e)
            self._enabled = False
        return self._enabled

    @contextmanager
    def span(self, name: str, attributes: Optional[Dict[str, Any]] = None):
        if not self._enabled or self._tracer is None:
            yield None
            return
        with self._tracer.start_as_current_span(name) as sp:
            for k, v in (attributes or {}).items():
                sp.set_attribute(k, v)
            try:
                yield sp
            except Exception as e:
                sp.set_status(trace.Status(trace.StatusCode.ERROR, str(e)))
                raise

    def trace_inference(self, func: Callable) -> Callable:
        @functools.wraps(func)
        async def wrapper(*args, **kwargs):
            t0 = time.perf_counter()
            with self.span(f"inference.{func.__name__}") as sp:
                out = await func(*args, **kwargs)
                if sp is not None:
                    sp.set_attribute("inference.latency_ms", (time.perf_counter() - t0) * 1000)
                    if isinstance(out, dict) and "usage" in out:
                        sp.set_attribute("inference.tokens", out["usage"].get("completion_tokens", 0))
                return out
        return wrapper


@dataclass
class MetricsCollector:
    worker_id: str
    model_name: str = ""
    worker_role: str = "hybrid"
    _request_count: int = 0
    _token_count: int = 0
    _error_count: int = 0
    _latency_sum: float = 0.0
    _last_update: float = field(default_factory=time.time)
    _total_tokens: int = 0
    _tps: float = 0.0

    def record_request(self, phase: str, latency_seconds: float, tokens: int = 0, success: bool = True) -> None:
        self._request_count += 1
        self._token_count += tokens
        self._total_tokens += tokens
        self._latency_sum += latency_seconds
        if not success:
            self._error_count += 1
        if HAS_PROMETHEUS:
            INFERENCE_REQUESTS_TOTAL.labels(model=self.model_name, worker_id=self.worker_id,
                                            status="success" if success else "error").inc()
            INFERENCE_LATENCY.labels(model=self.model_name, phase=phase, worker_role=self.worker_role).observe(latency_seconds)
            if tokens > 0:
                TOKENS_GENERATED.labels(model=self.model_name, worker_id=self.worker_id).inc(tokens)

    def record_batch(self, phase: str, batch_size: int) -> None:
        if HAS_PROMETHEUS:
            BATCH_SIZE.labels(phase=phase).observe(batch_size)

    def record_queue(self, phase: str, size: int) -> None:
        if HAS_PROMETHEUS:
            QUEUE_SIZE.labels(phase=phase).set(size)

    def record_kv_cache_stats(self, level: str, hit_rate: float, size_bytes: int = 0, evictions: int = 0) -> None:
        if HAS_PROMETHEUS:
            KV_CACHE_HIT_RATE.labels(level=level).set(hit_rate)
            if size_bytes > 0:
                KV_CACHE_SIZE_BYTES.labels(level=level, worker_id=self.worker_id).set(size_bytes)
            if evictions > 0:
                KV_CACHE_EVICTIONS.labels(level=level, worker_id=self.worker_id).inc(evictions)

    def record_gpu_stats(self, gpu_id: int, memory_used: int, memory_total: int, utilization: float = 0.0) -> None:
        if HAS_PROMETHEUS:
            GPU_MEMORY_USED.labels(worker_id=self.worker_id, gpu_id=str(gpu_id)).set(memory_used)
            GPU_MEMORY_TOTAL.labels(worker_id=self.worker_id, gpu_id=str(gpu_id)).set(memory_total)
            GPU_UTILIZATION.labels(worker_id=self.worker_id, gpu_id=str(gpu_id)).set(utilization)

    def record_migration(self, source: str, target: str, seconds: float) -> None:
        if HAS_PROMETHEUS:
            KV_MIGRATION_LATENCY.labels(source_worker=source, target_worker=target).observe(seconds)

    def record_hops(self, hops: int) -> None:
        if HAS_PROMETHEUS:
            DISTRIBUTED_HOPS.labels(model=self.model_name).observe(hops)

    def record_speculative_stats(self, accept_rate: float, speedup: float) -> None:
        if HAS_PROMETHEUS:
            SPECULATIVE_ACCEPT_RATE.labels(worker_id=self.worker_id).set(accept_rate)
            SPECULATIVE_SPEEDUP.labels(worker_id=self.worker_id).set(speedup)

    def record_worker_status(self, status_value: float) -> None:
        if HAS_PROMETHEUS:
            WORKER_STATUS.labels(worker_id=self.worker_id, role=self.worker_role).set(status_value)

    def update_tokens_per_second(self) -> None:
        now = time.time()
        dt = now - self._last_update
        if dt > 0:
            self._tps = self._token_count / dt
            if HAS_PROMETHEUS:
                TOKENS_PER_SECOND.labels(model=self.model_name, worker_id=self.worker_id).set(self._tps)
        self._token_count = 0
        self._last_update = now

    def record_engine_stats(self, stats: Dict[str, Any]) -> None:
        """Feed a ``dgi`` engine stats dict (NativeLLMEngine.get_status()['engine'])."""
        if not stats:
            return
        self.record_queue("prefill", int(stats.get("waiting", 0)))
        self.record_queue("decode", int(stats.get("running", 0)))
        self.record_kv_cache_stats("gpu", float(stats.get("prefix_hit_rate", 0.0)))

    def get_summary(self) -> Dict[str, Any]:
        n = self._request_count
        return {"worker_id": self.worker_id, "model_name": self.model_name, "worker_role": self.worker_role,
                "total_requests": n, "total_tokens": self._total_tokens, "error_count": self._error_count,
                "error_rate": self._error_count / n if n else 0.0,
                "avg_latency_ms": self._latency_sum / n * 1000.0 if n else 0.0, "tokens_per_second": self._tps}


def create_metrics_endpoint():
    if not HAS_PROMETHEUS:
        async def metrics_disabled():
            return {"error": "prometheus_client not installed"}
        return metrics_disabled

    async def metrics():
        from fastapi import Response
        return Response(content=generate_latest(), media_type=CONTENT_TYPE_LATEST)
    return metrics


def setup_metrics_routes(app, ready_check: Optional[Callable[[], bool]] = None) -> None:
    """Mount ``/metrics`` (Prometheus), ``/live`` and ``/ready`` as one router."""
    from fastapi import APIRouter
    router = APIRouter(tags=["observability"])
    router.add_api_route("/metrics", create_metrics_endpoint(), methods=["GET"], include_in_schema=False)

    async def live():
        return {"status": "healthy", "timestamp": time.time()}

    async def ready():
        ok = True if ready_check is None else bool(ready_check())
        return {"status": "ready" if ok else "not_ready", "timestamp": time.time()}
    router.add_api_route("/live", live, methods=["GET"])
    router.add_api_route("/ready", ready, methods=["GET"])
    app.include_router(router)


class StructuredLogger:
    def __init__(self, name: str = "distributed-inference"):
        self.logger = logging.getLogger(name)
        self._context: Dict[str, Any] = {}

    def set_context(self, **kwargs) -> None:
        self._context.update(kwargs)

    def clear_context(self) -> None:
        self._context.clear()

    _RESERVED = frozenset(logging.LogRecord("", 0, "", 0, "", (), None).__dict__) | {"message", "asctime"}

    def _format_extra(self, extra: Dict[str, Any]) -> Dict[str, Any]:
        # LogRecord attribute names cannot be overridden through ``extra``
        return {(f"x_{k}" if k in self._RESERVED else k): v for k, v in {**self._context, **extra}.items()}

    def info(self, message: str, **extra) -> None:
        self.logger.info(message, extra=self._format_extra(extra))

    def warning(self, message: str, **extra) -> None:
        self.logger.warning(message, extra=self._format_extra(extra))

    def error(self, message: str, **extra) -> None:
        self.logger.error(message, extra=self._format_extra(extra))

    def debug(self, message: str, **extra) -> None:
        self.logger.debug(message, extra=self._format_extra(extra))
