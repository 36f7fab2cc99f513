"""Worker daemon (reference worker/main.py:28-521).

Registers with the control plane (or re-uses saved credentials), loads the
configured engines, heartbeats, and pulls jobs.  MI355X-first difference:
the ``llm`` engine is a continuous-batching ``dgi`` runtime, so the daemon
keeps up to ``max_concurrent_jobs`` jobs in flight at once (each on a
worker thread that blocks in ``engine.inference``) and they batch together
inside the engine step loop; the reference processed one job at a time.

Graceful shutdown (SIGINT/SIGTERM): stop pulling, tell the server
``going-offline``, drain in-flight jobs, then ``offline``.
"""
from __future__ import annotations

import logging
import os
import random
import signal
import sys
import threading
import time
from concurrent.futures import Future, ThreadPoolExecutor
from datetime import datetime
from typing import Any, Dict, List, Optional

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from api_client import APIClient  # noqa: E402
from config import WorkerConfig, load_config  # noqa: E402
from engines import ENGINE_REGISTRY, create_llm_engine, get_engine  # noqa: E402
from observability_bridge import load_observability  # noqa: E402

logger = logging.getLogger("worker")


class _JobBatcher:
    """Job-level ``ContinuousBatcher`` on its own event-loop thread, for engines
    that batch whole requests (HF / vLLM / SGLang adapters).  The native dgi
    engines batch per iteration themselves and bypass it."""

    def __init__(self, engine, max_batch_size: int, max_wait_ms: float):
        import asyncio
        from batch_processor import ContinuousBatcher
        self.loop = asyncio.new_event_loop()
        self.thread = threading.Thread(target=self.loop.run_forever, name="job-batcher", daemon=True)
        self.thread.start()
        self.batcher = ContinuousBatcher(engine, max_batch_size=max_batch_size, max_wait_ms=max_wait_ms)
        asyncio.run_coroutine_threadsafe(self.batcher.start(), self.loop).result()

    def run(self, job_id: str, params: Dict[str, Any], timeout: float) -> Dict[str, Any]:
        import asyncio
        return asyncio.run_coroutine_threadsafe(self.batcher.submit(job_id, params, timeout=timeout),
                                                self.loop).result()

    def close(self) -> None:
        import asyncio
        try:
            asyncio.run_coroutine_threadsafe(self.batcher.stop(), self.loop).result(timeout=10)
        finally:
            self.loop.call_soon_threadsafe(self.loop.stop)

LLM_BACKENDS = {"native", "transformers", "mi355x", "dgi", "llm_native", "sglang", "vllm", "vllm_async",
                "mi355x-node", "node", "llm_node"}


class Worker:
    def __init__(self, config: Optional[WorkerConfig] = None, config_path: str = "config.yaml"):
        self.config = config or load_config(config_path)
        self.config_path = config_path
        self.api_client = APIClient(self.config.server.url, self.config.token, self.config.server.timeout,
                                    verify_ssl=self.config.server.verify_ssl)
        self.worker_id: Optional[str] = self.config.worker_id
        self.engines: Dict[str, Any] = {}
        self.remote_config: Dict[str, Any] = {}
        self.config_version = 0
        self.running = False
        self.accepting_jobs = True
        self.shutdown_event = threading.Event()
        self._inflight: Dict[str, Future] = {}
        self._lock = threading.Lock()
        self._executor: Optional[ThreadPoolExecutor] = None
        self._jobs_this_hour = 0
        self._hour = -1
        self._last_job_end = 0.0
        self.direct_server = None
        self._hb_thread: Optional[threading.Thread] = None
        self._batchers: Dict[str, _JobBatcher] = {}
        self.metrics = None
        self.tracer = None
        self._setup_observability()

    # ------------------------------------------------------------------ state
    @property
    def current_job_id(self) -> Optional[str]:
        with self._lock:
            return next(iter(self._inflight), None)

    @property
    def status(self) -> str:
        if not self.accepting_jobs:
            return "going_offline"
        return "busy" if self.inflight_count() >= self.max_concurrent_jobs() else "online"

    def inflight_count(self) -> int:
        with self._lock:
            return len(self._inflight)

    def max_concurrent_jobs(self) -> int:
        return max(1, int(self.config.load_control.max_concurrent_jobs))

    def _get_gpu_info(self) -> Dict[str, Any]:
        try:
            from engines.base import gpu_summary
            return gpu_summary(self.config.gpu.device_id) or {}
        except Exception:
            return {}

    # ------------------------------------------------------------------ registration
    def _register(self) -> None:
        if self.worker_id and self.config.token:
            self.api_client.set_credentials(self.config.token, self.config.signing_secret)
            if self._verify_credentials():
                logger.info("reusing credentials of worker %s", self.worker_id)
                return
            if self.config.refresh_token and self.api_client.refresh_token(self.worker_id, self.config.refresh_token):
                self._persist_tokens(self.api_client.token, None)
                return
            logger.warning("saved credentials rejected; registering again")
        self._do_register()

    def _do_register(self) -> None:
        from machine_id import MachineFingerprint
        gpu = self._get_gpu_info()
        fp = MachineFingerprint.get_or_create()
        d = self.config.direct
        data = self.api_client.register(
            name=self.config.name or f"worker-{fp['machine_id'][:8]}", region=self.config.region,
            country=self.config.country, city=self.config.city, timezone=self.config.timezone,
            gpu_model=gpu.get("name"), gpu_memory_gb=gpu.get("memory_total_gb"),
            gpu_count=len(self.config.gpu.device_ids) or gpu.get("count", 1) or 1, cpu_cores=os.cpu_count(),
            supported_types=list(self.engines or self.config.supported_types),
            direct_url=d.public_url or (f"http://{d.host}:{d.port}" if d.enabled else None),
            supports_direct=d.enabled, machine_id=fp["machine_id"], hardware_details=fp.get("details"),
            role=self.config.role,
            # a continuous-batching engine serves many jobs at once: advertise how many this
            # worker runs concurrently (the control plane otherwise assigns one at a time)
            capabilities={"max_concurrent_jobs": self.max_concurrent_jobs(),
                          "continuous_batching": any(type(e).__name__ in ("NativeLLMEngine", "NodeLLMEngine")
                                                     for e in self.engines.values())})
        self.worker_id = data["worker_id"]
        self.config.worker_id = self.worker_id
        self.config.signing_secret = data.get("signing_secret")
        self._persist_tokens(data["token"], data.get("refresh_token"))
        logger.info("registered as worker %s", self.worker_id)

    def _persist_tokens(self, token: str, refresh: Optional[str]) -> None:
        self.config.token = token
        if refresh:
            self.config.refresh_token = refresh
        try:
            self.config.save(self.config_path)
        except OSError as e:
            logger.warning("cannot persist credentials: %s", e)

    def _verify_credentials(self) -> bool:
        return bool(self.worker_id and self.config.token and
                    self.api_client.verify_credentials(self.worker_id, self.config.token))

    def _refresh_token_if_needed(self) -> None:
        if self.config.refresh_token and self.worker_id:
            data = self.api_client.refresh_token(self.worker_id, self.config.refresh_token)
            if data:
                self._persist_tokens(data["token"], data.get("refresh_token"))

    # ------------------------------------------------------------------ remote config / load control
    def _fetch_remote_config(self) -> None:
        cfg = self.api_client.get_config(self.worker_id) if self.worker_id else None
        if not cfg:
            return
        self.remote_config = cfg
        self.config_version = int(cfg.get("version", 0))
        if cfg.get("load_control"):
            self._apply_load_control(cfg["load_control"])

    def _apply_load_control(self, lc: Dict[str, Any]) -> None:
        cur = self.config.load_control
        for k in ("acceptance_rate", "max_concurrent_jobs", "max_jobs_per_hour", "working_hours_start",
                  "working_hours_end"):
            if k in lc and lc[k] is not None:
                setattr(cur, k, lc[k])
        self.cooldown_seconds = int(lc.get("cooldown_seconds") or 0)

    def _should_accept_job(self) -> bool:
        lc = self.config.load_control
        now = datetime.now()
        s, e = lc.working_hours_start, lc.working_hours_end
        if s is not None and e is not None:
            inside = (s <= now.hour < e) if s <= e else (now.hour >= s or now.hour < e)
            if not inside:
                return False
        hour = int(time.time() // 3600)
        if hour != self._hour:
            self._hour, self._jobs_this_hour = hour, 0
        if lc.max_jobs_per_hour and self._jobs_this_hour >= lc.max_jobs_per_hour:
            return False
        if time.time() - self._last_job_end < getattr(self, "cooldown_seconds", 0):
            return False
        return lc.acceptance_rate >= 1.0 or random.random() < lc.acceptance_rate

    # ------------------------------------------------------------------ engines
    def _load_engines(self) -> None:
        model_cfgs = self.remote_config.get("model_configs", {}) if self.remote_config else {}
        for t in list(self.config.supported_types):
            cfg = self.config.engine_config(t)
            if t == "llm" and len(cfg.get("device_ids") or []) > 1 and cfg.get("backend") in ("mi355x", "dgi"):
                cfg["backend"] = "mi355x-node"      # a multi-GPU worker serves through the node server
            if t in model_cfgs:
                cfg.update({k: v for k, v in model_cfgs[t].items() if v is not None and k != "model_id"})
            try:
                if t == "llm" and str(cfg.get("backend", "native")).lower() in LLM_BACKENDS:
                    engine = create_llm_engine(cfg)
                else:
                    engine = get_engine(t)(cfg)
                engine.load_model()
                self.engines[t] = engine
                self._maybe_batcher(t, engine)
                logger.info("engine %s loaded (%s)", t, type(engine).__name__)
            except Exception as e:
                logger.error("failed to load engine %s: %s", t, e)
                self.config.supported_types.remove(t)

    def _get_loaded_models(self) -> List[str]:
        out = []
        for e in self.engines.values():
            mid = getattr(e, "model_id", None) or (getattr(e, "config", {}) or {}).get("model_id")
            if mid:
                out.append(str(mid))
        return out

    # ------------------------------------------------------------------ jobs
    def _setup_observability(self) -> None:
        obs_cfg = self.config.observability
        try:
            obs = load_observability()
        except Exception as e:  # pragma: no cover - optional deps
            logger.info("observability unavailable: %s", e)
            return
        if obs is None:
            return
        if obs_cfg.metrics.enabled:
            self.metrics = obs.MetricsCollector(worker_id=self.config.worker_id or "unregistered",
                                                model_name=str(self.config.engine_config("llm").get("model_id", "")),
                                                worker_role=self.config.role)
        self.tracer = obs.TracingManager(service_name="gpu-worker")
        if obs_cfg.tracing.enabled and self.tracer.setup(obs_cfg.tracing.exporter, obs_cfg.tracing.endpoint,
                                                         obs_cfg.tracing.sample_rate):
            from dgi.utils.trace import set_tracer
            set_tracer(self.tracer)      # engine step phases become child spans

    def _maybe_batcher(self, job_type: str, engine) -> None:
        b = self.config.inference.batch
        native = type(engine).__name__ in ("NativeLLMEngine", "NodeLLMEngine")
        batchable = hasattr(engine, "batch_inference_async") or hasattr(engine, "batch_inference")
        if job_type == "llm" and not native and batchable and b.max_batch_size > 1:
            self._batchers[job_type] = _JobBatcher(engine, b.max_batch_size, b.max_wait_ms)

    def execute(self, job_type: str, params: Dict[str, Any], job_id: str = "direct") -> Dict[str, Any]:
        if job_type == "llm" and params.get("pd"):
            return self._execute_pd(params, job_id)
        return self._execute(job_type, params, job_id)

    def _execute_pd(self, params: Dict[str, Any], job_id: str) -> Dict[str, Any]:
        """Cluster P/D job (server services/pd_runtime.py).

        Prefill phase: one token, reported with the KV key the decode placement
        uses; a native engine keeps the sequence's pages under that key and the
        result names the URL they can be pulled from (``GET /kv/{key}`` on this
        worker's direct server).  Decode phase: the full completion on the worker
        the P/D scheduler chose — from the pulled pages when ``kv_url`` is given
        (no prompt recompute: the reference's ``TransferKVCache`` made real,
        dgi/kv/transfer.py), else by re-prefilling.  Inside one MI355X node dgi
        migrates KV over RCCL instead (dgi/parallel/pd.py)."""
        phase = params.get("pd_phase", "prefill")
        key = f"{getattr(self, 'worker_id', None)}:{job_id}"
        engine = getattr(self, "engines", {}).get("llm")
        if phase == "prefill":
            if engine is not None and hasattr(engine, "prefill_export"):
                out = engine.prefill_export({**params, "max_tokens": 1}, key)
                base = self._kv_pull_base()
                return {**out, "phase": "prefill", "first_token": out.get("response", ""), "kv_cache_key": key,
                        "kv_url": f"{base.rstrip('/')}/kv/{key}" if base else None}
            out = self._execute("llm", {**params, "max_tokens": 1}, job_id)
            return {**out, "phase": "prefill", "first_token": out.get("response", ""), "kv_cache_key": key}
        clean = {k: v for k, v in params.items() if k not in ("pd_phase", "first_token", "kv_url", "kv_token")}
        if engine is not None and hasattr(engine, "decode_import"):
            # decode placed on the worker that prefilled: the pages are in our own store
            store = getattr(engine, "kv_exports", None)
            own = store.take(key, check_token=False) if store is not None else None
            if own is not None:
                out = engine.decode_import(clean, own)
                return {**out, "phase": "decode", "kv_source": "local", "reprefilled": False,
                        "kv_bytes": len(own), "kv_pull_ms": 0.0}
            url = params.get("kv_url")
            if url and self._kv_url_ok(url, job_id):
                try:
                    import httpx
                    t0 = time.perf_counter()
                    r = httpx.get(url, timeout=60.0, follow_redirects=False,
                                  headers={"X-KV-Token": str(params.get("kv_token") or "")})
                    r.raise_for_status()
                    pull_ms = (time.perf_counter() - t0) * 1000.0
                    out = engine.decode_import(clean, r.content)
                    return {**out, "phase": "decode", "kv_source": params.get("kv_source"), "reprefilled": False,
                            "kv_bytes": len(r.content), "kv_pull_ms": round(pull_ms, 2)}
                except Exception as e:     # source gone / evicted: fall back to recomputing the prompt
                    logger.warning("KV pull from %s failed (%s): re-prefilling", url, e)
        out = self._execute("llm", clean, job_id)
        return {**out, "phase": "decode", "kv_source": params.get("kv_source"), "reprefilled": True}

    def _kv_pull_base(self) -> Optional[str]:
        """Base URL decode workers pull this worker's exported KV from: the direct
        server's public URL.  A loopback address is only reachable from this host,
        so it is advertised only when the operator set it explicitly (a decode
        worker elsewhere would pull from its own localhost and silently re-prefill)."""
        base = getattr(self, "direct_url", None)
        if not base:
            return None
        from urllib.parse import urlparse
        host = (urlparse(base).hostname or "").lower()
        explicit = bool(getattr(getattr(getattr(self, "config", None), "direct", None), "public_url", None))
        if host in ("127.0.0.1", "localhost", "::1") and not explicit and not getattr(self, "kv_loopback_ok", False):
            if not getattr(self, "_warned_loopback", False):
                logger.warning("direct server has no public URL (set GPU_DIRECT_PUBLIC_URL): exported KV is not "
                               "advertised to decode workers on other hosts")
                self._warned_loopback = True
            return None
        return base

    @staticmethod
    def _kv_url_ok(url: str, job_id: str) -> bool:
        """Only pull what the coordinator can have handed us: an http(s) ``/kv/<worker>:<job>``
        URL of THIS job, no query, no credentials (a client-supplied URL is stripped by the
        coordinator; this refuses anything else that reaches the worker)."""
        from urllib.parse import unquote, urlparse
        u = urlparse(url)
        if u.scheme not in ("http", "https") or not u.hostname or u.username or u.password or u.query:
            return False
        path = unquote(u.path)
        return path.startswith("/kv/") and path.endswith(f":{job_id}") and "/" not in path[4:]

    def _execute(self, job_type: str, params: Dict[str, Any], job_id: str = "direct") -> Dict[str, Any]:
        engine = self.engines.get(job_type)
        if engine is None:
            raise ValueError(f"No engine for type: {job_type}")
        t0 = time.perf_counter()
        ok = False
        span = self.tracer.span("job.execute", {"job.id": job_id, "job.type": job_type}) if self.tracer else None
        try:
            if span is not None:
                span.__enter__()
            batcher = self._batchers.get(job_type)
            if batcher is not None:
                out = batcher.run(job_id, params, timeout=float(params.get("timeout", 300)))
            else:
                out = engine.inference(params)
            ok = True
            return out
        finally:
            if span is not None:
                span.__exit__(None, None, None)
            if self.metrics is not None:
                toks = 0
                if ok and isinstance(out, dict):
                    toks = int((out.get("usage") or {}).get("completion_tokens", 0) or 0)
                self.metrics.record_request("e2e", time.perf_counter() - t0, toks, ok)

    def _process_job(self, job: Dict[str, Any]) -> None:
        job_id, t0 = job["job_id"], time.time()
        try:
            result = self.execute(job["type"], job.get("params") or {}, job_id)
            ms = int((time.time() - t0) * 1000)
            usage = (result or {}).get("usage") if isinstance(result, dict) else None
            self.api_client.complete_job(self.worker_id, job_id, True, result=result, processing_time_ms=ms,
                                         usage=usage)
            logger.info("job %s done in %d ms", job_id, ms)
        except Exception as e:
            logger.error("job %s failed: %s", job_id, e)
            try:
                self.api_client.complete_job(self.worker_id, job_id, False, error=str(e))
            except Exception as e2:
                logger.error("cannot report failure of %s: %s", job_id, e2)
        finally:
            with self._lock:
                self._inflight.pop(job_id, None)
            self._last_job_end = time.time()

    def _dispatch(self, job: Dict[str, Any]) -> None:
        with self._lock:
            self._inflight[job["job_id"]] = self._executor.submit(self._process_job, job)
        self._jobs_this_hour += 1

    def _main_loop(self) -> None:
        while self.running:
            if not self.accepting_jobs:
                if self.inflight_count() == 0:
                    break
                self.shutdown_event.wait(0.2)
                continue
            got = False
            free = self.max_concurrent_jobs() - self.inflight_count()
            if free > 0 and self._should_accept_job():
                wait = float(getattr(self.config, "long_poll_s", 0.0) or 0.0)
                try:
                    # a burst of queued jobs in one round trip (GET next-jobs), else one (next-job)
                    jobs = self.api_client.fetch_next_jobs(self.worker_id, free, wait=wait)
                except Exception as e:
                    logger.error("fetch failed: %s", e)
                    jobs = []
                for job in jobs:
                    self._dispatch(job)
                    got = True
            if not got:
                self.shutdown_event.wait(self.config.poll_interval)

    # ------------------------------------------------------------------ heartbeat
    def _heartbeat_once(self) -> None:
        gpu = self._get_gpu_info()
        stats = None
        llm = self.engines.get("llm")
        if llm is not None:
            try:
                stats = llm.get_status().get("engine")
            except Exception:
                stats = None
        resp = self.api_client.heartbeat(self.worker_id, self.status, self.current_job_id,
                                         gpu.get("memory_used_gb"), list(self.engines), self._get_loaded_models(),
                                         self.config_version, engine_stats=stats)
        if resp.get("config_changed") or resp.get("action") == "reload_config":
            self._fetch_remote_config()
        if resp.get("action") == "refresh_token":
            self._refresh_token_if_needed()
        elif resp.get("action") == "shutdown":
            self.request_shutdown(graceful=True)

    def _heartbeat_loop(self) -> None:
        while self.running and not self.shutdown_event.is_set():
            try:
                self._heartbeat_once()
            except Exception as e:
                logger.error("heartbeat error: %s", e)
            self.shutdown_event.wait(self.config.heartbeat_interval)

    # ------------------------------------------------------------------ lifecycle
    def _start_direct_server(self) -> None:
        if not self.config.direct.enabled:
            return
        from direct_server import DirectServer
        self.direct_server = DirectServer(self, self.config.direct.host, self.config.direct.port)
        self.direct_server.start_background()
        d = self.config.direct
        # where decode workers pull this worker's exported KV (cluster P/D, GET /kv/{key})
        self.direct_url = d.public_url or f"http://{'127.0.0.1' if d.host in ('0.0.0.0', '') else d.host}:{d.port}"

    def start(self, install_signals: bool = True) -> None:
        self._load_engines()
        if not self.engines:
            raise RuntimeError("no engine could be loaded")
        self._register()
        self._fetch_remote_config()
        self._executor = ThreadPoolExecutor(max_workers=max(self.max_concurrent_jobs(), 1),
                                            thread_name_prefix="job")
        self.running = True
        if install_signals and threading.current_thread() is threading.main_thread():
            signal.signal(signal.SIGINT, self._signal_handler)
            signal.signal(signal.SIGTERM, self._signal_handler)
        self._hb_thread = threading.Thread(target=self._heartbeat_loop, name="heartbeat", daemon=True)
        self._hb_thread.start()
        self._start_direct_server()
        logger.info("worker %s serving %s", self.worker_id, list(self.engines))
        try:
            self._main_loop()
        finally:
            self.shutdown()

    def request_shutdown(self, graceful: bool = True) -> None:
        if not self.accepting_jobs:
            return
        self.accepting_jobs = False
        try:
            if self.worker_id:
                self.api_client.notify_going_offline(self.worker_id, finish_current=graceful)
        except Exception as e:
            logger.warning("going-offline notification failed: %s", e)
        if not graceful:
            self.running = False
        self.shutdown_event.set()

    def shutdown(self) -> None:
        self.running = False
        self.shutdown_event.set()
        if self._executor is not None:
            self._executor.shutdown(wait=True)
        for b in self._batchers.values():
            b.close()
        self._batchers.clear()
        if self.worker_id:
            self.api_client.notify_offline(self.worker_id)
        if self.direct_server is not None:
            self.direct_server.stop()
        for e in self.engines.values():
            try:
                e.unload_model()
            except Exception:
                pass
        self.api_client.close()

    def _signal_handler(self, signum, frame) -> None:
        logger.info("signal %s: graceful shutdown", signum)
        self.request_shutdown(graceful=True)


def main(argv: Optional[List[str]] = None) -> int:
    import argparse
    ap = argparse.ArgumentParser(description="GPU inference worker")
    ap.add_argument("--config", default="config.yaml")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    Worker(config_path=a.config).start()
    return 0


if __name__ == "__main__":
    sys.exit(main())
