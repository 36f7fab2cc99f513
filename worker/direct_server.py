"""Worker direct-connect HTTP server (reference worker/direct_server.py:15-140).

``/health``, ``/status``, ``POST /inference`` (same request/response models)
plus ``POST /inference/stream`` (SSE token stream for LLM engines).  Unlike
the reference it does not reject requests while another job runs: requests
are admitted up to the worker's ``max_concurrent_jobs`` and batch together
inside the continuous-batching engine.
"""
from __future__ import annotations

import asyncio
import json
import logging
import threading
import time
from typing import Any, Dict, Optional

from fastapi import FastAPI, HTTPException, Request
from fastapi.responses import StreamingResponse
from pydantic import BaseModel

logger = logging.getLogger(__name__)

# params of the coordinator's cluster P/D job path, never taken from a direct caller
DIRECT_STRIP = ("pd", "pd_phase", "kv_url", "kv_token", "kv_source", "first_token")


class DirectInferenceRequest(BaseModel):
    type: str
    params: Dict[str, Any]
    timeout_seconds: int = 300


class DirectInferenceResponse(BaseModel):
    success: bool
    result: Optional[Dict[str, Any]] = None
    error: Optional[str] = None
    processing_time_ms: int = 0


class DirectServer:
    def __init__(self, worker, host: str = "0.0.0.0", port: int = 8080):
        self.worker = worker
        self.host = host
        self.port = port
        self.app = FastAPI(title="Worker Direct API")
        self.server = None
        self._thread: Optional[threading.Thread] = None
        self._setup_routes()

    def _admit(self, job_type: str):
        w = self.worker
        if not w.accepting_jobs:
            raise HTTPException(503, "Worker is going offline")
        if w.inflight_count() >= w.max_concurrent_jobs():
            raise HTTPException(503, "Worker is at capacity")
        engine = w.engines.get(job_type)
        if engine is None:
            raise HTTPException(400, f"Unsupported type: {job_type}. Supported: {list(w.engines)}")
        return engine

    def _setup_routes(self) -> None:
        app = self.app
        try:   # /metrics (Prometheus), /live, /ready — same routes as the control plane
            from observability_bridge import load_observability
            obs = load_observability()
            if obs is not None:
                obs.setup_metrics_routes(app, ready_check=lambda: bool(self.worker.engines))
        except Exception as e:  # pragma: no cover - optional deps
            logger.info("metrics routes not mounted: %s", e)

        @app.get("/health")
        async def health():
            return {"status": "healthy", "worker_id": self.worker.worker_id, "worker_status": self.worker.status,
                    "supported_types": list(self.worker.engines.keys())}

        @app.get("/status")
        async def status():
            w = self.worker
            return {"worker_id": w.worker_id, "status": w.status, "current_job": w.current_job_id,
                    "inflight_jobs": w.inflight_count(), "supported_types": list(w.engines.keys()),
                    "gpu_info": w._get_gpu_info(), "accepting_jobs": w.accepting_jobs,
                    "engines": {k: e.get_status() for k, e in w.engines.items()}}

        @app.get("/kv/{key}")
        async def kv_pull(key: str, request: Request):
            """Cluster P/D: the pages of a sequence this worker prefilled (dgi.kv.transfer
            blob), pulled once by the decode worker the scheduler placed it on.  The
            pull must present the export's secret (``X-KV-Token``), which the
            coordinator hands only to that decode worker; anything else gets 404 and
            leaves the blob in place."""
            from fastapi.responses import Response
            eng = self.worker.engines.get("llm")
            store = getattr(eng, "kv_exports", None)
            token = request.headers.get("X-KV-Token")
            blob = await asyncio.to_thread(store.take, key, token) if (store is not None and token) else None
            if blob is None:
                raise HTTPException(404, "no exported KV under that key for this token")
            return Response(content=blob, media_type="application/octet-stream")

        @app.post("/inference", response_model=DirectInferenceResponse)
        async def direct_inference(req: DirectInferenceRequest):
            self._admit(req.type)
            t0 = time.time()
            # cluster P/D phases only come from the coordinator's job path: a direct caller
            # cannot make this worker pull KV from a URL of its choosing
            params = {k: v for k, v in (req.params or {}).items() if k not in DIRECT_STRIP}
            try:
                result = await asyncio.wait_for(
                    asyncio.to_thread(self.worker.execute, req.type, params, "direct"),
                    timeout=req.timeout_seconds)
                return DirectInferenceResponse(success=True, result=result,
                                               processing_time_ms=int((time.time() - t0) * 1000))
            except asyncio.TimeoutError:
                return DirectInferenceResponse(success=False, error="timeout",
                                               processing_time_ms=int((time.time() - t0) * 1000))
            except Exception as e:
                logger.error("direct inference error: %s", e)
                return DirectInferenceResponse(success=False, error=str(e),
                                               processing_time_ms=int((time.time() - t0) * 1000))

        @app.post("/inference/stream")
        async def direct_stream(req: DirectInferenceRequest):
            engine = self._admit(req.type)
            if not hasattr(engine, "stream_generate"):
                raise HTTPException(400, f"engine {req.type} does not stream")
            from engines.llm_base import GenerationConfig
            p = req.params
            cfg = GenerationConfig(**{k: p[k] for k in ("max_tokens", "temperature", "top_p", "top_k", "stop")
                                      if k in p})

            async def events():
                n = 0
                try:
                    async for piece in engine.stream_generate(p.get("messages") or [], cfg):
                        n += 1
                        yield f"data: {json.dumps({'token': piece})}\n\n"
                    yield f"data: {json.dumps({'done': True, 'tokens': n})}\n\n"
                except Exception as e:
                    yield f"data: {json.dumps({'error': str(e)})}\n\n"
            return StreamingResponse(events(), media_type="text/event-stream")

    def start(self) -> None:
        import uvicorn
        config = uvicorn.Config(self.app, host=self.host, port=self.port, log_level="warning")
        self.server = uvicorn.Server(config)
        self.server.run()

    def start_background(self) -> threading.Thread:
        self._thread = threading.Thread(target=self.start, name="direct-server", daemon=True)
        self._thread.start()
        return self._thread

    def stop(self) -> None:
        if self.server is not None:
            self.server.should_exit = True
