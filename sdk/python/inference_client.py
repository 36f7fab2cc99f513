"""Python SDK for the control plane (reference sdk/python/inference_client.py:13-399).

* server jobs: ``chat`` / ``generate_image`` (sync via ``/jobs/sync`` or async
  submit), ``create_job`` / ``get_job`` / ``wait_for_job``, queue stats, workers;
* direct mode: nearest direct-capable worker (cached 60 s) then
  ``POST {worker}/inference``; ``stream_chat`` reads the worker's SSE stream;
* fail-over: every server call tries ``base_url`` then each fallback URL,
  ``max_retries`` rounds with exponential backoff; 4xx errors are not retried.
"""
from __future__ import annotations

import json
import logging
import time
from typing import Any, Dict, Iterator, List, Optional

import httpx

logger = logging.getLogger(__name__)

DIRECT_CACHE_TTL_S = 60.0


class InferenceClient:
    def __init__(self, base_url: str, api_key: Optional[str] = None, timeout: int = 120, max_retries: int = 3,
                 fallback_urls: Optional[List[str]] = None):
        self.base_url = base_url.rstrip("/")
        self.api_key = api_key
        self.timeout = timeout
        self.max_retries = max_retries
        self.fallback_urls = [u.rstrip("/") for u in (fallback_urls or [])]
        self.client = httpx.Client(timeout=timeout)
        self._direct_worker_cache: Dict[str, Dict[str, Any]] = {}

    def _headers(self) -> Dict[str, str]:
        h = {"Content-Type": "application/json"}
        if self.api_key:
            h["X-API-Key"] = self.api_key
        return h

    def _request_with_fallback(self, method: str, path: str, **kwargs) -> httpx.Response:
        kwargs.setdefault("headers", self._headers())
        bases = [self.base_url] + self.fallback_urls
        err: Optional[Exception] = None
        for attempt in range(max(1, self.max_retries)):
            for base in bases:
                try:
                    r = self.client.request(method, f"{base}{path}", **kwargs)
                    r.raise_for_status()
                    return r
                except httpx.HTTPStatusError as e:
                    if 400 <= e.response.status_code < 500:
                        raise
                    err = e
                except (httpx.TimeoutException, httpx.RequestError) as e:
                    err = e
                logger.warning("%s %s%s failed: %s", method, base, path, err)
            if attempt + 1 < self.max_retries:
                time.sleep(2 ** attempt)
        raise err  # type: ignore[misc]

    # ------------------------------------------------------------------ LLM
    @staticmethod
    def _llm_params(messages, max_tokens, temperature, **extra) -> Dict[str, Any]:
        p = {"messages": messages, "max_tokens": max_tokens, "temperature": temperature}
        p.update({k: v for k, v in extra.items() if v is not None})
        return p

    def chat(self, messages: List[Dict[str, str]], max_tokens: int = 2048, temperature: float = 0.7,
             region: Optional[str] = None, sync: bool = True, timeout: Optional[int] = None,
             use_direct: bool = False, top_p: Optional[float] = None, top_k: Optional[int] = None,
             stop: Optional[List[str]] = None) -> Dict[str, Any]:
        params = self._llm_params(messages, max_tokens, temperature, top_p=top_p, top_k=top_k, stop=stop)
        if use_direct:
            return self._direct_inference("llm", params)
        return self._submit("llm", params, region, sync, timeout)

    def stream_chat(self, messages: List[Dict[str, str]], max_tokens: int = 2048,
                    temperature: float = 0.7) -> Iterator[str]:
        """Token stream from the nearest direct worker (SSE ``/inference/stream``)."""
        w = self._get_nearest_worker("llm")
        body = {"type": "llm", "params": self._llm_params(messages, max_tokens, temperature)}
        with self.client.stream("POST", f"{w['direct_url'].rstrip('/')}/inference/stream", json=body,
                                timeout=self.timeout) as r:
            r.raise_for_status()
            for line in r.iter_lines():
                if not line.startswith("data: "):
                    continue
                ev = json.loads(line[6:])
                if "error" in ev:
                    raise RuntimeError(ev["error"])
                if ev.get("done"):
                    return
                yield ev["token"]

    # ------------------------------------------------------------------ images
    def generate_image(self, prompt: str, negative_prompt: str = "", width: int = 1024, height: int = 1024,
                       steps: int = 4, seed: Optional[int] = None, region: Optional[str] = None, sync: bool = True,
                       timeout: Optional[int] = None, use_direct: bool = False) -> Dict[str, Any]:
        params = {"prompt": prompt, "negative_prompt": negative_prompt, "width": width, "height": height,
                  "steps": steps}
        if seed is not None:
            params["seed"] = seed
        if use_direct:
            return self._direct_inference("image_gen", params)
        return self._submit("image_gen", params, region, sync, timeout)

    # ------------------------------------------------------------------ jobs
    def _submit(self, job_type: str, params: Dict[str, Any], region: Optional[str], sync: bool,
                timeout: Optional[int]) -> Dict[str, Any]:
        t = timeout or self.timeout
        path = "/api/v1/jobs/sync" if sync else "/api/v1/jobs"
        body = {"type": job_type, "params": params, "region": region, "timeout_seconds": t}
        kw: Dict[str, Any] = {"headers": self._headers(), "json": body, "timeout": t + 10}
        if sync:
            kw["params"] = {"timeout": t}
        return self._request_with_fallback("POST", path, **kw).json()

    def create_job(self, job_type: str, params: Dict[str, Any], priority: int = 0, region: Optional[str] = None,
                   allow_cross_region: bool = True, timeout_seconds: int = 300) -> Dict[str, Any]:
        body = {"type": job_type, "params": params, "priority": priority, "region": region,
                "allow_cross_region": allow_cross_region, "timeout_seconds": timeout_seconds}
        return self._request_with_fallback("POST", "/api/v1/jobs", headers=self._headers(), json=body).json()

    def get_job(self, job_id: str) -> Dict[str, Any]:
        return self._request_with_fallback("GET", f"/api/v1/jobs/{job_id}", headers=self._headers()).json()

    def cancel_job(self, job_id: str) -> Dict[str, Any]:
        return self._request_with_fallback("DELETE", f"/api/v1/jobs/{job_id}", headers=self._headers()).json()

    def wait_for_job(self, job_id: str, timeout: int = 300, poll_interval: float = 1.0) -> Dict[str, Any]:
        deadline = time.time() + timeout
        while True:
            job = self.get_job(job_id)
            if job.get("status") in ("completed", "failed", "cancelled", "timeout"):
                return job
            if time.time() >= deadline:
                raise TimeoutError(f"job {job_id} not finished within {timeout}s")
            time.sleep(poll_interval)

    # ------------------------------------------------------------------ direct mode
    def _get_nearest_worker(self, job_type: str) -> Dict[str, Any]:
        key = f"direct_{job_type}"
        hit = self._direct_worker_cache.get(key)
        if hit is not None and time.time() - hit["cached_at"] < DIRECT_CACHE_TTL_S:
            return hit["worker"]
        w = self._request_with_fallback("GET", f"/api/v1/jobs/direct/nearest?job_type={job_type}",
                                        headers=self._headers()).json()
        self._direct_worker_cache[key] = {"worker": w, "cached_at": time.time()}
        return w

    def _direct_inference(self, job_type: str, params: Dict[str, Any]) -> Dict[str, Any]:
        w = self._get_nearest_worker(job_type)
        logger.info("direct inference via %s (%s)", w.get("direct_url"), w.get("region"))
        r = self.client.post(f"{w['direct_url'].rstrip('/')}/inference", json={"type": job_type, "params": params},
                             timeout=self.timeout)
        r.raise_for_status()
        return r.json()

    # ------------------------------------------------------------------ info
    def get_queue_stats(self, region: Optional[str] = None) -> Dict[str, Any]:
        path = "/api/v1/jobs/stats/queue" + (f"?region={region}" if region else "")
        return self._request_with_fallback("GET", path, headers=self._headers()).json()

    def list_workers(self, region: Optional[str] = None, status: Optional[str] = None) -> List[Dict[str, Any]]:
        q = "&".join(f"{k}={v}" for k, v in (("region", region), ("status", status)) if v)
        return self._request_with_fallback("GET", "/api/v1/workers" + (f"?{q}" if q else ""),
                                           headers=self._headers()).json()

    def close(self) -> None:
        self.client.close()

    def __enter__(self) -> "InferenceClient":
        return self

    def __exit__(self, *exc) -> None:
        self.close()


def chat(message: str, base_url: str = "http://localhost:8000", **kwargs) -> str:
    with InferenceClient(base_url) as c:
        out = c.chat([{"role": "user", "content": message}], **kwargs)
    return ((out.get("result") or {}).get("response")) or ""


def generate_image(prompt: str, base_url: str = "http://localhost:8000", **kwargs) -> Dict[str, Any]:
    with InferenceClient(base_url) as c:
        return c.generate_image(prompt, **kwargs)
