"""Worker → control-plane HTTP client (reference worker/api_client.py:15-288).

Signed requests: ``X-Signature = HMAC-SHA256(secret, "METHOD:path:sha256(body):ts")``
over the exact JSON body sent (canonical ``sort_keys`` form, which is what
the server re-derives).  Retries 5xx / transport errors with exponential
backoff; 4xx surfaces immediately.
"""
from __future__ import annotations

import hashlib
import hmac
import json
import logging
import time
from typing import Any, Dict, List, Optional
from urllib.parse import urlsplit

import httpx

logger = logging.getLogger(__name__)


def _canon(payload: Any) -> str:
    return json.dumps(payload, sort_keys=True, separators=(",", ":"))


class APIClient:
    def __init__(self, base_url: str, token: Optional[str] = None, timeout: int = 30, max_retries: int = 3,
                 verify_ssl: bool = True):
        self.base_url = base_url.rstrip("/")
        self.token = token
        self.signing_secret: Optional[str] = None
        self.timeout = timeout
        self.max_retries = max_retries
        self.client = httpx.Client(timeout=timeout, verify=verify_ssl)
        self._batch_claim = True        # GET next-jobs until a server answers that it has none

    def set_credentials(self, token: str, signing_secret: Optional[str] = None) -> None:
        self.token = token
        self.signing_secret = signing_secret

    def _sign_request(self, method: str, path: str, body: Optional[str], timestamp: int) -> str:
        digest = hashlib.sha256((body or "").encode()).hexdigest()
        msg = f"{method.upper()}:{path}:{digest}:{timestamp}"
        return hmac.new(self.signing_secret.encode(), msg.encode(), hashlib.sha256).hexdigest()

    def _headers(self, body: Optional[str] = None, path: str = "", method: str = "POST") -> Dict[str, str]:
        h = {"Content-Type": "application/json"}
        if self.token:
            h["X-Worker-Token"] = self.token
        if self.signing_secret and body:
            ts = int(time.time())
            h["X-Timestamp"] = str(ts)
            h["X-Signature"] = self._sign_request(method, path, body, ts)
        return h

    def _request_with_retry(self, method: str, url: str, **kwargs) -> httpx.Response:
        err: Optional[Exception] = None
        for attempt in range(self.max_retries):
            try:
                r = self.client.request(method, url, **kwargs)
                r.raise_for_status()
                return r
            except httpx.HTTPStatusError as e:
                if 400 <= e.response.status_code < 500:
                    raise
                err = e
            except httpx.RequestError as e:
                err = e
            if attempt + 1 < self.max_retries:
                delay = 2 ** attempt
                logger.warning("request %s %s failed (%s); retry in %ss", method, url, err, delay)
                time.sleep(delay)
        raise err  # type: ignore[misc]

    def _post(self, path: str, payload: Optional[Dict[str, Any]] = None, params=None) -> httpx.Response:
        body = _canon(payload if payload is not None else {})
        url = f"{self.base_url}{path}"
        return self._request_with_retry("POST", url, content=body, params=params,
                                        headers=self._headers(body, urlsplit(url).path))

    # ----------------------------------------------------------------- endpoints
    def register(self, name: str, region: str, country: Optional[str] = None, city: Optional[str] = None,
                 timezone: Optional[str] = None, gpu_model: Optional[str] = None,
                 gpu_memory_gb: Optional[float] = None, gpu_count: int = 1, cpu_cores: Optional[int] = None,
                 ram_gb: Optional[float] = None, supported_types: Optional[List[str]] = None,
                 direct_url: Optional[str] = None, supports_direct: bool = False, **extra) -> Dict[str, Any]:
        payload = {"name": name, "region": region, "country": country, "city": city, "timezone": timezone,
                   "gpu_model": gpu_model, "gpu_memory_gb": gpu_memory_gb, "gpu_count": gpu_count,
                   "cpu_cores": cpu_cores, "ram_gb": ram_gb, "supported_types": supported_types or [],
                   "direct_url": direct_url, "supports_direct": supports_direct, **extra}
        data = self._post("/api/v1/workers/register", payload).json()
        self.set_credentials(data["token"], data.get("signing_secret"))
        return data

    def heartbeat(self, worker_id: str, status: str, current_job_id: Optional[str] = None,
                  gpu_memory_used_gb: Optional[float] = None, supported_types: Optional[List[str]] = None,
                  loaded_models: Optional[List[str]] = None, config_version: int = 0,
                  engine_stats: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        payload = {"status": status, "current_job_id": current_job_id, "gpu_memory_used_gb": gpu_memory_used_gb,
                   "supported_types": supported_types, "loaded_models": loaded_models,
                   "config_version": config_version}
        if engine_stats:
            payload["engine_stats"] = engine_stats
        return self._post(f"/api/v1/workers/{worker_id}/heartbeat", payload).json()

    def fetch_next_job(self, worker_id: str, wait: float = 0.0) -> Optional[Dict[str, Any]]:
        """The next job or None.  ``wait`` > 0 long-polls: the server holds the request until a
        job is queued or ``wait`` seconds pass (a server without long-poll answers at once)."""
        try:
            kw: Dict[str, Any] = {"headers": self._headers()}
            if wait > 0:
                kw["params"] = {"wait": wait}
                kw["timeout"] = max(float(self.timeout), wait + 10.0)
            r = self.client.get(f"{self.base_url}/api/v1/workers/{worker_id}/next-job", **kw)
        except httpx.RequestError as e:
            logger.warning("next-job failed: %s", e)
            return None
        if r.status_code in (204, 404):
            return None
        r.raise_for_status()
        data = r.json() if r.content else None
        return data or None

    def fetch_next_jobs(self, worker_id: str, max_jobs: int, wait: float = 0.0) -> List[Dict[str, Any]]:
        """Up to ``max_jobs`` jobs in one request (``GET next-jobs``, one claim transaction on the
        server).  A server without that endpoint (the reference's) answers 404/405: from then on
        this client falls back to ``fetch_next_job``."""
        if max_jobs <= 1 or not self._batch_claim:
            job = self.fetch_next_job(worker_id, wait)
            return [job] if job else []
        try:
            kw: Dict[str, Any] = {"headers": self._headers(), "params": {"max": int(max_jobs)}}
            if wait > 0:
                kw["params"]["wait"] = wait
                kw["timeout"] = max(float(self.timeout), wait + 10.0)
            r = self.client.get(f"{self.base_url}/api/v1/workers/{worker_id}/next-jobs", **kw)
        except httpx.RequestError as e:
            logger.warning("next-jobs failed: %s", e)
            return []
        if r.status_code in (404, 405):
            self._batch_claim = False
            job = self.fetch_next_job(worker_id, wait)
            return [job] if job else []
        if r.status_code == 204:
            return []
        r.raise_for_status()
        data = r.json() if r.content else None
        return list(data or [])

    def complete_job(self, worker_id: str, job_id: str, success: bool, result: Optional[Dict[str, Any]] = None,
                     error: Optional[str] = None, processing_time_ms: Optional[int] = None,
                     usage: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        payload = {"success": success, "result": result, "error": error, "processing_time_ms": processing_time_ms}
        if usage:
            payload["usage"] = usage
        return self._post(f"/api/v1/workers/{worker_id}/jobs/{job_id}/complete", payload).json()

    def notify_going_offline(self, worker_id: str, finish_current: bool = True) -> Dict[str, Any]:
        return self._post(f"/api/v1/workers/{worker_id}/going-offline", {},
                          params={"finish_current": str(finish_current).lower()}).json()

    def notify_offline(self, worker_id: str) -> Dict[str, Any]:
        try:
            return self._post(f"/api/v1/workers/{worker_id}/offline", {}).json()
        except Exception as e:
            logger.warning("offline notification failed: %s", e)
            return {"status": "error", "error": str(e)}

    def verify_credentials(self, worker_id: str, token: str) -> bool:
        try:
            r = self.client.post(f"{self.base_url}/api/v1/workers/{worker_id}/verify",
                                 headers={"X-Worker-Token": token, "Content-Type": "application/json"})
            return r.status_code == 200 and bool(r.json().get("valid"))
        except Exception:
            return False

    def get_config(self, worker_id: str) -> Optional[Dict[str, Any]]:
        try:
            r = self.client.get(f"{self.base_url}/api/v1/workers/{worker_id}/config", headers=self._headers())
        except Exception as e:
            logger.warning("config fetch failed: %s", e)
            return None
        if r.status_code != 200:
            return None
        return r.json()

    def refresh_token(self, worker_id: str, refresh_token: str) -> Optional[Dict[str, Any]]:
        try:
            r = self.client.post(f"{self.base_url}/api/v1/workers/{worker_id}/refresh-token",
                                 json={"refresh_token": refresh_token})
        except Exception as e:
            logger.warning("token refresh failed: %s", e)
            return None
        if r.status_code != 200:
            return None
        data = r.json()
        self.token = data["token"]
        return data

    def close(self) -> None:
        self.client.close()
