"""SGLang adapter (optional; reference worker/engines/llm_sglang.py).

Uses a running SGLang server (``sglang.server_url``, HTTP ``/generate``) or
starts ``sglang.Runtime`` in-process.  Never required on MI355X (the native
``llm_native`` / ``llm_node`` engines provide RadixAttention-style prefix
caching, chunked prefill and continuous batching themselves).
"""
from __future__ import annotations

import asyncio
from typing import Any, AsyncIterator, Dict, List, Optional

from ._chat import format_messages
from .llm_base import GenerationConfig, GenerationResult, LLMBackend, LLMBaseEngine


async def _request(req):
    """aiohttp's ``session.post()`` is both awaitable and an async context manager;
    accept either form (test doubles and wrapped sessions return a coroutine)."""
    if not hasattr(req, "__aenter__") and hasattr(req, "__await__"):
        return await req
    return req


class SGLangEngine(LLMBaseEngine):
    def __init__(self, config: Dict[str, Any]):
        super().__init__(config)
        self.backend_type = LLMBackend.SGLANG
        self.runtime = None
        self._server_process = None
        self._sglang_config = dict(config.get("sglang", {}) or {})
        self._cache_hits = 0
        self._cache_misses = 0

    @property
    def server_url(self) -> Optional[str]:
        return self._sglang_config.get("server_url")

    def load_model(self) -> None:
        if self.server_url:
            self.loaded = True
            return
        import sglang
        kw = {k: v for k, v in self._sglang_config.items()
              if k in ("tp_size", "mem_fraction_static", "chunked_prefill_size", "max_running_requests",
                       "context_length")}
        if self.config.get("quantization"):
            kw["quantization"] = self.config["quantization"]
        if not self._sglang_config.get("enable_prefix_caching", True):
            kw["disable_radix_cache"] = True
        self.runtime = sglang.Runtime(model_path=self.config["model_id"], **kw)
        self._sglang_config.setdefault("server_url", self.runtime.url)
        self.loaded = True

    def _format_messages(self, messages) -> str:
        return format_messages(self.tokenizer, messages)

    def _url(self) -> str:
        return (self.server_url or "http://localhost:30000").rstrip("/")

    async def _generate_with_native_api(self, messages, cfg: GenerationConfig) -> GenerationResult:
        """SGLang's own ``/generate`` route (carries ``cached_tokens`` in meta_info)."""
        import aiohttp
        body = {"text": self._format_messages(messages),
                "sampling_params": {"max_new_tokens": cfg.max_tokens, "temperature": cfg.temperature,
                                    "top_p": cfg.top_p, "top_k": cfg.top_k if cfg.top_k else -1,
                                    "stop": cfg.stop_sequences}}
        async with aiohttp.ClientSession() as session:
            async with session.post(f"{self._url()}/generate", json=body) as resp:
                if resp.status != 200:
                    raise RuntimeError(f"SGLang /generate error {resp.status}: {await resp.text()}")
                d = await resp.json()
        meta = d.get("meta_info", {}) or {}
        p, c = int(meta.get("prompt_tokens", 0)), int(meta.get("completion_tokens", 0))
        fr = meta.get("finish_reason")
        fr = fr.get("type") if isinstance(fr, dict) else (fr or "stop")
        return GenerationResult(text=d.get("text", ""), prompt_tokens=p, completion_tokens=c, total_tokens=p + c,
                                finish_reason=fr, cached_tokens=int(meta.get("cached_tokens", 0)))

    async def _generate_with_http_api(self, messages, cfg: GenerationConfig) -> GenerationResult:
        """OpenAI-compatible ``/v1/chat/completions`` (fallback route)."""
        import aiohttp
        payload = {"model": self.config.get("model_id"), "messages": messages, "max_tokens": cfg.max_tokens,
                   "temperature": cfg.temperature, "top_p": cfg.top_p}
        if cfg.stop_sequences:
            payload["stop"] = cfg.stop_sequences
        async with aiohttp.ClientSession() as session:
            async with await _request(session.post(f"{self._url()}/v1/chat/completions", json=payload)) as resp:
                if resp.status != 200:
                    raise RuntimeError(f"SGLang API error {resp.status}: {await resp.text()}")
                d = await resp.json()
        if "error" in d:
            raise RuntimeError(f"SGLang API error: {d['error']}")
        choice = (d.get("choices") or [{}])[0]
        usage = d.get("usage", {}) or {}
        return GenerationResult(text=(choice.get("message") or {}).get("content", ""),
                                prompt_tokens=int(usage.get("prompt_tokens", 0)),
                                completion_tokens=int(usage.get("completion_tokens", 0)),
                                total_tokens=int(usage.get("total_tokens", 0)),
                                finish_reason=choice.get("finish_reason") or "stop",
                                cached_tokens=int(usage.get("cached_tokens", 0)))

    async def generate_async(self, messages, config: Optional[GenerationConfig] = None) -> GenerationResult:
        cfg = config or GenerationConfig()
        try:
            res = await self._generate_with_native_api(messages, cfg)
        except Exception:
            res = await self._generate_with_http_api(messages, cfg)
        if res.cached_tokens:
            self._cache_hits += 1
        else:
            self._cache_misses += 1
        return res

    async def batch_generate(self, batch_messages, config: Optional[GenerationConfig] = None) -> List[GenerationResult]:
        res = await asyncio.gather(*[self.generate_async(m, config) for m in batch_messages], return_exceptions=True)
        return [r if isinstance(r, GenerationResult) else
                GenerationResult(text="", prompt_tokens=0, completion_tokens=0, total_tokens=0, finish_reason="error")
                for r in res]

    async def stream_generate(self, messages, config: Optional[GenerationConfig] = None) -> AsyncIterator[str]:
        """SSE stream of ``/generate`` (``stream: true``): yields text deltas."""
        import json

        import aiohttp
        cfg = config or GenerationConfig()
        body = {"text": self._format_messages(messages), "stream": True,
                "sampling_params": {"max_new_tokens": cfg.max_tokens, "temperature": cfg.temperature,
                                    "top_p": cfg.top_p, "stop": cfg.stop_sequences}}
        sent = ""
        async with aiohttp.ClientSession() as session:
            async with session.post(f"{self._url()}/generate", json=body) as resp:
                if resp.status != 200:
                    raise RuntimeError(f"SGLang stream error {resp.status}: {await resp.text()}")
                async for raw in resp.content:
                    line = raw.decode("utf-8", "ignore").strip()
                    if not line.startswith("data:"):
                        continue
                    data = line[5:].strip()
                    if data == "[DONE]":
                        break
                    text = json.loads(data).get("text", "")
                    if len(text) > len(sent):   # SGLang streams the cumulative text
                        yield text[len(sent):]
                        sent = text

    def supports_streaming(self) -> bool:
        return True

    def supports_prefix_caching(self) -> bool:
        return bool(self._sglang_config.get("enable_prefix_caching", True))

    def supports_batch_inference(self) -> bool:
        return True

    def get_cache_stats(self) -> Dict[str, Any]:
        n = self._cache_hits + self._cache_misses
        return {"hits": self._cache_hits, "misses": self._cache_misses, "hit_rate": self._cache_hits / n if n else 0.0}

    def get_status(self) -> Dict[str, Any]:
        s = super().get_status()
        s.update(backend="sglang", cache_stats=self.get_cache_stats(),
                 features=["paged_attention", "radix_attention", "continuous_batching", "chunked_prefill"])
        return s

    def unload_model(self) -> None:
        if self.runtime is not None:
            try:
                self.runtime.shutdown()
            except Exception:
                pass
            self.runtime = None
        if self._server_process is not None:
            self._server_process.terminate()
            self._server_process = None
        self.loaded = False
