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

    async def _post(self, prompt: str, cfg: GenerationConfig) -> Dict[str, Any]:
        import httpx
        body = {"text": prompt, "sampling_params": {"max_new_tokens": cfg.max_tokens, "temperature": cfg.temperature,
                                                    "top_p": cfg.top_p, "top_k": cfg.top_k if cfg.top_k else -1,
                                                    "stop": cfg.stop_sequences}}
        async with httpx.AsyncClient(timeout=None) as c:
            r = await c.post(f"{self.server_url.rstrip('/')}/generate", json=body)
            r.raise_for_status()
            return r.json()

    async def generate_async(self, messages, config: Optional[GenerationConfig] = None) -> GenerationResult:
        cfg = config or GenerationConfig()
        d = await self._post(self._format_messages(messages), cfg)
        meta = d.get("meta_info", {}) or {}
        p, c = int(meta.get("prompt_tokens", 0)), int(meta.get("completion_tokens", 0))
        cached = int(meta.get("cached_tokens", 0))
        if cached:
            self._cache_hits += 1
        else:
            self._cache_misses += 1
        fr = meta.get("finish_reason")
        fr = fr.get("type") if isinstance(fr, dict) else (fr or "stop")
        return GenerationResult(text=d.get("text", ""), prompt_tokens=p, completion_tokens=c, total_tokens=p + c,
                                finish_reason=fr, cached_tokens=cached)

    async def batch_generate(self, batch_messages, config: Optional[GenerationConfig] = None) -> List[GenerationResult]:
        res = await asyncio.gather(*[self.generate_async(m, config) for m in batch_messages], return_exceptions=True)
        return [r if isinstance(r, GenerationResult) else
                GenerationResult(text="", prompt_tokens=0, completion_tokens=0, total_tokens=0, finish_reason="error")
                for r in res]

    async def stream_generate(self, messages, config: Optional[GenerationConfig] = None) -> AsyncIterator[str]:
        res = await self.generate_async(messages, config)
        yield res.text

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
