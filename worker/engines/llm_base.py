"""LLM engine contract (compatible with reference worker/engines/llm_base.py:16-216).

Async generation, batch generation, default streaming, and a sync
``inference(params)`` bridge returning the job-result dict
``{"response", "usage": {prompt,completion,total,cached}, "finish_reason"}``.
The bridge reuses ONE background event-loop thread instead of spawning a
thread per call when invoked from inside a running loop.
"""
from __future__ import annotations

import asyncio
import logging
import threading
from abc import abstractmethod
from dataclasses import dataclass
from enum import Enum
from typing import Any, AsyncIterator, Dict, List, Optional

from .base import BaseEngine

logger = logging.getLogger(__name__)


class LLMBackend(Enum):
    NATIVE = "native"
    SGLANG = "sglang"
    VLLM = "vllm"
    NATIVE_MI355X = "mi355x"


@dataclass
class GenerationConfig:
    max_tokens: int = 2048
    temperature: float = 0.7
    top_p: float = 0.9
    top_k: int = 50
    stop_sequences: Optional[List[str]] = None
    stream: bool = False


@dataclass
class GenerationResult:
    text: str
    prompt_tokens: int
    completion_tokens: int
    total_tokens: int
    finish_reason: str = "stop"
    cached_tokens: int = 0


class _LoopThread:
    """A lazily started daemon thread owning one asyncio loop."""

    _lock = threading.Lock()
    _loop: Optional[asyncio.AbstractEventLoop] = None

    @classmethod
    def run(cls, coro):
        with cls._lock:
            if cls._loop is None or cls._loop.is_closed():
                loop = asyncio.new_event_loop()
                t = threading.Thread(target=loop.run_forever, name="llm-sync-bridge", daemon=True)
                t.start()
                cls._loop = loop
        return asyncio.run_coroutine_threadsafe(coro, cls._loop).result()


def generation_config_from_params(params: Dict[str, Any]) -> GenerationConfig:
    return GenerationConfig(max_tokens=params.get("max_tokens", 2048), temperature=params.get("temperature", 0.7),
                            top_p=params.get("top_p", 0.9), top_k=params.get("top_k", 50),
                            stop_sequences=params.get("stop", None), stream=params.get("stream", False))


def result_to_response(result: GenerationResult) -> Dict[str, Any]:
    return {
        "response": result.text,
        "usage": {"prompt_tokens": result.prompt_tokens, "completion_tokens": result.completion_tokens,
                  "total_tokens": result.total_tokens, "cached_tokens": result.cached_tokens},
        "finish_reason": result.finish_reason,
    }


class LLMBaseEngine(BaseEngine):
    def __init__(self, config: Dict[str, Any]):
        super().__init__(config)
        self.backend_type: LLMBackend = LLMBackend.NATIVE
        self.tokenizer = None
        self._batch_processor = None

    @abstractmethod
    async def generate_async(self, messages: List[Dict[str, str]],
                             config: Optional[GenerationConfig] = None) -> GenerationResult: ...

    @abstractmethod
    async def batch_generate(self, batch_messages: List[List[Dict[str, str]]],
                             config: Optional[GenerationConfig] = None) -> List[GenerationResult]: ...

    async def stream_generate(self, messages: List[Dict[str, str]],
                              config: Optional[GenerationConfig] = None) -> AsyncIterator[str]:
        result = await self.generate_async(messages, config)
        yield result.text

    @staticmethod
    def _run_coroutine_in_new_thread(coro):
        return _LoopThread.run(coro)

    @staticmethod
    def _messages_of(params: Dict[str, Any]) -> List[Dict[str, str]]:
        """Chat messages of a job; a bare ``prompt`` becomes one user turn."""
        if params.get("messages"):
            return params["messages"]
        if params.get("prompt") is not None:
            return [{"role": "user", "content": str(params["prompt"])}]
        return []

    def inference(self, params: Dict[str, Any]) -> Dict[str, Any]:
        messages = self._messages_of(params)
        cfg = generation_config_from_params(params)
        try:
            asyncio.get_running_loop()
        except RuntimeError:
            result = asyncio.run(self.generate_async(messages, cfg))
        else:
            result = self._run_coroutine_in_new_thread(self.generate_async(messages, cfg))
        return result_to_response(result)

    async def batch_inference_async(self, params_list: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
        """Fast path of the ContinuousBatcher (worker/batch_processor.py)."""
        if not params_list:
            return []
        cfg = generation_config_from_params(params_list[0])
        res = await self.batch_generate([self._messages_of(p) for p in params_list], cfg)
        return [result_to_response(r) for r in res]

    def supports_streaming(self) -> bool:
        return False

    def supports_prefix_caching(self) -> bool:
        return False

    def supports_batch_inference(self) -> bool:
        return False

    def get_backend_info(self) -> Dict[str, Any]:
        return {"backend": self.backend_type.value, "supports_streaming": self.supports_streaming(),
                "supports_prefix_caching": self.supports_prefix_caching(),
                "supports_batch_inference": self.supports_batch_inference()}

    def get_status(self) -> Dict[str, Any]:
        s = super().get_status()
        s["backend_info"] = self.get_backend_info()
        return s


def create_llm_engine(config: Dict[str, Any]) -> LLMBaseEngine:
    """Duplicate factory kept for API parity; delegates to the registry."""
    from . import create_llm_engine as _create
    return _create(config)
