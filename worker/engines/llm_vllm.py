"""vLLM adapters (optional; reference worker/engines/llm_vllm.py).

Kept so deployments that already run vLLM can register it through the same
engine registry.  The MI355X path is ``llm_native`` / ``llm_node``; vLLM is
imported lazily and never required.  Config keys under ``vllm`` are passed
through (``tensor_parallel_size``, ``gpu_memory_utilization``,
``max_model_len``, ``max_num_seqs``, ``enable_prefix_caching``,
``enable_chunked_prefill``).
"""
from __future__ import annotations

import asyncio
import uuid
from typing import Any, AsyncIterator, Dict, List, Optional

from ._chat import format_messages
from .llm_base import GenerationConfig, GenerationResult, LLMBackend, LLMBaseEngine

_PASS = ("tensor_parallel_size", "gpu_memory_utilization", "max_model_len", "max_num_seqs", "enable_prefix_caching",
         "enable_chunked_prefill", "dtype", "quantization", "trust_remote_code", "swap_space")


def _sampling(cfg: GenerationConfig):
    from vllm import SamplingParams
    return SamplingParams(max_tokens=cfg.max_tokens, temperature=cfg.temperature, top_p=cfg.top_p,
                          top_k=cfg.top_k if cfg.top_k and cfg.top_k > 0 else -1, stop=cfg.stop_sequences)


def _free_device_memory() -> None:
    import torch
    if torch.cuda.is_available():
        torch.cuda.empty_cache()


def _result(out) -> GenerationResult:
    o = out.outputs[0]
    p = len(out.prompt_token_ids or [])
    c = len(o.token_ids or [])
    return GenerationResult(text=o.text, prompt_tokens=p, completion_tokens=c, total_tokens=p + c,
                            finish_reason=o.finish_reason or "stop")


class VLLMEngine(LLMBaseEngine):
    def __init__(self, config: Dict[str, Any]):
        super().__init__(config)
        self.backend_type = LLMBackend.VLLM
        self.llm = None
        self._default_sampling_params = None
        self._vllm_config = dict(config.get("vllm", {}) or {})

    def load_model(self) -> None:
        from vllm import LLM
        kw = {k: v for k, v in self._vllm_config.items() if k in _PASS}
        if self.config.get("quantization"):
            kw.setdefault("quantization", self.config["quantization"])
        self.llm = LLM(model=self.config["model_id"], **kw)
        self.tokenizer = self.llm.get_tokenizer()
        self.loaded = True

    def _format_messages(self, messages: List[Dict[str, str]]) -> str:
        return format_messages(self.tokenizer, messages)

    def _generate_sync(self, messages, cfg: GenerationConfig) -> GenerationResult:
        outs = self.llm.generate([self._format_messages(messages)], _sampling(cfg))
        return _result(outs[0])

    async def generate_async(self, messages, config: Optional[GenerationConfig] = None) -> GenerationResult:
        return await asyncio.to_thread(self._generate_sync, messages, config or GenerationConfig())

    async def batch_generate(self, batch_messages, config: Optional[GenerationConfig] = None) -> List[GenerationResult]:
        cfg = config or GenerationConfig()
        prompts = [self._format_messages(m) for m in batch_messages]
        outs = await asyncio.to_thread(self.llm.generate, prompts, _sampling(cfg))
        return [_result(o) for o in outs]

    def supports_streaming(self) -> bool:
        return False

    def supports_prefix_caching(self) -> bool:
        return bool(self._vllm_config.get("enable_prefix_caching", False))

    def supports_batch_inference(self) -> bool:
        return True

    def get_status(self) -> Dict[str, Any]:
        s = super().get_status()
        s.update(backend="vllm", features=["paged_attention", "continuous_batching", "tensor_parallelism"]
                 + (["prefix_caching"] if self.supports_prefix_caching() else []), vllm_config=self._vllm_config)
        return s

    def unload_model(self) -> None:
        self.llm = None
        self.tokenizer = None
        self._default_sampling_params = None
        self.loaded = False
        _free_device_memory()


class VLLMAsyncEngine(LLMBaseEngine):
    def __init__(self, config: Dict[str, Any]):
        super().__init__(config)
        self.backend_type = LLMBackend.VLLM
        self.engine = None
        self._vllm_config = dict(config.get("vllm", {}) or {})

    def load_model(self) -> None:
        from vllm import AsyncEngineArgs, AsyncLLMEngine
        kw = {k: v for k, v in self._vllm_config.items() if k in _PASS}
        self.engine = AsyncLLMEngine.from_engine_args(AsyncEngineArgs(model=self.config["model_id"], **kw))
        self.loaded = True

    def _format_messages(self, messages) -> str:
        return format_messages(self.tokenizer, messages)

    async def generate_async(self, messages, config: Optional[GenerationConfig] = None) -> GenerationResult:
        final = None
        async for out in self.engine.generate(self._format_messages(messages), _sampling(config or GenerationConfig()),
                                              uuid.uuid4().hex):
            final = out
        return _result(final)

    async def batch_generate(self, batch_messages, config: Optional[GenerationConfig] = None) -> List[GenerationResult]:
        res = await asyncio.gather(*[self.generate_async(m, config) for m in batch_messages], return_exceptions=True)
        return [r if isinstance(r, GenerationResult) else
                GenerationResult(text="", prompt_tokens=0, completion_tokens=0, total_tokens=0, finish_reason="error")
                for r in res]

    async def stream_generate(self, messages, config: Optional[GenerationConfig] = None) -> AsyncIterator[str]:
        prev = ""
        async for out in self.engine.generate(self._format_messages(messages), _sampling(config or GenerationConfig()),
                                              uuid.uuid4().hex):
            text = out.outputs[0].text
            if len(text) > len(prev):
                yield text[len(prev):]
                prev = text

    def supports_streaming(self) -> bool:
        return True

    def supports_prefix_caching(self) -> bool:
        return bool(self._vllm_config.get("enable_prefix_caching", False))

    def supports_batch_inference(self) -> bool:
        return True

    def get_status(self) -> Dict[str, Any]:
        s = super().get_status()
        s.update(backend="vllm_async", async_mode=True,
                 features=["paged_attention", "continuous_batching", "tensor_parallelism", "async_inference",
                           "streaming"] + (["prefix_caching"] if self.supports_prefix_caching() else []))
        return s

    def unload_model(self) -> None:
        self.engine = None
        self.tokenizer = None
        self.loaded = False
        _free_device_memory()
