"""Engine registry (API-compatible with reference worker/engines/__init__.py:51-193).

Registered engines:
  llm          HF Transformers (CPU / portable path)
  llm_native   dgi MI355X-native runtime (alias: ``mi355x``, ``dgi``)
  llm_node     dgi node server (whole-node P/D + pipeline; alias ``mi355x-node``)
  image_gen    diffusers pipeline (lazy dependency)
  vision       HF vision-language model (lazy dependency)
Lazy optional adapters (external servers, never required):
  llm_sglang, llm_vllm, llm_vllm_async
"""
from __future__ import annotations

from typing import Any, Dict

from .base import BaseEngine
from .image_gen import ImageGenEngine
from .llm import LLMEngine
from .llm_base import GenerationConfig, GenerationResult, LLMBackend, LLMBaseEngine
from .llm_native import NativeLLMEngine
from .llm_node import NodeLLMEngine
from .vision import VisionEngine


def _get_sglang_engine():
    from .llm_sglang import SGLangEngine
    return SGLangEngine


def _get_vllm_engine():
    from .llm_vllm import VLLMEngine
    return VLLMEngine


def _get_vllm_async_engine():
    from .llm_vllm import VLLMAsyncEngine
    return VLLMAsyncEngine


ENGINE_REGISTRY: Dict[str, type] = {
    "llm": LLMEngine,
    "llm_native": NativeLLMEngine,
    "llm_node": NodeLLMEngine,
    "image_gen": ImageGenEngine,
    "vision": VisionEngine,
}

_LAZY_ENGINES = {
    "llm_sglang": _get_sglang_engine,
    "llm_vllm": _get_vllm_engine,
    "llm_vllm_async": _get_vllm_async_engine,
}

_BACKEND_ALIASES = {
    "native": "llm",
    "transformers": "llm",
    "mi355x": "llm_native",
    "dgi": "llm_native",
    "mi355x-node": "llm_node",
    "node": "llm_node",
    "sglang": "llm_sglang",
    "vllm": "llm_vllm",
    "vllm_async": "llm_vllm_async",
}


def get_engine(engine_type: str) -> type:
    name = _BACKEND_ALIASES.get(engine_type, engine_type)
    if name in ENGINE_REGISTRY:
        return ENGINE_REGISTRY[name]
    if name in _LAZY_ENGINES:
        try:
            cls = _LAZY_ENGINES[name]()
        except ImportError as e:
            raise ImportError(f"Engine '{name}' requires additional dependencies: {e}")
        ENGINE_REGISTRY[name] = cls
        return cls
    raise ValueError(f"Unknown engine type: {engine_type}")


def create_llm_engine(config: Dict[str, Any]) -> LLMBaseEngine:
    backend = str(config.get("backend", "native")).lower()
    name = _BACKEND_ALIASES.get(backend, backend)
    if not name.startswith("llm"):
        raise ValueError(f"'{backend}' is not a valid LLM backend")
    return get_engine(name)(config)


def list_engines() -> dict:
    out = {name: {"available": True, "loaded": True} for name in ENGINE_REGISTRY}
    for name, loader in _LAZY_ENGINES.items():
        if name in out:
            continue
        try:
            loader()
            out[name] = {"available": True, "loaded": False}
        except ImportError as e:
            out[name] = {"available": False, "error": str(e)}
    return out


def native_gpu_available() -> bool:
    try:
        import torch
        if not torch.cuda.is_available():
            return False
        from dgi import ops
        return ops.native_available()
    except Exception:
        return False


def get_recommended_backend() -> str:
    """MI355X native runtime when a GPU + built kernels are present, else HF native."""
    if native_gpu_available():
        return "mi355x"
    return "native"


__all__ = ["BaseEngine", "LLMBaseEngine", "LLMBackend", "GenerationConfig", "GenerationResult", "LLMEngine",
           "NativeLLMEngine", "NodeLLMEngine", "ImageGenEngine", "VisionEngine", "ENGINE_REGISTRY", "get_engine",
           "create_llm_engine", "list_engines", "get_recommended_backend"]
