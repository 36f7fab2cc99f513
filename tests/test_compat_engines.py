"""Worker engine layer: base contracts, registry and the optional adapters.

Behavioural parity with the reference's tests/test_worker_engines_*.py and
worker/tests/test_llm_base_inference_event_loop.py: BaseEngine status,
LLMBaseEngine sync bridge (inside and outside a running loop), default
streaming and backend info; registry aliases / lazy entries / recommended
backend; SGLang and vLLM adapters driven against mocked libraries and a
mocked aiohttp session.  The engines are imported flat (``engines.*`` with
worker/ on sys.path) as the reference suite does.
"""
import asyncio
import sys
from typing import Dict, List, Optional
from unittest.mock import AsyncMock, MagicMock, patch

import pytest

from engines import (ENGINE_REGISTRY, LLMEngine, create_llm_engine, get_engine, get_recommended_backend,
                     list_engines)
from engines.base import BaseEngine
from engines.llm_base import GenerationConfig, GenerationResult, LLMBackend, LLMBaseEngine


def _ok(text="ok", p=1, c=1, reason="stop"):
    return GenerationResult(text=text, prompt_tokens=p, completion_tokens=c, total_tokens=p + c, finish_reason=reason)


class _Base(BaseEngine):
    def load_model(self):
        self.loaded = True

    def inference(self, params):
        return {"ok": True}

    def unload_model(self):
        self.loaded = False


class _LLM(LLMBaseEngine):
    def load_model(self):
        self.loaded = True

    def unload_model(self):
        self.loaded = False

    async def generate_async(self, messages, config: Optional[GenerationConfig] = None):
        await asyncio.sleep(0)
        return _ok(text="echo:" + messages[-1]["content"], p=3, c=2)

    async def batch_generate(self, batch_messages, config=None):
        return [await self.generate_async(m, config) for m in batch_messages]


# ----------------------------------------------------------------------------- base contracts

def test_base_status_keys():
    s = _Base(config={}).get_status()
    assert {"loaded", "device"} <= set(s)


def test_sync_bridge_outside_loop_returns_job_dict():
    out = _LLM(config={}).inference({"messages": [{"role": "user", "content": "hi"}]})
    assert out["response"] == "echo:hi"
    assert out["usage"] == {"prompt_tokens": 3, "completion_tokens": 2, "total_tokens": 5, "cached_tokens": 0}
    assert out["finish_reason"] == "stop"


def test_sync_bridge_inside_running_loop():
    eng = _LLM(config={})

    async def call():
        return eng.inference({"messages": [{"role": "user", "content": "in-loop"}]})

    assert asyncio.run(call())["response"] == "echo:in-loop"


def test_sync_bridge_accepts_prompt_only_params():
    out = _LLM(config={}).inference({"prompt": "plain"})
    assert out["response"] == "echo:plain"


def test_default_stream_yields_whole_text():
    async def run():
        return [c async for c in _LLM(config={}).stream_generate([{"role": "user", "content": "s"}])]

    assert asyncio.run(run()) == ["echo:s"]


def test_backend_info_defaults():
    e = _LLM(config={})
    info = e.get_backend_info()
    assert info["backend"] == e.backend_type.value and info["supports_streaming"] is False


def test_generation_dataclass_defaults():
    c = GenerationConfig()
    assert (c.max_tokens, c.temperature, c.top_p, c.top_k, c.stop_sequences, c.stream) == (2048, 0.7, 0.9, 50,
                                                                                            None, False)
    r = GenerationResult(text="t", prompt_tokens=1, completion_tokens=1, total_tokens=2)
    assert r.finish_reason == "stop" and r.cached_tokens == 0
    assert LLMBackend.NATIVE_MI355X.value == "mi355x"


# ----------------------------------------------------------------------------- registry

@pytest.mark.parametrize("alias", ["native", "transformers", "llm"])
def test_registry_llm_aliases(alias):
    assert get_engine(alias) is ENGINE_REGISTRY["llm"] is LLMEngine


def test_registry_unknown_and_prefix_validation():
    with pytest.raises(ValueError):
        get_engine("does_not_exist")
    with pytest.raises(ValueError):
        create_llm_engine({"backend": "image_gen"})


def test_registry_lists_lazy_and_native_entries():
    eng = list_engines()
    assert eng["llm"]["available"] is True
    assert {"llm_sglang", "llm_vllm", "llm_native"} <= set(eng)


def test_registry_mi355x_alias_and_recommendation():
    from engines import NativeLLMEngine
    assert get_engine("mi355x") is NativeLLMEngine
    assert get_recommended_backend() in {"native", "sglang", "vllm", "vllm_async"}


# ----------------------------------------------------------------------------- SGLang adapter

@pytest.fixture
def sglang_cls():
    with patch.dict(sys.modules, {"sglang": MagicMock()}):
        sys.modules.pop("engines.llm_sglang", None)
        from engines.llm_sglang import SGLangEngine
        yield SGLangEngine


def test_sglang_init(sglang_cls):
    e = sglang_cls({"model_id": "m", "quantization": "int8",
                    "sglang": {"tp_size": 2, "mem_fraction_static": 0.9, "enable_prefix_caching": True}})
    assert e.backend_type is LLMBackend.SGLANG and e.runtime is None and e._server_process is None
    assert (e._cache_hits, e._cache_misses) == (0, 0)
    assert e._sglang_config["tp_size"] == 2 and e.config["quantization"] == "int8"


def _mock_aiohttp_post(payload, status=200):
    resp = MagicMock()
    resp.status = status
    resp.json = AsyncMock(return_value=payload)
    resp.text = AsyncMock(return_value="err")
    ctx = MagicMock()
    ctx.__aenter__ = AsyncMock(return_value=resp)
    ctx.__aexit__ = AsyncMock(return_value=None)
    session = MagicMock()
    session.post = MagicMock(return_value=ctx)
    sctx = MagicMock()
    sctx.__aenter__ = AsyncMock(return_value=session)
    sctx.__aexit__ = AsyncMock(return_value=None)
    return sctx, session


async def test_sglang_openai_http_route(sglang_cls):
    e = sglang_cls({"model_id": "m", "sglang": {"server_url": "http://h:30000"}})
    sctx, session = _mock_aiohttp_post({"choices": [{"message": {"content": "Hello!"}, "finish_reason": "stop"}],
                                        "usage": {"prompt_tokens": 10, "completion_tokens": 8, "total_tokens": 18}})
    with patch("aiohttp.ClientSession", return_value=sctx):
        r = await e._generate_with_http_api([{"role": "user", "content": "Hi"}], GenerationConfig(max_tokens=100))
    assert (r.text, r.prompt_tokens, r.completion_tokens, r.finish_reason) == ("Hello!", 10, 8, "stop")
    url, kw = session.post.call_args[0][0], session.post.call_args[1]
    assert url == "http://h:30000/v1/chat/completions" and kw["json"]["max_tokens"] == 100


async def test_sglang_native_route_counts_cache_hits(sglang_cls):
    e = sglang_cls({"model_id": "m", "sglang": {"server_url": "http://h:1"}})
    sctx, session = _mock_aiohttp_post({"text": "hey", "meta_info": {"prompt_tokens": 4, "completion_tokens": 2,
                                                                     "cached_tokens": 3,
                                                                     "finish_reason": {"type": "length"}}})
    with patch("aiohttp.ClientSession", return_value=sctx):
        r = await e.generate_async([{"role": "user", "content": "x"}])
    assert (r.text, r.cached_tokens, r.finish_reason, r.total_tokens) == ("hey", 3, "length", 6)
    assert session.post.call_args[0][0] == "http://h:1/generate"
    assert e.get_cache_stats()["hits"] == 1


async def test_sglang_falls_back_to_openai_route(sglang_cls):
    e = sglang_cls({"model_id": "m"})
    e._generate_with_native_api = AsyncMock(side_effect=RuntimeError("no native"))
    e._generate_with_http_api = AsyncMock(return_value=_ok("fallback"))
    assert (await e.generate_async([{"role": "user", "content": "x"}])).text == "fallback"
    assert e.get_cache_stats()["misses"] == 1


async def test_sglang_batch_isolates_errors(sglang_cls):
    e = sglang_cls({"model_id": "m"})

    async def gen(messages, config=None):
        if "error" in str(messages):
            raise RuntimeError("boom")
        return _ok("OK")

    e.generate_async = gen
    res = await e.batch_generate([[{"role": "user", "content": "a"}], [{"role": "user", "content": "error"}],
                                  [{"role": "user", "content": "b"}]])
    assert [r.text for r in res] == ["OK", "", "OK"] and res[1].finish_reason == "error"


def test_sglang_features_cache_status_unload(sglang_cls):
    e = sglang_cls({"model_id": "m", "sglang": {"enable_prefix_caching": False}})
    assert e.supports_streaming() and e.supports_batch_inference() and not e.supports_prefix_caching()
    assert e.get_cache_stats() == {"hits": 0, "misses": 0, "hit_rate": 0.0}
    e._cache_hits, e._cache_misses = 10, 5
    assert e.get_cache_stats()["hit_rate"] == pytest.approx(10 / 15)
    st = e.get_status()
    assert {"paged_attention", "radix_attention", "continuous_batching"} <= set(st["features"])
    assert "cache_stats" in st
    rt, proc = MagicMock(), MagicMock()
    e.runtime, e._server_process, e.loaded = rt, proc, True
    e.unload_model()
    rt.shutdown.assert_called_once()
    proc.terminate.assert_called_once()
    assert e.runtime is None and e._server_process is None and not e.loaded


# ----------------------------------------------------------------------------- vLLM adapters

@pytest.fixture
def vllm_mod():
    mv = MagicMock()
    with patch.dict(sys.modules, {"vllm": mv}):
        sys.modules.pop("engines.llm_vllm", None)
        import engines.llm_vllm as mod
        yield mod, mv


def _vllm_out(text, prompt_ids, out_ids, reason="stop"):
    o = MagicMock()
    o.outputs = [MagicMock(text=text, token_ids=out_ids, finish_reason=reason)]
    o.prompt_token_ids = prompt_ids
    return o


def test_vllm_init(vllm_mod):
    mod, _ = vllm_mod
    e = mod.VLLMEngine({"model_id": "m", "vllm": {"tensor_parallel_size": 2, "gpu_memory_utilization": 0.9,
                                                  "max_model_len": 4096}})
    assert e.backend_type is LLMBackend.VLLM and e.llm is None and e._default_sampling_params is None
    assert e._vllm_config["max_model_len"] == 4096


def test_vllm_message_formatting(vllm_mod):
    mod, _ = vllm_mod
    e = mod.VLLMEngine({"model_id": "m"})
    e.tokenizer = None
    s = e._format_messages([{"role": "system", "content": "Be brief."}, {"role": "user", "content": "Hello"}])
    assert "system: Be brief." in s and "user: Hello" in s and s.rstrip().endswith("assistant:")
    tok = MagicMock()
    tok.apply_chat_template.return_value = "<|im_start|>user\nHello<|im_end|>"
    e.tokenizer = tok
    assert "<|im_start|>" in e._format_messages([{"role": "user", "content": "Hello"}])
    tok.apply_chat_template.assert_called_once()


def test_vllm_sync_generate_maps_output(vllm_mod):
    mod, mv = vllm_mod
    e = mod.VLLMEngine({"model_id": "m"})
    e.tokenizer = None
    e.llm = MagicMock()
    e.llm.generate.return_value = [_vllm_out("Generated", [1, 2, 3], [4, 5, 6, 7, 8])]
    r = e._generate_sync([{"role": "user", "content": "Hello"}], GenerationConfig(max_tokens=100, temperature=0.8))
    assert (r.text, r.prompt_tokens, r.completion_tokens, r.total_tokens) == ("Generated", 3, 5, 8)
    kw = mv.SamplingParams.call_args.kwargs
    assert kw["max_tokens"] == 100 and kw["temperature"] == 0.8


async def test_vllm_async_wrappers(vllm_mod):
    mod, _ = vllm_mod
    e = mod.VLLMEngine({"model_id": "m"})
    e.tokenizer = None
    e._generate_sync = MagicMock(return_value=_ok("Hello!"))
    assert (await e.generate_async([{"role": "user", "content": "x"}])).text == "Hello!"
    e.llm = MagicMock()
    e.llm.generate.return_value = [_vllm_out(f"R{i}", [1, 2], [3, 4, 5]) for i in range(3)]
    res = await e.batch_generate([[{"role": "user", "content": str(i)}] for i in range(3)])
    assert [r.text for r in res] == ["R0", "R1", "R2"]
    assert len(e.llm.generate.call_args[0][0]) == 3       # one batched call


def test_vllm_features_and_unload(vllm_mod):
    mod, _ = vllm_mod
    e = mod.VLLMEngine({"model_id": "m", "vllm": {"enable_prefix_caching": True}})
    assert not e.supports_streaming() and e.supports_prefix_caching() and e.supports_batch_inference()
    assert {"paged_attention", "continuous_batching", "tensor_parallelism"} <= set(e.get_status()["features"])
    e.llm, e.tokenizer, e._default_sampling_params, e.loaded = MagicMock(), MagicMock(), MagicMock(), True
    with patch("torch.cuda.is_available", return_value=False):
        e.unload_model()
    assert e.llm is None and e.tokenizer is None and e._default_sampling_params is None and not e.loaded


def test_vllm_async_engine_surface(vllm_mod):
    mod, _ = vllm_mod
    e = mod.VLLMAsyncEngine({"model_id": "m", "vllm": {"tensor_parallel_size": 4, "enable_prefix_caching": True}})
    assert e.backend_type is LLMBackend.VLLM and e.engine is None and e._vllm_config["tensor_parallel_size"] == 4
    assert e.supports_streaming() and e.supports_prefix_caching() and e.supports_batch_inference()
    st = e.get_status()
    assert st["async_mode"] is True and {"async_inference", "streaming"} <= set(st["features"])
    e.tokenizer = None
    s = e._format_messages([{"role": "user", "content": "What is AI?"}, {"role": "assistant", "content": "AI is..."}])
    assert "user: What is AI?" in s and "assistant: AI is..." in s
    e.engine, e.tokenizer, e.loaded = MagicMock(), MagicMock(), True
    with patch("torch.cuda.is_available", return_value=False):
        e.unload_model()
    assert e.engine is None and e.tokenizer is None and not e.loaded


async def test_vllm_async_batch_isolates_errors(vllm_mod):
    mod, _ = vllm_mod
    e = mod.VLLMAsyncEngine({"model_id": "m"})
    n = {"c": 0}

    async def gen(messages, config=None):
        n["c"] += 1
        if n["c"] == 2:
            raise RuntimeError("x")
        return _ok("OK")

    e.generate_async = gen
    res = await e.batch_generate([[{"role": "user", "content": str(i)}] for i in range(3)])
    assert [r.text for r in res] == ["OK", "", "OK"] and res[1].finish_reason == "error"


async def test_vllm_async_streams_text_deltas(vllm_mod):
    mod, _ = vllm_mod
    e = mod.VLLMAsyncEngine({"model_id": "m"})
    e.tokenizer = None

    async def gen(prompt, sp, rid):
        for t in ("He", "Hell", "Hello"):
            yield _vllm_out(t, [1], [2])

    e.engine = MagicMock()
    e.engine.generate = gen
    chunks = [c async for c in e.stream_generate([{"role": "user", "content": "x"}])]
    assert chunks == ["He", "ll", "o"]
