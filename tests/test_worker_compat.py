"""Reference-surface tests for the worker package (engines registry, batcher,
KV facade, model shards, sessions, shard servers, proto wire format).

Behaviour pinned here follows the reference's own suite plus
the fixed defects listed in Appendix E."""
import asyncio
import time
import sys
import types
from unittest.mock import MagicMock, patch

import numpy as np
import pytest
import torch
import torch.nn as nn

from common.data_structures import SessionConfig, WorkerInfo, WorkerState
from common.serialization import TensorSerializer, serialize_tensor


# ---------------------------------------------------------------- engines
def test_registry_aliases_lazy_and_native():
    from engines import ENGINE_REGISTRY, LLMEngine, NativeLLMEngine, create_llm_engine, get_engine, list_engines
    from engines import get_recommended_backend
    assert get_engine("native") is LLMEngine and get_engine("transformers") is LLMEngine
    assert get_engine("mi355x") is NativeLLMEngine and ENGINE_REGISTRY["llm_native"] is NativeLLMEngine
    with pytest.raises(ValueError):
        get_engine("nope")
    with pytest.raises(ValueError):
        create_llm_engine({"backend": "image_gen"})
    eng = list_engines()
    assert eng["llm"]["available"] and "llm_sglang" in eng and "llm_vllm" in eng
    assert get_recommended_backend() in {"native", "mi355x", "sglang", "vllm", "vllm_async"}


def test_llm_base_sync_bridge_inside_and_outside_loop():
    from engines.llm_base import GenerationConfig, GenerationResult, LLMBaseEngine

    class E(LLMBaseEngine):
        def load_model(self):
            self.loaded = True

        def unload_model(self):
            self.loaded = False

        async def generate_async(self, messages, config=None):
            await asyncio.sleep(0)
            return GenerationResult("ok", 1, 2, 3, cached_tokens=1)

        async def batch_generate(self, batch_messages, config=None):
            return [await self.generate_async(m, config) for m in batch_messages]

    e = E({})
    out = e.inference({"messages": [{"role": "user", "content": "hi"}]})
    assert out == {"response": "ok", "usage": {"prompt_tokens": 1, "completion_tokens": 2, "total_tokens": 3,
                                               "cached_tokens": 1}, "finish_reason": "stop"}

    async def inside():
        return e.inference({"messages": []})
    assert asyncio.run(inside())["response"] == "ok"
    assert GenerationConfig().max_tokens == 2048 and GenerationConfig().top_k == 50
    assert e.get_backend_info()["supports_streaming"] is False


def test_native_engine_cpu_end_to_end_with_batcher():
    from batch_processor import ContinuousBatcher
    from engines import NativeLLMEngine
    eng = NativeLLMEngine({"model_id": "llama-tiny", "device": "cpu", "num_blocks": 128, "max_model_len": 512,
                           "max_num_seqs": 8})
    eng.load_model()
    try:
        async def run():
            b = ContinuousBatcher(eng, max_batch_size=4, max_wait_ms=5)
            await b.start()
            msgs = [{"role": "user", "content": f"hello {i}"} for i in range(3)]
            rs = await asyncio.gather(*[b.submit(f"j{i}", {"messages": [m], "max_tokens": 5, "temperature": 0})
                                        for i, m in enumerate(msgs)])
            chunks = [c async for c in eng.stream_generate([msgs[0]], __import__("engines").GenerationConfig(
                max_tokens=4, temperature=0))]
            await b.stop()
            return rs, chunks
        rs, chunks = asyncio.run(run())
        assert all(r["usage"]["completion_tokens"] == 5 for r in rs)
        assert isinstance("".join(chunks), str)
        st = eng.get_status()
        assert "radix_attention" in st["features"] and st["engine"]["finished"] >= 3
    finally:
        eng.unload_model()


def test_hf_llm_engine_opt125m_random_init_greedy_is_deterministic():
    """BASELINE config #1: OPT-125m greedy on CPU through engines/base (random init, no network)."""
    from engines import LLMEngine
    outs = []
    for _ in range(2):
        e = LLMEngine({"model_id": "facebook/opt-125m", "device": "cpu", "seed": 0})
        e.load_model()
        outs.append(e.inference({"messages": [{"role": "user", "content": "hi"}], "max_tokens": 4,
                                 "temperature": 0, "ignore_eos": True}))
        e.unload_model()
    assert outs[0]["tokens"] == outs[1]["tokens"] and outs[0]["usage"]["completion_tokens"] == 4


# ---------------------------------------------------------------- batcher
def test_batcher_prefix_hash_and_grouping():
    from batch_processor import ContinuousBatcher, PendingRequest, RequestPriority
    b = ContinuousBatcher(engine=object(), max_batch_size=4)
    assert b._compute_prefix_hash({"messages": [{"role": "user", "content": "x"}]}) == ""
    h = b._compute_prefix_hash({"messages": [{"role": "system", "content": "s"}]})
    assert len(h) == 16 and h == b._compute_prefix_hash({"messages": [{"role": "system", "content": "s"}]})
    reqs = []
    for jid, p in (("a1", "p1"), ("a2", "p1"), ("b1", "p2"), ("c1", "")):
        r = PendingRequest(RequestPriority.NORMAL.value, time.time(), jid, {}, MagicMock(), p)
        b._pending.append(r)
        if p:
            b._pending_by_prefix[p].append(r)
        reqs.append(r)
    batch = b._select_batch_with_prefix_grouping()
    assert batch[0].prefix_hash == "p1" and batch[1].prefix_hash == "p1" and len(batch) == 4


def test_batcher_flows():
    from batch_processor import AdaptiveBatcher, ContinuousBatcher

    class Async:
        async def batch_inference_async(self, ps):
            return [{"v": p.get("v")} for p in ps]

    class Sync:
        def batch_inference(self, ps):
            return [{"v": p.get("v")} for p in ps]

    class Err:
        async def batch_inference_async(self, ps):
            return [{"ok": True}, RuntimeError("boom")]

    class Slow:
        async def batch_inference_async(self, ps):
            await asyncio.sleep(0.2)
            return [{} for _ in ps]

    async def run():
        for eng in (Async(), Sync()):
            b = ContinuousBatcher(eng, max_batch_size=2, max_wait_ms=1, enable_prefix_grouping=False)
            await b.start()
            r = await asyncio.gather(b.submit("1", {"v": 1}, timeout=1), b.submit("2", {"v": 2}, timeout=1))
            assert [x["v"] for x in r] == [1, 2]
            await b.stop()
        b = ContinuousBatcher(Err(), max_batch_size=2, max_wait_ms=1)
        await b.start()
        t1 = asyncio.create_task(b.submit("1", {}, timeout=1))
        t2 = asyncio.create_task(b.submit("2", {}, timeout=1))
        assert (await t1)["ok"]
        with pytest.raises(RuntimeError):
            await t2
        await b.stop()
        b = ContinuousBatcher(Slow(), max_batch_size=10, max_wait_ms=1000)
        await b.start()
        with pytest.raises(asyncio.TimeoutError):
            await b.submit("1", {}, timeout=0.01)
        assert b.get_stats()["queue_size"] == 0
        await b.stop()
        b = ContinuousBatcher(Async(), max_queue_size=1, max_batch_size=10, max_wait_ms=1000)
        await b.start()
        t = asyncio.create_task(b.submit("1", {}, timeout=1))
        await asyncio.sleep(0)
        with pytest.raises(RuntimeError):
            await b.submit("2", {}, timeout=1)
        t.cancel()
        await b.stop()
        with pytest.raises(RuntimeError, match="not running"):
            await ContinuousBatcher(Async()).submit("x", {})
    asyncio.run(run())
    a = AdaptiveBatcher(engine=object(), min_batch_size=1, max_batch_size=10, target_latency_ms=100)
    a._current_batch_size, a._latency_history = 10, [200.0] * 10
    a._adapt_batch_size()
    assert a._current_batch_size < 10
    a._current_batch_size, a._latency_history = 5, [50.0] * 10
    a._adapt_batch_size()
    assert a._current_batch_size > 5


# ---------------------------------------------------------------- KV facade
def test_paged_kv_cache_cpu_alloc_free_evict():
    from distributed.kv_cache import CacheBlock, CacheLocation, KVCachePool, PagedKVCache
    c = PagedKVCache(4, 8, 64, 16, 3, device="cpu", dtype=torch.float32)
    b = c.allocate_block(0, "p")
    assert b is not None and b.prefix_hash == "p" and b.block_id in c._blocks and b.location == CacheLocation.CPU
    b.add_ref()
    c.free_block(b.block_id)
    assert b.block_id in c._blocks and b.ref_count == 1
    c.free_block(b.block_id)
    assert b.block_id not in c._blocks and b.block_id in c._free_blocks
    for _ in range(3):
        c.allocate_block(0)
    assert len(c._free_blocks) == 0
    assert c.allocate_block(0) is not None and c.get_stats()["evictions"] == 1
    assert c.get_block("missing") is None and c.get_stats()["misses"] == 1
    blk = CacheBlock("x", block_size=16, num_tokens=16)
    assert blk.is_full and not blk.is_shared
    pool = KVCachePool(4, 8, 64, 16, 2, device="cpu")
    assert all(len(lb) == 2 for lb in pool.allocate_sequence(32))
    with pytest.raises(RuntimeError, match="Failed to allocate"):
        pool.allocate_sequence(64)


def test_tiered_kv_manager_flow_and_redis():
    from distributed.kv_cache import DistributedKVCacheManager
    m = DistributedKVCacheManager(2, 4, 32, gpu_cache_blocks=5, cpu_cache_gb=0.001, device="cpu")
    assert m.compute_prefix_hash([1, 2, 300]) != m.compute_prefix_hash([1, 2, 301])
    calls = []

    async def compute():
        calls.append(1)
        return torch.randn(4, 16, 32), torch.randn(4, 16, 32)

    async def run():
        await m.get_or_compute("p", 0, compute)
        await m.get_or_compute("p", 0, compute)
        r = MagicMock()
        r.get = MagicMock(return_value=asyncio.sleep(0, result=None))
        mm = DistributedKVCacheManager(2, 4, 32, redis_client=None, device="cpu")
        assert await mm._get_from_redis("k") is None
    asyncio.run(run())
    assert len(calls) == 1 and m.get_stats()["l1_hits"] == 1 and m.get_stats()["misses"] == 1
    k, v = torch.randn(2, 3, 4).to(torch.bfloat16), torch.randn(2, 3, 4).to(torch.bfloat16)
    k2, v2 = m._deserialize_kv(m._serialize_kv(k, v))
    assert torch.equal(k, k2) and torch.equal(v, v2)
    m.cpu_cache_max_items = 2
    for i in range(4):
        m._add_to_cpu_cache(f"k{i}", k, v)
    assert list(m.cpu_cache) == ["k2", "k3"]


# ---------------------------------------------------------------- model shard
def test_model_shard_api_and_planning():
    from distributed.model_shard import (ModelShard, ShardedModelLoader, _create_device_map_for_layers,
                                         _get_embedding_module, _get_layer_module, _get_norm_module,
                                         get_layer_range_for_worker)
    s = ModelShard("m", 0, 10, device="cpu", dtype=torch.float32)
    assert s.get_memory_usage() == 0.0 and s.get_layer_count() == 0
    with pytest.raises(RuntimeError, match="only be called on the last shard"):
        s.get_logits(torch.randn(1, 2, 8))
    s.is_last_shard = True
    with pytest.raises(RuntimeError, match="No lm_head"):
        s.get_logits(torch.randn(1, 2, 8))
    s.lm_head = nn.Linear(8, 11)
    assert s.get_logits(torch.randn(1, 2, 8)).shape == (1, 2, 11)

    class Blk(nn.Module):
        def forward(self, h, **kw):
            return h + 1, (h, h)
    s2 = ModelShard("m", 0, 2, device="cpu")
    s2.layers.append(Blk())
    out, kv = s2.forward(torch.zeros(1, 3, 4), use_cache=True)
    assert torch.all(out == 1) and len(kv) == 1
    assert [get_layer_range_for_worker(10, 3, i) for i in range(3)] == [(0, 4), (4, 7), (7, 10)]
    assert get_layer_range_for_worker(5, 10, 9) == (5, 5)
    model = MagicMock()
    model.model.layers = nn.ModuleList([nn.Linear(2, 2)])
    assert _get_layer_module(model, None) is model.model.layers
    g = MagicMock()
    del g.model
    g.transformer.h = nn.ModuleList([nn.Linear(2, 2)])
    g.transformer.wte = nn.Embedding(4, 2)
    g.transformer.ln_f = nn.LayerNorm(2)
    assert _get_layer_module(g) is g.transformer.h and _get_embedding_module(g) is g.transformer.wte
    assert _get_norm_module(g) is g.transformer.ln_f
    d = _create_device_map_for_layers(None, 25, 32, "cuda:0", False, True)
    assert "model.embed_tokens" not in d and d["lm_head"] == "cuda:0" and "model.layers.24" not in d
    with patch("distributed.model_shard.AutoConfig") as ac:
        ac.from_pretrained.return_value = types.SimpleNamespace(num_hidden_layers=80, hidden_size=8192,
                                                                num_attention_heads=64, num_key_value_heads=8,
                                                                intermediate_size=28672, vocab_size=128256)
        ld = ShardedModelLoader("x")
        assert ld.analyze_model()["total_layers"] == 80
        plan = ld.create_shard_plan([192.0] * 2)
        assert plan[0][0] == 0 and plan[-1][1] == 80
        with pytest.raises(ValueError, match="Insufficient memory"):
            ld.create_shard_plan([8.0])


# ---------------------------------------------------------------- sessions
class _FakeWS:
    def __init__(self, worker_info, session_id=None):
        from distributed.session import SessionState
        self.worker_info, self.session_id, self.state = worker_info, "s", SessionState.INITIALIZING
        self.next_session, self.history, self.calls = None, [], 0

    async def connect(self, timeout=30.0):
        from distributed.session import SessionState
        self.state = SessionState.READY

    async def forward(self, h, position, kv_cache_keys=None, record=True):
        self.calls += 1
        if self.worker_info.worker_id == "dead":
            raise RuntimeError("down")
        self.history.append((h, position))
        return h, kv_cache_keys or []

    async def replay(self, history):
        self.history = list(history)

    async def close(self):
        from distributed.session import SessionState
        self.state = SessionState.CLOSED


def test_distributed_session_retry_failover_and_manager():
    from distributed.session import DistributedInferenceSession, SessionManager, SessionState
    cfg = SessionConfig(model_name="m", max_length=10, max_retries=2, connect_timeout=1.0)
    route = [WorkerInfo("w1", state=WorkerState.ONLINE, api_endpoint="http://a"),
             WorkerInfo("dead", state=WorkerState.ONLINE, api_endpoint="http://b")]

    async def run():
        with patch("distributed.session.WorkerSession", _FakeWS), \
                patch("distributed.session.asyncio.sleep", return_value=asyncio.sleep(0)):
            spare = WorkerInfo("spare", state=WorkerState.ONLINE, api_endpoint="http://c")
            s = DistributedInferenceSession(cfg, route, failover=lambda w: spare)
            await s.setup()
            out = await s.step(np.zeros((1, 2), np.float32))
            assert out.shape == (1, 2) and s.position == 2
            st = s.get_stats()
            assert st["failovers"] == 1 and st["retries"] >= 1 and s.route[1].worker_id == "spare"
            with pytest.raises(ValueError):
                await s.step(np.zeros((1, 9), np.float32))
            await s.close()
            assert s.state == SessionState.CLOSED
            s2 = DistributedInferenceSession(cfg, route[1:])
            await s2.setup()
            with pytest.raises(RuntimeError):
                await s2.step(np.zeros((1, 1), np.float32))
            mgr = SessionManager(max_sessions=1)
            a = await mgr.create_session(cfg, route[:1])
            a.state = SessionState.CLOSED
            assert await mgr.create_session(cfg, route[:1]) is not None
            await mgr.close_all()
    asyncio.run(run())


def test_worker_session_http_roundtrip_and_exit():
    from distributed.session import SessionState, WorkerSession

    class Resp:
        def __init__(self, status, js=None):
            self.status, self.js = status, js

        async def json(self):
            return self.js

        async def text(self):
            return "bad"

        async def __aenter__(self):
            return self

        async def __aexit__(self, *a):
            return False

    class Http:
        def __init__(self, fwd_status=200, result=None):
            self.fwd_status, self.result, self.closed = fwd_status, result, False

        def get(self, url):
            return Resp(200)

        def post(self, url, json=None):
            if url.endswith("/inference/forward"):
                return Resp(self.fwd_status, self.result)
            return Resp(200, {})

        async def close(self):
            self.closed = True

    hidden = np.arange(6, dtype=np.float32).reshape(2, 3)
    fake = Http(result={"output": serialize_tensor(hidden), "kv_cache_keys": ["k1"]})

    async def run():
        with patch("distributed.session.aiohttp.ClientSession", return_value=fake):
            ws = WorkerSession(WorkerInfo("w", state=WorkerState.ONLINE, api_endpoint="http://w"))
            await ws.connect()
            out, keys = await ws.forward(hidden, 5, ["x"])
            assert keys == ["k1"] and np.array_equal(np.asarray(out), hidden) and ws.position == 8
            await ws.close()
            assert ws.state == SessionState.CLOSED and fake.closed
        with patch("distributed.session.aiohttp.ClientSession", return_value=Http(fwd_status=500)):
            ws = WorkerSession(WorkerInfo("w", state=WorkerState.ONLINE, api_endpoint="http://w"))
            await ws.connect()
            with pytest.raises(RuntimeError):
                await ws.forward(np.zeros((1, 1), np.float32), 0)
            assert ws.state == SessionState.ERROR
    asyncio.run(run())
    n = {"c": 0}

    async def fake_close(self):
        n["c"] += 1
    ws = WorkerSession(WorkerInfo("w", state=WorkerState.ONLINE))
    ws.close = types.MethodType(fake_close, ws)
    ws.__exit__(None, None, None)

    async def inside():
        ws.__exit__(None, None, None)
    asyncio.run(inside())
    assert n["c"] == 2


# ---------------------------------------------------------------- shard servers / proto
def test_stateful_native_shard_chain_matches_engine_and_grpc_health():
    from distributed.grpc_server import GRPCServer, InferenceServicer
    from distributed.model_shard import ModelShard
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.sched.request import SamplingParams
    a = InferenceServicer(ModelShard.from_native("llama-tiny", 0, 1, device="cpu", num_blocks=64))
    b = InferenceServicer(ModelShard.from_native("llama-tiny", 1, 2, device="cpu", num_blocks=64))
    prompt = [1, 5, 9, 13, 17, 21, 25]

    async def run():
        x, pos, out = torch.tensor([prompt]), 0, []
        for _ in range(4):
            d, sh, dt = TensorSerializer.serialize(x)
            r0 = await a.Forward({"session_id": "s", "input": d, "shape": list(sh), "dtype": dt, "position": pos})
            r1 = await b.Forward({"session_id": "s", "input": r0["output"], "shape": r0["shape"],
                                  "dtype": r0["dtype"], "position": pos})
            lg = TensorSerializer.deserialize(r1["output"], tuple(r1["shape"]), r1["dtype"])
            out.append(int(lg[0, -1].float().argmax()))
            pos += x.shape[1]
            x = torch.tensor([[out[-1]]])
        assert (await b.CloseSession({"session_id": "s"}))["success"]
        srv = GRPCServer(a, "127.0.0.1", 0)
        await srv.start()
        import grpc
        from proto import inference_pb as pb
        ch = grpc.aio.insecure_channel(f"127.0.0.1:{srv.port}")
        hc = ch.unary_unary(f"/{pb.FULL_SERVICE}/HealthCheck", request_serializer=pb.HealthCheckRequest.SerializeToString,
                            response_deserializer=pb.HealthCheckResponse.FromString)
        healthy = (await hc(pb.HealthCheckRequest(include_stats=True))).healthy
        await ch.close()
        await srv.stop()
        return out, healthy
    out, healthy = asyncio.run(run())
    e = LLMEngine(EngineConfig(model="llama-tiny", device="cpu", num_blocks=64, max_model_len=256, max_num_seqs=4))
    ref = e.generate([prompt], SamplingParams(max_tokens=4, temperature=0, ignore_eos=True))[0].output
    assert out == ref and healthy


def test_proto_messages_roundtrip():
    from proto import inference_pb as pb
    r = pb.InferenceRequest(session_id="s", hidden_states=b"\x00\x01", shape=[1, 2, 3], position=7)
    r.metadata["k"] = "v"
    r2 = pb.InferenceRequest.FromString(r.SerializeToString())
    assert list(r2.shape) == [1, 2, 3] and r2.metadata["k"] == "v" and r2.position == 7
    kv = pb.KVCacheRequest(prefix_key="p", layers=[pb.KVCacheLayer(layer_idx=3, keys=b"k", values=b"v")])
    assert pb.KVCacheRequest.FromString(kv.SerializeToString()).layers[0].layer_idx == 3
    assert set(pb.METHODS) == {"StreamInference", "Forward", "TransferKVCache", "CreateSession", "CloseSession",
                               "HealthCheck"}


# ---------------------------------------------------------------- optional external-server adapters
def test_vllm_and_sglang_adapters_with_mocked_libraries():
    import asyncio
    from unittest.mock import MagicMock, patch
    mv = MagicMock()
    with patch.dict(sys.modules, {"vllm": mv, "sglang": MagicMock()}):
        from engines.llm_base import GenerationConfig, LLMBackend
        from engines.llm_sglang import SGLangEngine
        from engines.llm_vllm import VLLMAsyncEngine, VLLMEngine
        e = VLLMEngine({"model_id": "m", "vllm": {"tensor_parallel_size": 2, "enable_prefix_caching": True}})
        assert e.backend_type == LLMBackend.VLLM and e.llm is None and e._vllm_config["tensor_parallel_size"] == 2
        assert "assistant:" in e._format_messages([{"role": "user", "content": "hi"}])
        out = MagicMock()
        out.outputs = [MagicMock(text="ok", token_ids=[1, 2], finish_reason="stop")]
        out.prompt_token_ids = [5]
        e.llm = MagicMock()
        e.llm.generate.return_value = [out]
        r = e._generate_sync([{"role": "user", "content": "hi"}], GenerationConfig(max_tokens=4))
        assert (r.text, r.prompt_tokens, r.completion_tokens) == ("ok", 1, 2)
        assert len(asyncio.run(e.batch_generate([[{"role": "user", "content": "a"}]]))) == 1
        assert e.supports_prefix_caching() and not e.supports_streaming()
        assert "tensor_parallelism" in e.get_status()["features"]
        assert VLLMAsyncEngine({"model_id": "m"}).supports_streaming()
        s = SGLangEngine({"model_id": "m", "sglang": {"tp_size": 2}})
        assert s.runtime is None and s._server_process is None and s.get_cache_stats()["hit_rate"] == 0.0
        s._cache_hits, s._cache_misses = 10, 5
        assert s.get_cache_stats()["hit_rate"] == 10 / 15
        assert "radix_attention" in s.get_status()["features"]
        proc = MagicMock()
        s._server_process, s.loaded = proc, True
        s.unload_model()
        proc.terminate.assert_called_once()
        assert s._server_process is None and not s.loaded
    from engines import get_engine
    with patch.dict(sys.modules, {"vllm": mv}):
        assert get_engine("vllm").__name__ == "VLLMEngine"
