"""Layer-range model shards (worker/distributed/model_shard.py).

Behavioural parity with the reference's
tests/test_worker_distributed_model_shard.py: LayerInfo, the ModelShard
facade (memory / layer count / logits guards, forward over stub layers with
and without cache), ShardedModelLoader planning with a patched module-level
``AutoConfig``, the even layer split (remainder to the first workers),
HF module-introspection helpers and device maps, and split coverage
invariants.  Native (dgi) shards and the MI355X-oriented splitter are
checked on CPU as well.
"""
from unittest.mock import MagicMock, patch

import pytest
import torch
import torch.nn as nn

from worker.distributed.model_shard import (LayerInfo, ModelShard, ShardedModelLoader, _create_device_map_for_layers,
                                            _get_embedding_module, _get_layer_module, _get_norm_module,
                                            get_layer_range_for_worker)
from dgi.parallel.plan import plan_layer_split


def _cfg(L=32, H=4096, nh=32, nkv=8, inter=14336):
    c = MagicMock()
    c.num_hidden_layers, c.hidden_size, c.num_attention_heads = L, H, nh
    c.num_key_value_heads, c.intermediate_size, c.vocab_size = nkv, inter, 128256
    return c


@pytest.fixture
def shard():
    return ModelShard(model_id="m", start_layer=0, end_layer=10, device="cpu", dtype=torch.float32)


@pytest.fixture
def stub_layer():
    layer = MagicMock()
    layer.return_value = (torch.randn(1, 6, 64), (torch.randn(1, 4, 6, 16), torch.randn(1, 4, 6, 16)))
    return layer


# ----------------------------------------------------------------------------- LayerInfo / ModelShard

def test_layer_info_fields():
    li = LayerInfo(layer_idx=3, layer_name="model.layers.3", param_count=10, memory_bytes=20)
    assert (li.layer_idx, li.layer_name, li.param_count, li.memory_bytes) == (3, "model.layers.3", 10, 20)


def test_shard_initial_state(shard):
    assert (shard.model_id, shard.start_layer, shard.end_layer, shard.device, shard.dtype) == \
        ("m", 0, 10, "cpu", torch.float32)
    assert len(shard.layers) == 0 and shard.config is None
    assert not shard.is_first_shard and not shard.is_last_shard


def test_shard_memory_and_layer_count(shard):
    assert shard.get_memory_usage() == 0.0 and shard.get_layer_count() == 0
    shard.layers.append(nn.Linear(256, 256))
    shard.layers.append(nn.Linear(256, 256))
    assert shard.get_layer_count() == 2
    expected = 2 * (256 * 256 + 256) * 4 / 1024 ** 3
    assert shard.get_memory_usage() == pytest.approx(expected)


def test_logits_guards_and_projection(shard):
    h = torch.randn(1, 4, 32)
    with pytest.raises(RuntimeError, match="only be called on the last shard"):
        shard.get_logits(h)
    shard.is_last_shard = True
    with pytest.raises(RuntimeError, match="No lm_head available"):
        shard.get_logits(h)
    shard.lm_head = nn.Linear(32, 100)
    assert shard.get_logits(h).shape == (1, 4, 100)


def test_forward_middle_shard_collects_kv(stub_layer):
    s = ModelShard("m", 5, 10, device="cpu")
    s.layers.append(stub_layer)
    s.layers.append(stub_layer)
    out, kv = s.forward(torch.randn(1, 6, 64), use_cache=True)
    assert stub_layer.call_count == 2 and out.shape == (1, 6, 64) and len(kv) == 2


def test_forward_first_shard_embeds_ids(stub_layer):
    s = ModelShard("m", 0, 5, device="cpu")
    s.is_first_shard = True
    s.embed_tokens = nn.Embedding(100, 64)
    s.layers.append(stub_layer)
    out, _ = s.forward(torch.randint(0, 100, (1, 6)), use_cache=True)
    passed = stub_layer.call_args[0][0]
    assert torch.is_floating_point(passed) and passed.shape == (1, 6, 64) and out is not None


def test_forward_last_shard_applies_norm():
    s = ModelShard("m", 25, 32, device="cpu")
    s.is_last_shard = True
    s.norm = nn.LayerNorm(64, elementwise_affine=False)
    layer = MagicMock(return_value=(torch.randn(2, 3, 64) * 5 + 3, None))
    s.layers.append(layer)
    out, _ = s.forward(torch.randn(2, 3, 64))
    assert out.mean(-1).abs().max() < 1e-4


def test_forward_without_cache_returns_none():
    s = ModelShard("m", 0, 5, device="cpu")
    s.layers.append(MagicMock(return_value=(torch.randn(1, 6, 64), None)))
    out, kv = s.forward(torch.randn(1, 6, 64), use_cache=False)
    assert out is not None and kv is None


def test_forward_passes_past_kv_per_layer(stub_layer):
    s = ModelShard("m", 0, 2, device="cpu")
    s.layers.append(stub_layer)
    s.layers.append(stub_layer)
    s.forward(torch.randn(1, 6, 64), past_key_values=["kv0", "kv1"])
    assert [c.kwargs["past_key_value"] for c in stub_layer.call_args_list] == ["kv0", "kv1"]


def test_native_shard_materialises_only_its_layers():
    s = ModelShard.from_native("llama-tiny", 1, 2, device="cpu", dtype=torch.float32, num_blocks=8)
    assert not s.is_first_shard and s.is_last_shard
    assert s.get_layer_count() == 1 and s.get_memory_usage() > 0
    full = ModelShard.from_native("llama-tiny", 0, 2, device="cpu", dtype=torch.float32, num_blocks=8)
    assert full.is_first_shard and full.get_memory_usage() > s.get_memory_usage()


# ----------------------------------------------------------------------------- loader

def test_loader_initial_state():
    ld = ShardedModelLoader(model_id="m")
    assert (ld.model_id, ld.config, ld.total_layers) == ("m", None, 0)


@patch("worker.distributed.model_shard.AutoConfig")
def test_analyze_model_reports_per_layer_memory(auto):
    auto.from_pretrained.return_value = _cfg()
    info = ShardedModelLoader("m").analyze_model()
    assert (info["model_id"], info["total_layers"], info["hidden_size"], info["num_attention_heads"]) == \
        ("m", 32, 4096, 32)
    # GQA attention + SwiGLU MLP in bf16: ~0.40 GiB per Llama-3-8B layer
    assert info["memory_per_layer_gb"] == pytest.approx(0.405, abs=0.01)


@patch("worker.distributed.model_shard.AutoConfig")
def test_shard_plan_covers_all_layers_in_order(auto):
    auto.from_pretrained.return_value = _cfg()
    plan = ShardedModelLoader("m").create_shard_plan([24.0, 24.0, 24.0], reserve_ratio=0.2)
    assert plan[0][0] == 0 and plan[-1][1] == 32
    assert all(a[1] == b[0] for a, b in zip(plan, plan[1:]))


@patch("worker.distributed.model_shard.AutoConfig")
def test_shard_plan_is_memory_proportional(auto):
    auto.from_pretrained.return_value = _cfg()
    plan = ShardedModelLoader("m").create_shard_plan([40.0, 20.0], reserve_ratio=0.0)
    sizes = [b - a for a, b in plan]
    assert sum(sizes) == 32 and sizes[0] > sizes[1]


@patch("worker.distributed.model_shard.AutoConfig")
def test_shard_plan_insufficient_memory(auto):
    auto.from_pretrained.return_value = _cfg(L=80, H=8192, nh=64, inter=28672)
    with pytest.raises(ValueError, match="Insufficient memory"):
        ShardedModelLoader("m").create_shard_plan([8.0], reserve_ratio=0.2)


@patch("worker.distributed.model_shard.AutoConfig")
def test_shard_plan_70b_on_mi355x_fits_one_gpu(auto):
    auto.from_pretrained.return_value = _cfg(L=80, H=8192, nh=64, inter=28672)
    assert ShardedModelLoader("m").create_shard_plan([288.0], reserve_ratio=0.2) == [(0, 80)]


# ----------------------------------------------------------------------------- even split

@pytest.mark.parametrize("L,W,expect", [
    (32, 4, [(0, 8), (8, 16), (16, 24), (24, 32)]),
    (10, 3, [(0, 4), (4, 7), (7, 10)]),
    (32, 1, [(0, 32)]),
    (5, 10, [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5)] + [(5, 5)] * 5),
])
def test_even_layer_split(L, W, expect):
    assert [get_layer_range_for_worker(L, W, i) for i in range(W)] == expect


@pytest.mark.parametrize("L,W", [(80, 5), (80, 3), (32, 7), (126, 8)])
def test_even_split_covers_each_layer_once(L, W):
    seen = []
    for i in range(W):
        a, b = get_layer_range_for_worker(L, W, i)
        seen += list(range(a, b))
    assert seen == list(range(L))


@pytest.mark.parametrize("L,S", [(80, 2), (80, 4), (32, 3)])
def test_head_weighted_split_gives_last_stage_fewer_layers(L, S):
    split = plan_layer_split(L, S, 1.0, 0.0, 2.0)
    assert split[0][0] == 0 and split[-1][1] == L
    sizes = [b - a for a, b in split]
    assert sizes[-1] <= min(sizes[:-1])


# ----------------------------------------------------------------------------- HF introspection

def test_layer_module_llama_and_gpt_and_missing():
    m = MagicMock()
    m.model.layers = nn.ModuleList([nn.Linear(2, 2)])
    assert _get_layer_module(m, None) is m.model.layers
    g = MagicMock()
    del g.model
    g.transformer.h = nn.ModuleList([nn.Linear(2, 2)])
    assert _get_layer_module(g, None) is g.transformer.h
    n = MagicMock()
    del n.model
    del n.transformer
    del n.gpt_neox
    assert _get_layer_module(n, None) is None


def test_layer_module_opt_decoder():
    m = MagicMock()
    del m.model.layers
    m.model.decoder.layers = nn.ModuleList([nn.Linear(2, 2)])
    assert _get_layer_module(m) is m.model.decoder.layers


def test_embedding_and_norm_modules():
    m = MagicMock()
    m.model.embed_tokens = nn.Embedding(10, 4)
    m.model.norm = nn.LayerNorm(4)
    assert _get_embedding_module(m, None) is m.model.embed_tokens
    assert _get_norm_module(m, None) is m.model.norm
    g = MagicMock()
    del g.model
    g.transformer.wte = nn.Embedding(10, 4)
    g.transformer.ln_f = nn.LayerNorm(4)
    assert _get_embedding_module(g, None) is g.transformer.wte
    assert _get_norm_module(g, None) is g.transformer.ln_f


@pytest.mark.parametrize("a,b,emb,head", [(10, 20, False, False), (0, 10, True, False), (25, 32, False, True),
                                          (0, 32, True, True)])
def test_device_map(a, b, emb, head):
    dm = _create_device_map_for_layers(None, a, b, "cuda:0", include_embeddings=emb, include_lm_head=head)
    assert ("model.embed_tokens" in dm) == emb
    assert ("lm_head" in dm) == head and ("model.norm" in dm) == head
    assert dm[f"model.layers.{a}"] == "cuda:0" and dm[f"model.layers.{b - 1}"] == "cuda:0"
    assert f"model.layers.{b}" not in dm


def test_device_maps_of_a_split_cover_every_layer():
    layers = set()
    for i in range(3):
        a, b = get_layer_range_for_worker(32, 3, i)
        dm = _create_device_map_for_layers(None, a, b, f"cuda:{i}", i == 0, i == 2)
        layers |= {int(k.rsplit(".", 1)[1]) for k in dm if k.startswith("model.layers.")}
    assert layers == set(range(32))
