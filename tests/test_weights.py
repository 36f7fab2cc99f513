"""Real-weight loading for the native runtime (dgi.models.weights).

The reference's live LLM path serves real checkpoints
(``AutoModelForCausalLM.from_pretrained``, worker/engines/llm.py:14-41) and
its pipeline shards load a layer range (worker/distributed/model_shard.py:
61-148).  Here a tiny HF model of each family is ``save_pretrained``'d as
safetensors into a temp dir (no network), the native engine loads it through
``EngineConfig(model_path=...)`` and must match HF's logits; shard-local loads
must read only their own layers.  Multi-process PP / TP loads from the same
files are in tests/test_parallel_cpu.py.
"""
import os

import pytest
import torch

transformers = pytest.importorskip("transformers")

from dgi.engine import EngineConfig, LLMEngine  # noqa: E402
from dgi.models.config import ModelConfig  # noqa: E402
from dgi.models.llama import LlamaModel  # noqa: E402
from dgi.models.weights import CheckpointReader, resolve_checkpoint  # noqa: E402
from dgi.sched.request import SamplingParams  # noqa: E402

from test_model_hf_parity import FAMILIES, _hf  # noqa: E402


def save_tiny(family, d, shard_size=None):
    model, cfg = _hf(family)
    kw = {"safe_serialization": True}
    if shard_size:
        kw["max_shard_size"] = shard_size
    model.save_pretrained(d, **kw)
    return model, cfg


def _last_logits(eng, prompt):
    captured = {}
    orig = eng.model.compute_logits

    def spy(h, residual, idx):
        out = orig(h, residual, idx)
        captured["logits"] = out.detach().clone()
        return out

    eng.model.compute_logits = spy
    eng.generate([prompt], SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))
    return captured["logits"][-1]


@pytest.mark.parametrize("family", FAMILIES)
def test_engine_loads_safetensors_and_matches_hf(family, tmp_path):
    model, _ = save_tiny(family, str(tmp_path))
    eng = LLMEngine(EngineConfig(model="whatever", model_path=str(tmp_path), device="cpu", dtype=torch.float32,
                                 num_blocks=64, max_num_seqs=4, max_model_len=256, max_num_batched_tokens=64,
                                 use_graphs=False, enable_prefix_caching=False))
    assert eng.checkpoint == str(tmp_path)
    assert eng.model.load_info["tensors"] > 0
    prompt = [1, 33, 44, 55, 66, 77, 88, 99, 111, 222]
    with torch.no_grad():
        ref = model(torch.tensor([prompt])).logits[0, -1]
    torch.testing.assert_close(_last_logits(eng, prompt), ref, rtol=1e-4, atol=1e-4)
    # greedy continuation too
    reqs = eng.generate([prompt], SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True))
    with torch.no_grad():
        want = model.generate(torch.tensor([prompt]), max_new_tokens=6, do_sample=False, min_new_tokens=6,
                              pad_token_id=0)[0, len(prompt):].tolist()
    assert reqs[0].output == want


def test_model_dir_as_model_id_and_sharded_index(tmp_path):
    model, _ = save_tiny("llama", str(tmp_path), shard_size="200KB")
    assert os.path.exists(tmp_path / "model.safetensors.index.json")
    assert resolve_checkpoint(str(tmp_path)) == str(tmp_path)
    eng = LLMEngine(EngineConfig(model=str(tmp_path), device="cpu", dtype=torch.float32, num_blocks=64,
                                 max_num_seqs=4, max_model_len=256, max_num_batched_tokens=64, use_graphs=False,
                                 enable_prefix_caching=False))
    prompt = [1, 5, 9, 13, 2, 200]
    with torch.no_grad():
        ref = model(torch.tensor([prompt])).logits[0, -1]
    torch.testing.assert_close(_last_logits(eng, prompt), ref, rtol=1e-4, atol=1e-4)


def test_bf16_load_casts_and_stays_close(tmp_path):
    model, _ = save_tiny("qwen2", str(tmp_path))
    eng = LLMEngine(EngineConfig(model_path=str(tmp_path), device="cpu", dtype=torch.bfloat16, num_blocks=64,
                                 max_num_seqs=4, max_model_len=256, max_num_batched_tokens=64, use_graphs=False,
                                 enable_prefix_caching=False))
    assert eng.model.layers[0].qkv.dtype == torch.bfloat16
    prompt = [1, 3, 5, 7, 11, 13]
    with torch.no_grad():
        ref = model(torch.tensor([prompt])).logits[0, -1]
    got = _last_logits(eng, prompt).float()
    assert torch.nn.functional.cosine_similarity(got, ref, dim=0) > 0.999


def test_stage_reads_only_its_layers(tmp_path):
    save_tiny("llama", str(tmp_path))
    mc = ModelConfig.from_file(str(tmp_path))
    full = LlamaModel(mc, "cpu", torch.float32, checkpoint=str(tmp_path))
    first = LlamaModel(mc, "cpu", torch.float32, 0, 1, checkpoint=str(tmp_path))
    last = LlamaModel(mc, "cpu", torch.float32, 1, 2, checkpoint=str(tmp_path))
    assert first.load_info["bytes"] < full.load_info["bytes"]
    assert last.load_info["bytes"] < full.load_info["bytes"]
    assert first.lm_head is None and last.embed is None
    # disjoint ranges reassemble the full model bit for bit
    src = dict(full.tensors())
    for part in (first, last):
        for name, t in part.tensors():
            assert torch.equal(t, src[name]), name
    rd = CheckpointReader(str(tmp_path))
    assert "model.layers.1.mlp.down_proj.weight" in rd


def test_native_engine_refuses_silent_random_weights(tmp_path):
    from worker.engines.llm_native import NativeLLMEngine

    with pytest.raises(FileNotFoundError):
        NativeLLMEngine({"model_id": "someorg/not-cached-model", "device": "cpu"}).load_model()
    save_tiny("llama", str(tmp_path))
    e = NativeLLMEngine({"model_id": "someorg/tiny", "model_path": str(tmp_path), "device": "cpu",
                         "num_blocks": 64, "max_num_seqs": 4, "context_length": 256, "chunked_prefill_size": 64})
    e.load_model()
    try:
        st = e.get_status()
        assert st["engine"]["weights"] == str(tmp_path)
    finally:
        e.unload_model()


def test_hf_shard_chain_keeps_kv_across_decode_steps(tmp_path):
    """HF shards behind the gRPC/HTTP servicer keep a per-session KV cache
    (the reference passed use_cache without past_key_values, E-6): a 2-shard
    chain decoding token by token reproduces HF greedy generation, including a
    multi-token chunk appended over an existing prefix."""
    from worker.distributed.grpc_server import InferenceServicer
    from worker.distributed.model_shard import ModelShard

    model, _ = save_tiny("llama", str(tmp_path))
    shards = [ModelShard.from_pretrained(str(tmp_path), a, b, device="cpu", dtype=torch.float32)
              for a, b in ((0, 1), (1, 2))]
    svcs = [InferenceServicer(s) for s in shards]
    prompt = [1, 17, 99, 250, 3, 77, 401]
    with torch.no_grad():
        want = model.generate(torch.tensor([prompt]), max_new_tokens=6, do_sample=False, min_new_tokens=6,
                              pad_token_id=0)[0].tolist()

    def run(ids, pos):
        x = torch.tensor([ids])
        for sv in svcs:
            x = sv._forward(sv._session("s"), x, pos)
        with torch.inference_mode():
            return int(shards[-1].get_logits(x)[0, -1].argmax())

    # prefill the first 4 prompt tokens, then append the rest as one chunk, then decode
    run(prompt[:4], 0)
    tok = run(prompt[4:], 4)
    out = list(prompt) + [tok]
    for _ in range(5):
        tok = run([tok], len(out) - 1)
        out.append(tok)
    assert out == want
