"""Native model numerics against Hugging Face reference implementations.

The reference serves these families through HF ``transformers`` (its live
path is ``AutoModelForCausalLM.generate``, worker/engines/llm.py:43-86; the
default model is Qwen2.5-7B-Instruct and its README lists Llama-3.1-8B and
GLM-4-9B, worker/README.md:86-97).  Here a tiny random HF model of each
family is built in fp32, its state dict is loaded into the native
``LlamaModel`` with ``load_state_dict_hf``, and the native engine (paged KV,
chunked prefill, decode steps) must reproduce HF's prefill logits and its
greedy continuation.  CPU path (PyTorch reference ops); the same checks run
on the MI355X kernels in tests/test_kernels_gpu.py.
"""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from dgi.engine import EngineConfig, LLMEngine  # noqa: E402
from dgi.models.config import ModelConfig  # noqa: E402
from dgi.models.llama import LlamaModel  # noqa: E402
from dgi.sched.request import SamplingParams  # noqa: E402

H, I, L, NH, NKV, HD, V = 256, 512, 2, 8, 2, 32, 512


def _hf(family):
    common = dict(vocab_size=V, hidden_size=H, intermediate_size=I, num_hidden_layers=L, num_attention_heads=NH,
                  num_key_value_heads=NKV, max_position_embeddings=512, rms_norm_eps=1e-6, bos_token_id=1,
                  eos_token_id=2, tie_word_embeddings=False)
    if family == "llama":
        cfg = transformers.LlamaConfig(rope_theta=500000.0, attention_bias=False, **common)
        model = transformers.LlamaForCausalLM(cfg)
    elif family == "glm":
        cfg = transformers.GlmConfig(rope_theta=10000.0, partial_rotary_factor=0.5, attention_bias=True,
                                     head_dim=HD, pad_token_id=0, **common)
        model = transformers.GlmForCausalLM(cfg)
    else:
        cfg = transformers.Qwen2Config(rope_theta=1000000.0, **common)
        model = transformers.Qwen2ForCausalLM(cfg)
    torch.manual_seed(0)
    with torch.no_grad():
        for n, p in model.named_parameters():
            if "norm" in n:
                p.copy_(1.0 + 0.1 * torch.randn_like(p))
            else:
                p.normal_(0.0, 0.05)
    return model.eval(), cfg


def _native(cfg, model):
    mc = ModelConfig.from_hf_dict(cfg.to_dict(), name="hf-tiny")
    nm = LlamaModel(mc, "cpu", torch.float32, init="empty")
    nm.load_state_dict_hf(model.state_dict())
    eng = LLMEngine(EngineConfig(model="hf-tiny", device="cpu", dtype=torch.float32, num_blocks=64, max_num_seqs=4,
                                 max_model_len=256, max_num_batched_tokens=64, use_graphs=False,
                                 enable_prefix_caching=False), model_cfg=mc, model=nm)
    return mc, eng


FAMILIES = ["llama", "qwen2", "glm"]


@pytest.mark.parametrize("family", FAMILIES)
def test_config_translation(family):
    _, cfg = _hf(family)
    mc = ModelConfig.from_hf_dict(cfg.to_dict())
    assert (mc.hidden_size, mc.num_heads, mc.num_kv_heads, mc.head_dim) == (H, NH, NKV, HD)
    assert mc.qkv_bias == (family in ("qwen2", "glm"))
    assert mc.arch == family
    # transformers >= 5 nests theta under rope_parameters; it must not fall back to 1e4
    assert mc.rope_theta == {"qwen2": 1e6, "llama": 5e5, "glm": 1e4}[family]
    assert (mc.rope_dim, mc.rope_interleaved) == ((HD // 2, True) if family == "glm" else (HD, False))


@pytest.mark.parametrize("family", FAMILIES)
def test_greedy_continuation_matches_hf(family):
    model, cfg = _hf(family)
    _, eng = _native(cfg, model)
    prompts = [[1, 17, 99, 250, 3, 77, 401, 12, 8, 300, 45], [1, 5, 6]]
    n_new = 8
    reqs = eng.generate(prompts, SamplingParams(max_tokens=n_new, temperature=0.0, ignore_eos=True))
    for p, r in zip(prompts, reqs):
        with torch.no_grad():
            ref = model.generate(torch.tensor([p]), max_new_tokens=n_new, do_sample=False, min_new_tokens=n_new,
                                 pad_token_id=0)[0, len(p):].tolist()
        assert r.output == ref, (family, r.output, ref)


@pytest.mark.parametrize("family", FAMILIES)
def test_prefill_logits_match_hf(family):
    from dgi.runtime.batch import AttnMeta  # noqa: F401  (engine path below builds it)
    model, cfg = _hf(family)
    mc, eng = _native(cfg, model)
    prompt = [1, 33, 44, 55, 66, 77, 88, 99, 111, 222]
    with torch.no_grad():
        ref = model(torch.tensor([prompt])).logits[0, -1]
    # one greedy step exposes the native last-position logits through the sampler input
    captured = {}
    orig = eng.model.compute_logits

    def spy(h, residual, idx):
        out = orig(h, residual, idx)
        captured["logits"] = out.detach().clone()
        return out

    eng.model.compute_logits = spy
    eng.generate([prompt], SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))
    got = captured["logits"][-1]
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)
