"""Model configurations (Llama-3 8B/70B, Qwen2.5 7B/0.5B, GLM-4-9B, OPT-125m, tiny test models).

Mirrors the fields the reference reads from HF ``AutoConfig``
(worker/distributed/model_shard.py:273-311 uses hidden_size,
num_attention_heads, num_key_value_heads, intermediate_size,
num_hidden_layers) so ``ShardedModelLoader`` and the native runtime share one
description.  No network: presets are built in; ``from_hf_dict`` accepts a
local ``config.json`` dictionary.
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Optional


@dataclasses.dataclass
class ModelConfig:
    name: str
    arch: str = "llama"  # "llama" | "qwen2" | "opt"
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 8
    head_dim: int = 128
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = None
    rms_eps: float = 1e-5
    max_position: int = 8192
    tie_embeddings: bool = False
    qkv_bias: bool = False          # Qwen2 / GLM-4: biased q/k/v projections
    rotary_dim: Optional[int] = None  # rotated dims per head (GLM-4: head_dim / 2); None = head_dim
    rope_interleaved: bool = False  # GLM-4 / GPT-J pairing (2i, 2i+1) instead of NeoX (i, i+rd/2)
    bos_token_id: int = 128000
    eos_token_id: int = 128001

    @property
    def rope_dim(self) -> int:
        return self.rotary_dim or self.head_dim

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    @property
    def qkv_size(self) -> int:
        return self.q_size + 2 * self.kv_size

    def param_count(self) -> int:
        H, I, V, L = self.hidden_size, self.intermediate_size, self.vocab_size, self.num_layers
        per_layer = H * self.qkv_size + self.q_size * H + 2 * H * I + I * H + 2 * H
        if self.qkv_bias:
            per_layer += self.qkv_size
        emb = V * H * (1 if self.tie_embeddings else 2)
        return L * per_layer + emb + H

    def kv_bytes_per_token(self, dtype_bytes: int = 2, layers: Optional[int] = None) -> int:
        L = self.num_layers if layers is None else layers
        return 2 * L * self.num_kv_heads * self.head_dim * dtype_bytes

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    @staticmethod
    def from_hf_dict(d: dict, name: str = "hf") -> "ModelConfig":
        mt = d.get("model_type", "llama")
        if mt == "opt":
            H = d["hidden_size"]
            nh = d["num_attention_heads"]
            return ModelConfig(name=name, arch="opt", vocab_size=d["vocab_size"], hidden_size=H,
                               intermediate_size=d.get("ffn_dim", 4 * H), num_layers=d["num_hidden_layers"],
                               num_heads=nh, num_kv_heads=nh, head_dim=H // nh,
                               max_position=d.get("max_position_embeddings", 2048),
                               tie_embeddings=True, bos_token_id=d.get("bos_token_id", 2),
                               eos_token_id=d.get("eos_token_id", 2), rms_eps=1e-5)
        H = d["hidden_size"]
        nh = d["num_attention_heads"]
        # transformers >= 5 nests RoPE settings under ``rope_parameters``
        rp = d.get("rope_parameters") or {}
        theta = d.get("rope_theta", rp.get("rope_theta", 10000.0))
        scaling = d.get("rope_scaling")
        if scaling is None and rp.get("rope_type", "default") != "default":
            scaling = dict(rp)
        eos = d.get("eos_token_id", 2)
        if isinstance(eos, list):
            eos = eos[0]
        arch = {"qwen2": "qwen2", "glm": "glm"}.get(mt, "llama")
        hd = d.get("head_dim") or H // nh
        prf = d.get("partial_rotary_factor", rp.get("partial_rotary_factor", 1.0))
        rot = int(hd * prf) if prf and prf < 1.0 else None
        return ModelConfig(name=name, arch=arch, vocab_size=d["vocab_size"], hidden_size=H,
                           intermediate_size=d["intermediate_size"], num_layers=d["num_hidden_layers"],
                           num_heads=nh, num_kv_heads=d.get("num_key_value_heads", nh),
                           head_dim=d.get("head_dim") or H // nh, rope_theta=float(theta),
                           rope_scaling=scaling, rms_eps=d.get("rms_norm_eps", 1e-5),
                           max_position=d.get("max_position_embeddings", 8192),
                           tie_embeddings=d.get("tie_word_embeddings", False),
                           qkv_bias=bool(d.get("attention_bias", mt == "qwen2")),
                           rotary_dim=rot, rope_interleaved=(mt == "glm"),
                           bos_token_id=d.get("bos_token_id", 1), eos_token_id=eos)

    @staticmethod
    def from_file(path: str) -> "ModelConfig":
        if os.path.isdir(path):
            path = os.path.join(path, "config.json")
        with open(path) as f:
            return ModelConfig.from_hf_dict(json.load(f), name=os.path.basename(os.path.dirname(path)))


PRESETS: dict[str, ModelConfig] = {
    "llama3-8b": ModelConfig(name="llama3-8b"),
    "llama3-70b": ModelConfig(name="llama3-70b", hidden_size=8192, intermediate_size=28672, num_layers=80,
                              num_heads=64, num_kv_heads=8),
    # Small but shape-faithful (GQA 8:1, head_dim 128) Llama for tests / smoke.
    "llama-tiny": ModelConfig(name="llama-tiny", vocab_size=512, hidden_size=512, intermediate_size=1024,
                              num_layers=2, num_heads=8, num_kv_heads=1, head_dim=64, max_position=2048,
                              bos_token_id=1, eos_token_id=2),
    "llama-tiny-hd128": ModelConfig(name="llama-tiny-hd128", vocab_size=1024, hidden_size=1024,
                                    intermediate_size=2048, num_layers=4, num_heads=8, num_kv_heads=1,
                                    head_dim=128, max_position=4096, bos_token_id=1, eos_token_id=2),
    # GQA with 2 KV heads so tensor parallelism of degree 2 has a head per rank
    "llama-tiny-tp": ModelConfig(name="llama-tiny-tp", vocab_size=1024, hidden_size=1024, intermediate_size=2048,
                                 num_layers=2, num_heads=8, num_kv_heads=2, head_dim=128, max_position=4096,
                                 bos_token_id=1, eos_token_id=2),
    # Qwen2 / Qwen2.5 family (the reference's default LLM is Qwen2.5-7B-Instruct):
    # Llama block + biased QKV, GQA 7:1 (7B) / 7:1 (0.5B), theta 1e6
    "qwen2.5-7b": ModelConfig(name="qwen2.5-7b", arch="qwen2", vocab_size=152064, hidden_size=3584,
                              intermediate_size=18944, num_layers=28, num_heads=28, num_kv_heads=4, head_dim=128,
                              rope_theta=1000000.0, rms_eps=1e-6, max_position=32768, qkv_bias=True,
                              bos_token_id=151643, eos_token_id=151645),
    "qwen2.5-0.5b": ModelConfig(name="qwen2.5-0.5b", arch="qwen2", vocab_size=151936, hidden_size=896,
                                intermediate_size=4864, num_layers=24, num_heads=14, num_kv_heads=2, head_dim=64,
                                rope_theta=1000000.0, rms_eps=1e-6, max_position=32768, tie_embeddings=True,
                                qkv_bias=True, bos_token_id=151643, eos_token_id=151645),
    # shape-faithful tiny Qwen2 (biased QKV, GQA 7:1, tied embeddings) for tests
    "qwen-tiny": ModelConfig(name="qwen-tiny", arch="qwen2", vocab_size=1024, hidden_size=1024,
                             intermediate_size=1536, num_layers=2, num_heads=14, num_kv_heads=2, head_dim=128,
                             rope_theta=1000000.0, rms_eps=1e-6, max_position=4096, tie_embeddings=True,
                             qkv_bias=True, bos_token_id=1, eos_token_id=2),
    # GLM-4-9B (HF "glm"): Llama block + biased QKV, GQA 16:1, half-dim interleaved RoPE
    "glm-4-9b": ModelConfig(name="glm-4-9b", arch="glm", vocab_size=151552, hidden_size=4096,
                            intermediate_size=13696, num_layers=40, num_heads=32, num_kv_heads=2, head_dim=128,
                            rope_theta=10000.0, rms_eps=1.5625e-07, max_position=131072, qkv_bias=True,
                            rotary_dim=64, rope_interleaved=True, bos_token_id=151331, eos_token_id=151329),
    "glm-tiny": ModelConfig(name="glm-tiny", arch="glm", vocab_size=1024, hidden_size=1024, intermediate_size=1536,
                            num_layers=2, num_heads=8, num_kv_heads=2, head_dim=128, rope_theta=10000.0,
                            rms_eps=1.5625e-07, max_position=4096, qkv_bias=True, rotary_dim=64,
                            rope_interleaved=True, bos_token_id=1, eos_token_id=2),
    "opt-125m": ModelConfig(name="opt-125m", arch="opt", vocab_size=50272, hidden_size=768,
                            intermediate_size=3072, num_layers=12, num_heads=12, num_kv_heads=12, head_dim=64,
                            max_position=2048, tie_embeddings=True, bos_token_id=2, eos_token_id=2),
}

ALIASES = {
    "meta-llama/Meta-Llama-3-8B": "llama3-8b",
    "meta-llama/Meta-Llama-3-8B-Instruct": "llama3-8b",
    "meta-llama/Llama-3.1-8B-Instruct": "llama3-8b",
    "meta-llama/Meta-Llama-3-70B": "llama3-70b",
    "meta-llama/Meta-Llama-3-70B-Instruct": "llama3-70b",
    "facebook/opt-125m": "opt-125m",
    "Qwen/Qwen2.5-7B-Instruct": "qwen2.5-7b",
    "Qwen/Qwen2.5-7B": "qwen2.5-7b",
    "Qwen/Qwen2-7B-Instruct": "qwen2.5-7b",
    "Qwen/Qwen2.5-0.5B-Instruct": "qwen2.5-0.5b",
    "THUDM/glm-4-9b-chat-hf": "glm-4-9b",
    "THUDM/glm-4-9b-chat": "glm-4-9b",
    "THUDM/glm-4-9b-hf": "glm-4-9b",
}


def get_config(name_or_path: str) -> ModelConfig:
    """Preset, alias, HF config dir/file, or a family guess from the name.
    ``<model>@L<n>`` keeps the architecture and truncates it to ``n`` layers
    (multi-rank rehearsals of a big model's shapes on one GPU)."""
    if "@L" in name_or_path:
        base, n = name_or_path.rsplit("@L", 1)
        return dataclasses.replace(get_config(base), name=name_or_path, num_layers=int(n))
    key = ALIASES.get(name_or_path, name_or_path)
    if key in PRESETS:
        return dataclasses.replace(PRESETS[key])
    if os.path.exists(name_or_path):
        return ModelConfig.from_file(name_or_path)
    lk = key.lower()
    if "glm-4" in lk or "glm4" in lk:
        return dataclasses.replace(PRESETS["glm-4-9b"], name=name_or_path)
    if "qwen" in lk:
        return dataclasses.replace(PRESETS["qwen2.5-0.5b" if "0.5b" in lk else "qwen2.5-7b"], name=name_or_path)
    if "70b" in lk:
        return dataclasses.replace(PRESETS["llama3-70b"], name=name_or_path)
    if "8b" in lk or "7b" in lk:
        return dataclasses.replace(PRESETS["llama3-8b"], name=name_or_path)
    raise KeyError(f"unknown model {name_or_path!r}; presets: {sorted(PRESETS)}")
