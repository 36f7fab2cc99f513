"""Model configurations (Llama-3 8B/70B, OPT-125m, tiny test models).

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
    arch: str = "llama"  # "llama" | "opt"
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
    bos_token_id: int = 128000
    eos_token_id: int = 128001

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
        eos = d.get("eos_token_id", 2)
        if isinstance(eos, list):
            eos = eos[0]
        return ModelConfig(name=name, arch="llama", vocab_size=d["vocab_size"], hidden_size=H,
                           intermediate_size=d["intermediate_size"], num_layers=d["num_hidden_layers"],
                           num_heads=nh, num_kv_heads=d.get("num_key_value_heads", nh),
                           head_dim=d.get("head_dim", H // nh), rope_theta=d.get("rope_theta", 10000.0),
                           rope_scaling=d.get("rope_scaling"), rms_eps=d.get("rms_norm_eps", 1e-5),
                           max_position=d.get("max_position_embeddings", 8192),
                           tie_embeddings=d.get("tie_word_embeddings", False),
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
}


def get_config(name_or_path: str) -> ModelConfig:
    key = ALIASES.get(name_or_path, name_or_path)
    if key in PRESETS:
        return dataclasses.replace(PRESETS[key])
    if os.path.exists(name_or_path):
        return ModelConfig.from_file(name_or_path)
    lk = key.lower()
    if "70b" in lk:
        return dataclasses.replace(PRESETS["llama3-70b"], name=name_or_path)
    if "8b" in lk or "7b" in lk:
        return dataclasses.replace(PRESETS["llama3-8b"], name=name_or_path)
    raise KeyError(f"unknown model {name_or_path!r}; presets: {sorted(PRESETS)}")
