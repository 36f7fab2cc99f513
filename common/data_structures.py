"""Shared data types of the distributed inference platform (wire/API layer L1).

API-compatible with the reference's ``common/data_structures.py`` (roles,
worker/session/shard descriptors) so the server, the worker
and SDK code exchange the same dicts.  Differences, all deliberate:

* ``compute_prefix_hash`` hashes the ids as little-endian int32 (the
  reference's ``bytes(token_ids)`` raises for ids >= 256, Appendix E-11);
* ``estimate_kv_cache_size`` accepts ``num_kv_heads`` for GQA models
  (Llama-3: 8 KV heads, not 64);
* ``ModelShardConfig`` can be built from a ``dgi`` ModelConfig.
"""
from __future__ import annotations

import hashlib
import struct
import time
from dataclasses import dataclass, field
from enum import Enum
from typing import Any, Dict, List, Optional, Tuple


class WorkerRole(Enum):
    PREFILL = "prefill"   # compute-bound phase (DistServe prefill instance)
    DECODE = "decode"     # bandwidth-bound phase
    HYBRID = "hybrid"     # serves both phases


class WorkerState(Enum):
    OFFLINE = 0
    JOINING = 1
    ONLINE = 2
    BUSY = 3
    ERROR = 4


@dataclass
class BlockRange:
    """Half-open range of transformer layers ``[start, end)`` owned by a shard."""
    start: int
    end: int

    @property
    def length(self) -> int:
        return self.end - self.start

    def __contains__(self, layer_idx: int) -> bool:
        return self.start <= layer_idx < self.end

    def to_dict(self) -> Dict[str, int]:
        return {"start": self.start, "end": self.end}

    @classmethod
    def from_dict(cls, data: Dict[str, int]) -> "BlockRange":
        return cls(start=int(data["start"]), end=int(data["end"]))


@dataclass
class WorkerInfo:
    worker_id: str
    blocks: Optional[BlockRange] = None
    role: WorkerRole = WorkerRole.HYBRID
    state: WorkerState = WorkerState.OFFLINE
    gpu_name: str = ""
    gpu_memory_gb: float = 0.0
    gpu_memory_used_gb: float = 0.0
    throughput_tokens_per_sec: float = 0.0
    latency_ms: float = 0.0
    reliability_score: float = 1.0
    peer_address: str = ""
    api_endpoint: str = ""
    cache_tokens_available: int = 0
    cache_tokens_used: int = 0
    model_id: str = ""
    supported_models: List[str] = field(default_factory=list)
    last_heartbeat: float = field(default_factory=time.time)

    @property
    def cache_utilization(self) -> float:
        return self.cache_tokens_used / self.cache_tokens_available if self.cache_tokens_available else 0.0

    @property
    def gpu_utilization(self) -> float:
        return self.gpu_memory_used_gb / self.gpu_memory_gb if self.gpu_memory_gb else 0.0

    def is_healthy(self, timeout_seconds: float = 60.0) -> bool:
        if self.state in (WorkerState.OFFLINE, WorkerState.ERROR):
            return False
        return (time.time() - self.last_heartbeat) < timeout_seconds

    def to_dict(self) -> Dict[str, Any]:
        d = {k: getattr(self, k) for k in self.__dataclass_fields__}
        d["blocks"] = self.blocks.to_dict() if self.blocks else None
        d["role"] = self.role.value
        d["state"] = self.state.value
        d["supported_models"] = list(self.supported_models)
        return d

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "WorkerInfo":
        kw = {k: v for k, v in d.items() if k in cls.__dataclass_fields__}
        if kw.get("blocks") is not None:
            kw["blocks"] = BlockRange.from_dict(kw["blocks"])
        if "role" in kw:
            kw["role"] = WorkerRole(kw["role"])
        if "state" in kw:
            kw["state"] = WorkerState(kw["state"])
        return cls(**kw)


@dataclass
class InferenceState:
    """Per-session cursor carried between pipeline stages."""
    session_id: str
    position: int = 0
    kv_cache_keys: List[str] = field(default_factory=list)
    hidden_states_data: Optional[bytes] = None
    hidden_states_shape: Optional[Tuple[int, ...]] = None
    hidden_states_dtype: str = "float16"
    input_tokens: int = 0
    output_tokens: int = 0
    created_at: float = field(default_factory=time.time)
    updated_at: float = field(default_factory=time.time)

    def update_position(self, new_tokens: int) -> None:
        self.position += new_tokens
        self.updated_at = time.time()


@dataclass
class KVCacheBlock:
    """Metadata of one KV page (PagedAttention style, copy-on-write ref count)."""
    block_id: str
    layer_idx: int
    block_size: int = 16
    keys_data: Optional[bytes] = None
    values_data: Optional[bytes] = None
    num_heads: int = 0
    head_dim: int = 0
    ref_count: int = 1
    prefix_hash: str = ""
    location: str = "gpu"  # gpu | cpu | redis | remote

    @property
    def is_shared(self) -> bool:
        return self.ref_count > 1

    def increment_ref(self) -> None:
        self.ref_count += 1

    def decrement_ref(self) -> int:
        self.ref_count = max(0, self.ref_count - 1)
        return self.ref_count


@dataclass
class InferenceRequest:
    request_id: str
    session_id: str
    input_data: Optional[bytes] = None
    input_shape: Optional[Tuple[int, ...]] = None
    input_dtype: str = "float16"
    position: int = 0
    max_new_tokens: int = 512
    temperature: float = 0.7
    top_p: float = 0.9
    kv_cache_keys: List[str] = field(default_factory=list)
    next_worker_address: str = ""
    step_id: str = ""
    created_at: float = field(default_factory=time.time)


@dataclass
class InferenceResponse:
    request_id: str
    session_id: str
    output_data: Optional[bytes] = None
    output_shape: Optional[Tuple[int, ...]] = None
    output_dtype: str = "float16"
    updated_kv_keys: List[str] = field(default_factory=list)
    latency_ms: float = 0.0
    tokens_generated: int = 0
    success: bool = True
    error_message: str = ""


@dataclass
class SessionConfig:
    model_name: str
    max_length: int = 4096
    temperature: float = 0.7
    top_p: float = 0.9
    top_k: int = 50
    use_cache: bool = True
    stream: bool = False
    connect_timeout: float = 30.0
    request_timeout: float = 120.0
    max_retries: int = 3
    use_speculative_decoding: bool = False
    speculative_depth: int = 5


@dataclass
class ModelShardConfig:
    """worker_id -> layer range map of a layer-sharded (pipeline) deployment."""
    model_id: str
    total_layers: int
    shard_mapping: Dict[str, BlockRange] = field(default_factory=dict)
    hidden_size: int = 0
    num_attention_heads: int = 0
    num_key_value_heads: int = 0
    intermediate_size: int = 0
    vocab_size: int = 0
    memory_per_layer_gb: float = 0.0
    kv_cache_per_token_bytes: int = 0

    def get_worker_for_layer(self, layer_idx: int) -> Optional[str]:
        for wid, br in self.shard_mapping.items():
            if layer_idx in br:
                return wid
        return None

    def get_inference_route(self) -> List[Tuple[str, BlockRange]]:
        return sorted(self.shard_mapping.items(), key=lambda kv: kv[1].start)

    def is_complete(self) -> bool:
        """Every layer covered exactly once."""
        cover = [0] * self.total_layers
        for br in self.shard_mapping.values():
            for i in range(max(0, br.start), min(self.total_layers, br.end)):
                cover[i] += 1
        return all(c == 1 for c in cover)

    @classmethod
    def from_model_config(cls, mc, shard_mapping: Optional[Dict[str, BlockRange]] = None) -> "ModelShardConfig":
        H, I, L = mc.hidden_size, mc.intermediate_size, mc.num_layers
        per_layer = (H * mc.qkv_size + mc.q_size * H + 3 * H * I) * 2
        return cls(model_id=mc.name, total_layers=L, shard_mapping=dict(shard_mapping or {}), hidden_size=H,
                   num_attention_heads=mc.num_heads, num_key_value_heads=mc.num_kv_heads, intermediate_size=I,
                   vocab_size=mc.vocab_size, memory_per_layer_gb=per_layer / 1024 ** 3,
                   kv_cache_per_token_bytes=mc.kv_bytes_per_token())


def compute_prefix_hash(token_ids: List[int]) -> str:
    """16-hex-digit sha256 of the ids packed as little-endian int32."""
    data = struct.pack(f"<{len(token_ids)}i", *[int(t) for t in token_ids])
    return hashlib.sha256(data).hexdigest()[:16]


def estimate_kv_cache_size(num_layers: int, num_heads: int, head_dim: int, seq_length: int,
                           batch_size: int = 1, dtype_bytes: int = 2,
                           num_kv_heads: Optional[int] = None) -> int:
    """Bytes of K+V for ``batch_size`` sequences of ``seq_length`` tokens."""
    heads = num_heads if num_kv_heads is None else num_kv_heads
    return 2 * num_layers * batch_size * seq_length * heads * head_dim * dtype_bytes
