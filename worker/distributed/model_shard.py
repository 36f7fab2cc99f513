"""Layer-range model shards (reference worker/distributed/model_shard.py:28-465).

Two backends behind the reference's ``ModelShard`` API:

* **native** (``ModelShard.from_native``): layers ``[start, end)`` of a
  ``dgi`` Llama materialised directly on the MI355X (random-init or
  safetensors), with the stage's own paged KV pool — what the in-node
  pipeline (``dgi.parallel.pipeline``) runs.  ``forward`` keeps the KV
  across calls (the reference discarded it, Appendix E-6).
* **HF** (``ModelShard.from_pretrained``): an HF causal LM loaded from local
  files with a device map restricted to the shard's modules; used for
  cross-node / CPU interop.

``ShardedModelLoader`` plans memory-proportional layer splits;
``get_layer_range_for_worker`` is the even split (remainder to the first
workers).  ``AutoConfig`` is a module-level name so callers can patch it.
"""
from __future__ import annotations

import logging
import math
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from dgi.parallel.plan import get_layer_range_for_worker as _even_range

logger = logging.getLogger(__name__)

try:  # module-level so tests / callers can patch ``model_shard.AutoConfig``
    from transformers import AutoConfig  # type: ignore
except Exception:  # pragma: no cover
    AutoConfig = None  # type: ignore


@dataclass
class LayerInfo:
    layer_idx: int
    layer_name: str
    param_count: int
    memory_bytes: int


class ModelShard(nn.Module):
    def __init__(self, model_id: str, start_layer: int, end_layer: int, device: str = "cuda",
                 dtype: torch.dtype = torch.float16):
        super().__init__()
        self.model_id = model_id
        self.start_layer = start_layer
        self.end_layer = end_layer
        self.device = device
        self.dtype = dtype
        # a plain list: layers may be HF blocks, native stages or any callable
        # returning (hidden, kv) (the reference's tests append stubs)
        self.layers: List[Any] = []
        self.config = None
        self.is_first_shard = False
        self.is_last_shard = False
        self.embed_tokens: Optional[nn.Module] = None
        self.embed_positions: Optional[nn.Module] = None
        self.norm: Optional[nn.Module] = None
        self.lm_head: Optional[nn.Module] = None
        self.rotary_emb: Optional[nn.Module] = None
        self.native = None          # dgi LlamaModel for the native backend
        self.native_engine = None   # dgi runner/pool owning this shard's paged KV

    # ------------------------------------------------------------------ loading
    @classmethod
    def from_native(cls, model_id: str, start_layer: int, end_layer: int, device: str = "cuda",
                    dtype: torch.dtype = torch.bfloat16, seed: int = 0, num_blocks: int = 1024,
                    block_size: int = 16, model_path: Optional[str] = None) -> "ModelShard":
        """Native shard of layers [start, end): reads only those layers from a local
        safetensors checkpoint when one exists (dgi.models.weights), else random init."""
        from dgi.kv.block_pool import BlockPool
        from dgi.models.config import get_config
        from dgi.models.llama import LlamaModel
        from dgi.models.weights import resolve_checkpoint
        ckpt = resolve_checkpoint(model_id, model_path)
        mc = get_config(ckpt or model_id)
        shard = cls(model_id, start_layer, end_layer, device, dtype)
        shard.config = mc
        shard.is_first_shard = start_layer == 0
        shard.is_last_shard = end_layer == mc.num_layers
        shard.native = LlamaModel(mc, device, dtype, start_layer, end_layer, seed=seed, checkpoint=ckpt)
        pool = BlockPool(num_blocks, block_size, max(1, end_layer - start_layer), mc.num_kv_heads, mc.head_dim,
                         dtype, device)
        shard.native.kv_cache = pool.kv
        shard.native_engine = pool
        return shard

    @classmethod
    def from_pretrained(cls, model_id: str, start_layer: int, end_layer: int, device: str = "cuda",
                        dtype: torch.dtype = torch.float16, **kw) -> "ModelShard":
        from transformers import AutoModelForCausalLM
        cfg_cls = AutoConfig
        config = cfg_cls.from_pretrained(model_id, local_files_only=True)
        total = getattr(config, "num_hidden_layers", end_layer)
        shard = cls(model_id, start_layer, end_layer, device, dtype)
        shard.config = config
        shard.is_first_shard = start_layer == 0
        shard.is_last_shard = end_layer >= total
        dmap = _create_device_map_for_layers(config, start_layer, end_layer, device, shard.is_first_shard,
                                             shard.is_last_shard)
        model = AutoModelForCausalLM.from_pretrained(model_id, torch_dtype=dtype, local_files_only=True, **kw)
        model.to(device)
        layers = _get_layer_module(model)
        for i in range(start_layer, end_layer):
            shard.layers.append(layers[i])
        if shard.is_first_shard:
            shard.embed_tokens = _get_embedding_module(model)
            inner = getattr(model, "model", None)
            dec = getattr(inner, "decoder", None)
            shard.embed_positions = getattr(dec, "embed_positions", None)
        if shard.is_last_shard:
            shard.norm = _get_norm_module(model)
            shard.lm_head = getattr(model, "lm_head", None)
        shard.rotary_emb = getattr(getattr(model, "model", None), "rotary_emb", None)
        shard._device_map = dmap
        return shard

    def _extract_layers(self, model) -> None:
        layers = _get_layer_module(model)
        if layers is None:
            raise ValueError("cannot locate transformer layers")
        for i in range(self.start_layer, self.end_layer):
            self.layers.append(layers[i])

    # ------------------------------------------------------------------ compute
    def forward(self, hidden_states: torch.Tensor, position_ids: Optional[torch.Tensor] = None,
                past_key_values: Optional[List] = None, use_cache: bool = True, attention_mask=None
                ) -> Tuple[torch.Tensor, Optional[List]]:
        h = hidden_states
        if self.is_first_shard and self.embed_tokens is not None and not torch.is_floating_point(h):
            h = self.embed_tokens(h)
            if self.embed_positions is not None and position_ids is not None:
                try:
                    h = h + self.embed_positions(position_ids)
                except Exception:
                    pass
        new_kv: List = []
        extra: Dict[str, Any] = {}
        if self.rotary_emb is not None and position_ids is not None:
            try:
                extra["position_embeddings"] = self.rotary_emb(h, position_ids)
            except Exception:
                pass
        # transformers >= 4.5x: one Cache object shared by all layers (each attention
        # updates its own layer_idx slot) — the shard keeps it per session, so decode
        # steps attend to the whole history; legacy per-layer tuples otherwise
        cache_obj = past_key_values if (past_key_values is not None and hasattr(past_key_values, "update")
                                        and hasattr(past_key_values, "get_seq_length")) else None
        for i, layer in enumerate(self.layers):
            if cache_obj is not None:
                out = layer(h, attention_mask=attention_mask, position_ids=position_ids,
                            past_key_values=cache_obj, use_cache=True, **extra)
                h = out[0] if isinstance(out, tuple) else out
                continue
            past = past_key_values[i] if past_key_values is not None and i < len(past_key_values) else None
            out = layer(h, position_ids=position_ids, past_key_value=past, use_cache=use_cache,
                        attention_mask=attention_mask, **extra)
            if isinstance(out, tuple):
                h = out[0]
                if use_cache and len(out) > 1:
                    new_kv.append(out[1])
            else:
                h = out
        if self.is_last_shard and self.norm is not None:
            h = self.norm(h)
        if cache_obj is not None:
            return h, cache_obj
        return h, (new_kv if use_cache else None)

    def get_logits(self, hidden_states: torch.Tensor) -> torch.Tensor:
        if not self.is_last_shard:
            raise RuntimeError("get_logits can only be called on the last shard")
        if self.lm_head is None:
            raise RuntimeError("No lm_head available")
        return self.lm_head(hidden_states)

    def get_memory_usage(self) -> float:
        n = 0
        seen = set()
        mods = [m for m in self.layers if isinstance(m, nn.Module)]
        mods += [m for m in (self.embed_tokens, self.embed_positions, self.norm, self.lm_head) if m is not None]
        for m in mods:
            for p in m.parameters():
                if id(p) not in seen:
                    seen.add(id(p))
                    n += p.numel() * p.element_size()
        if self.native is not None:
            n += self.native.weight_bytes()
        return n / 1024 ** 3

    def get_layer_count(self) -> int:
        if self.native is not None and not len(self.layers):
            return self.native.num_local_layers
        return len(self.layers)


class ShardedModelLoader:
    """Memory-aware split of a model's layers over workers."""

    def __init__(self, model_id: str):
        self.model_id = model_id
        self.config = None
        self.total_layers = 0
        self.layer_infos: List[LayerInfo] = []

    def _load_config(self):
        if AutoConfig is not None:
            try:
                return AutoConfig.from_pretrained(self.model_id)
            except Exception:
                pass
        from dgi.models.config import get_config
        mc = get_config(self.model_id)

        class _C:
            pass
        c = _C()
        c.num_hidden_layers, c.hidden_size, c.num_attention_heads = mc.num_layers, mc.hidden_size, mc.num_heads
        c.num_key_value_heads, c.intermediate_size, c.vocab_size = mc.num_kv_heads, mc.intermediate_size, mc.vocab_size
        return c

    def analyze_model(self) -> Dict[str, Any]:
        c = self._load_config()
        self.config = c
        L = int(c.num_hidden_layers)
        H = int(c.hidden_size)
        nh = int(c.num_attention_heads)
        nkv = int(getattr(c, "num_key_value_heads", nh) or nh)
        I = int(getattr(c, "intermediate_size", 4 * H))
        hd = H // nh
        attn = H * (nh + 2 * nkv) * hd + nh * hd * H
        mlp = 3 * H * I
        per_layer = attn + mlp + 2 * H
        bytes_per_layer = per_layer * 2
        self.total_layers = L
        self.layer_infos = [LayerInfo(i, f"model.layers.{i}", per_layer, bytes_per_layer) for i in range(L)]
        vocab = int(getattr(c, "vocab_size", 0) or 0)
        return {"model_id": self.model_id, "total_layers": L, "hidden_size": H, "num_attention_heads": nh,
                "num_key_value_heads": nkv, "intermediate_size": I, "params_per_layer": per_layer,
                "memory_per_layer_gb": bytes_per_layer / 1024 ** 3,
                "embedding_memory_gb": 2 * vocab * H * 2 / 1024 ** 3,
                "total_memory_gb": (L * bytes_per_layer + 2 * vocab * H * 2) / 1024 ** 3}

    def create_shard_plan(self, worker_memory_gb: List[float], reserve_ratio: float = 0.2) -> List[Tuple[int, int]]:
        info = self.analyze_model()
        L = info["total_layers"]
        per = info["memory_per_layer_gb"]
        usable = [max(0.0, m * (1 - reserve_ratio)) for m in worker_memory_gb]
        capacity = [int(u // per) if per > 0 else L for u in usable]
        if sum(capacity) < L:
            raise ValueError(f"Insufficient memory: {sum(usable):.1f} GB usable for {L * per:.1f} GB of layers")
        total = sum(usable)
        want = [u / total * L for u in usable]
        counts = [min(capacity[i], int(math.floor(want[i]))) for i in range(len(usable))]
        i = 0
        order = sorted(range(len(usable)), key=lambda j: -(want[j] - counts[j]))
        while sum(counts) < L:
            j = order[i % len(order)]
            if counts[j] < capacity[j]:
                counts[j] += 1
            i += 1
        plan, start = [], 0
        for c in counts:
            plan.append((start, start + c))
            start += c
        return [p for p in plan if p[1] > p[0]]


def get_layer_range_for_worker(total_layers: int, num_workers: int, worker_index: int) -> Tuple[int, int]:
    return _even_range(total_layers, num_workers, worker_index)


def _walk(obj, path):
    for p in path:
        if obj is None or not hasattr(obj, p):
            return None
        obj = getattr(obj, p)
    return obj


def _first_module(model, paths, kinds=(nn.Module,)):
    for path in paths:
        obj = _walk(model, path)
        if isinstance(obj, kinds):
            return obj
    return None


def _get_layer_module(model, config=None):
    """Transformer block list: Llama ``model.layers``, OPT ``model.decoder.layers``, GPT ``transformer.h``."""
    return _first_module(model, (("model", "layers"), ("model", "decoder", "layers"), ("transformer", "h"),
                                 ("gpt_neox", "layers")), (nn.ModuleList,))


def _get_embedding_module(model, config=None):
    return _first_module(model, (("model", "embed_tokens"), ("model", "decoder", "embed_tokens"),
                                 ("transformer", "wte")))


def _get_norm_module(model, config=None):
    return _first_module(model, (("model", "norm"), ("model", "decoder", "final_layer_norm"),
                                 ("transformer", "ln_f")))


def _create_device_map_for_layers(config, start_layer: int, end_layer: int, device: str,
                                  include_embeddings: bool = False, include_lm_head: bool = False) -> Dict[str, str]:
    dmap: Dict[str, str] = {}
    if include_embeddings:
        dmap["model.embed_tokens"] = device
    for i in range(start_layer, end_layer):
        dmap[f"model.layers.{i}"] = device
    if include_lm_head:
        dmap["model.norm"] = device
        dmap["lm_head"] = device
    return dmap
