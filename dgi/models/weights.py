"""Checkpoint loading for the native runtime: HF safetensors -> dgi weight layout.

The reference serves real checkpoints through ``AutoModelForCausalLM.from_pretrained``
(worker/engines/llm.py:14-41) and loads a layer range per pipeline worker
(worker/distributed/model_shard.py:61-148).  Here the dgi model (any layer range,
any tensor-parallel rank) reads exactly the bytes it owns:

* shards are opened with ``safetensors.safe_open`` (memory-mapped, nothing
  is unpickled) and read tensor by tensor through ``get_slice``, so a
  pipeline stage touches only its own layers and a TP rank only its rows /
  columns of each projection — there is never a full CPU copy of the model;
* each slice lands directly in its place inside the fused device weights
  (q|k|v -> ``qkv``, gate|up -> ``gate_up``; GLM's already fused
  ``gate_up_proj`` is split per TP rank);
* tensors are cast to the model dtype on the way (fp32 / fp16 checkpoints
  load into bf16 weights).

``resolve_checkpoint`` finds a local checkpoint for a model id: an explicit
path, a directory given as the model id, or an offline Hugging Face cache
snapshot (``local_files_only`` — no network is ever used).
"""
from __future__ import annotations

import json
import os
from typing import Iterable, Optional

import torch


def _has_safetensors(d: str) -> bool:
    return os.path.isdir(d) and any(f.endswith(".safetensors") for f in os.listdir(d))


def resolve_checkpoint(model_id: Optional[str], model_path: Optional[str] = None) -> Optional[str]:
    """Directory holding ``config.json`` + ``*.safetensors`` for this model, or None
    (None means: random-init weights of the preset architecture)."""
    for cand in (model_path, model_id):
        if cand and os.path.isdir(cand) and _has_safetensors(cand):
            return cand
    if model_path:
        raise FileNotFoundError(f"model_path {model_path!r} has no *.safetensors files")
    if model_id and "/" in model_id and not os.path.exists(model_id):
        try:  # offline HF cache lookup only
            from huggingface_hub import snapshot_download

            d = snapshot_download(model_id, local_files_only=True, allow_patterns=["*.json", "*.safetensors"])
            if _has_safetensors(d):
                return d
        except Exception:
            return None
    return None


class CheckpointReader:
    """Name -> shard map over the safetensors files of one checkpoint directory."""

    def __init__(self, path: str):
        from safetensors import safe_open

        self.path = path
        self._open = safe_open
        idx = os.path.join(path, "model.safetensors.index.json")
        self.where: dict[str, str] = {}
        if os.path.exists(idx):
            with open(idx) as f:
                for name, fn in json.load(f)["weight_map"].items():
                    self.where[name] = os.path.join(path, fn)
        else:
            for fn in sorted(os.listdir(path)):
                if fn.endswith(".safetensors"):
                    full = os.path.join(path, fn)
                    with safe_open(full, framework="pt", device="cpu") as f:
                        for name in f.keys():
                            self.where[name] = full
        self._handles: dict[str, object] = {}
        self.bytes_read = 0

    def __contains__(self, name: str) -> bool:
        return name in self.where

    def names(self) -> Iterable[str]:
        return self.where.keys()

    def _h(self, name: str):
        fn = self.where[name]
        h = self._handles.get(fn)
        if h is None:
            h = self._handles[fn] = self._open(fn, framework="pt", device="cpu")
        return h

    def read(self, name: str, rows: Optional[tuple] = None, cols: Optional[tuple] = None) -> torch.Tensor:
        """Tensor ``name`` (optionally rows [a, b) / cols [a, b) only) as a CPU tensor."""
        sl = self._h(name).get_slice(name)
        if rows is None and cols is None:
            t = sl[:]
        elif cols is None:
            t = sl[rows[0]:rows[1]]
        elif rows is None:
            t = sl[:, cols[0]:cols[1]]
        else:
            t = sl[rows[0]:rows[1], cols[0]:cols[1]]
        self.bytes_read += t.numel() * t.element_size()
        return t

    def close(self) -> None:
        self._handles.clear()


def _put(dst: torch.Tensor, src: torch.Tensor) -> None:
    if tuple(dst.shape) != tuple(src.shape):
        raise ValueError(f"checkpoint tensor shape {tuple(src.shape)} != model slot {tuple(dst.shape)}")
    dst.copy_(src.to(dst.dtype), non_blocking=False)


def load_checkpoint(model, path: str, tp_rank: int = 0, tp: int = 1) -> dict:
    """Fill a ``LlamaModel`` (created with ``init="empty"``) from an HF checkpoint.

    ``model.cfg`` is the LOCAL config (per-rank heads / intermediate for TP);
    ``full`` is the checkpoint's.  Returns {"tensors": n, "bytes": b}."""
    model.norms_folded = False
    rd = CheckpointReader(path)
    c = model.cfg
    full = getattr(model, "full_cfg", c)
    hd = full.head_dim
    ql, kl = c.num_heads * hd, c.num_kv_heads * hd
    Il = c.intermediate_size
    q_rows = (tp_rank * ql, (tp_rank + 1) * ql)
    kv_rows = (tp_rank * kl, (tp_rank + 1) * kl)
    i_rows = (tp_rank * Il, (tp_rank + 1) * Il)
    n = 0
    for i, li in enumerate(range(model.layer_start, model.layer_end)):
        L = model.layers[i]
        p = f"model.layers.{li}."
        a = p + "self_attn."
        _put(L.qkv[:ql], rd.read(a + "q_proj.weight", rows=q_rows))
        _put(L.qkv[ql:ql + kl], rd.read(a + "k_proj.weight", rows=kv_rows))
        _put(L.qkv[ql + kl:], rd.read(a + "v_proj.weight", rows=kv_rows))
        n += 3
        if L.qkv_bias is not None:
            _put(L.qkv_bias[:ql], rd.read(a + "q_proj.bias", rows=q_rows))
            _put(L.qkv_bias[ql:ql + kl], rd.read(a + "k_proj.bias", rows=kv_rows))
            _put(L.qkv_bias[ql + kl:], rd.read(a + "v_proj.bias", rows=kv_rows))
            n += 3
        _put(L.o, rd.read(a + "o_proj.weight", cols=q_rows) if tp > 1 else rd.read(a + "o_proj.weight"))
        m = p + "mlp."
        if m + "gate_up_proj.weight" in rd:        # GLM-4: fused [gate; up]
            I = full.intermediate_size
            _put(L.gate_up[:Il], rd.read(m + "gate_up_proj.weight", rows=i_rows))
            _put(L.gate_up[Il:], rd.read(m + "gate_up_proj.weight", rows=(I + i_rows[0], I + i_rows[1])))
        else:
            _put(L.gate_up[:Il], rd.read(m + "gate_proj.weight", rows=i_rows))
            _put(L.gate_up[Il:], rd.read(m + "up_proj.weight", rows=i_rows))
        _put(L.down, rd.read(m + "down_proj.weight", cols=i_rows) if tp > 1 else rd.read(m + "down_proj.weight"))
        _put(L.in_norm, rd.read(p + "input_layernorm.weight"))
        _put(L.post_norm, rd.read(p + "post_attention_layernorm.weight"))
        n += 6
    if model.embed is not None:
        _put(model.embed, rd.read("model.embed_tokens.weight"))
        n += 1
    if model.has_head:
        _put(model.norm, rd.read("model.norm.weight"))
        n += 1
        if model.lm_head is not model.embed:
            if "lm_head.weight" in rd:
                _put(model.lm_head, rd.read("lm_head.weight"))
            else:   # tied checkpoint served by an untied slot (last stage without the embedding)
                _put(model.lm_head, rd.read("model.embed_tokens.weight"))
            n += 1
    out = {"tensors": n, "bytes": rd.bytes_read, "path": path}
    rd.close()
    return out
