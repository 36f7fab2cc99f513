"""Tensor parallelism inside one node (the reference only forwarded
``tensor_parallel_size`` / ``tp_size`` to vLLM/SGLang, llm_vllm.py:56,66,
llm_sglang.py:61,71).

Megatron-style sharding of each Llama layer over ``tp`` GPUs:

* QKV and gate|up are column-parallel (each rank owns ``nh/tp`` query heads,
  ``nkv/tp`` KV heads and ``I/tp`` MLP columns — so each rank's paged KV pool
  holds only its own KV heads);
* O and down are row-parallel; their partial outputs are summed with ONE
  RCCL all-reduce each (``[T, H]`` bf16) — two per layer;
* embedding, norms and the LM head are replicated, so every rank samples the
  same token and the engines stay in lock-step (SPMD: every rank runs the
  same scheduler on the same requests).

On MI355X a 70B model fits on one GPU, so TP is a latency tool (per-token
decode time falls with tp while weight traffic per GPU shrinks); xGMI is
point-to-point, so the all-reduce of a decode step (T x 16 KiB) is
latency-bound and RCCL picks its one-shot/direct algorithm for it.
"""
from __future__ import annotations

import dataclasses
import math
from typing import Optional

import torch
import torch.distributed as dist

from dgi.engine import EngineConfig, LLMEngine, engine_block_budget
from dgi.models.config import ModelConfig, get_config
from dgi.models.llama import LlamaLayerWeights, LlamaModel, _rand


def tp_local_config(cfg: ModelConfig, tp: int) -> ModelConfig:
    if cfg.num_heads % tp or cfg.num_kv_heads % tp or cfg.intermediate_size % tp:
        raise ValueError(f"{cfg.name}: heads {cfg.num_heads}/{cfg.num_kv_heads} and intermediate "
                         f"{cfg.intermediate_size} must be divisible by tp={tp}")
    return dataclasses.replace(cfg, num_heads=cfg.num_heads // tp, num_kv_heads=cfg.num_kv_heads // tp,
                               intermediate_size=cfg.intermediate_size // tp)


class TPLlamaModel(LlamaModel):
    """Rank ``tp_rank`` of a ``tp``-way tensor-parallel Llama (weights bit-identical
    to the slices of the TP=1 random init)."""

    def __init__(self, cfg: ModelConfig, device, dtype, tp_rank: int, tp: int, group=None, seed: int = 0,
                 checkpoint: Optional[str] = None):
        self.full_cfg = cfg
        self.tp_rank, self.tp = tp_rank, tp
        self.group = group
        super().__init__(tp_local_config(cfg, tp), device, dtype, seed=seed, checkpoint=checkpoint)
        self.reduce = self._all_reduce if tp > 1 else None

    def _all_reduce(self, h: torch.Tensor) -> None:
        if h.device.type == "cpu" and h.dtype == torch.bfloat16:   # gloo reduces fp32
            f = h.float()
            dist.all_reduce(f, group=self.group)
            h.copy_(f)
        else:
            dist.all_reduce(h, group=self.group)

    def _init_random(self, seed: int):
        full, c, dev, dt = self.full_cfg, self.cfg, self.device, self.dtype
        H, I, Il = full.hidden_size, full.intermediate_size, c.intermediate_size
        r = self.tp_rank
        hd = full.head_dim
        q0, q1 = r * c.num_heads * hd, (r + 1) * c.num_heads * hd
        k0 = full.q_size + r * c.num_kv_heads * hd
        v0 = full.q_size + full.kv_size + r * c.num_kv_heads * hd
        kl = c.num_kv_heads * hd
        std = 0.02
        gen = torch.Generator(device=dev)
        for li in range(self.layer_start, self.layer_end):
            gen.manual_seed(seed * 1000003 + li * 7919 + 1)
            ln1 = 1.0 + 0.1 * _rand((H,), gen, dev, torch.float32, 1.0)
            qkv = _rand((full.qkv_size, H), gen, dev, dt, std)
            o = _rand((H, full.q_size), gen, dev, dt, std / math.sqrt(2 * full.num_layers))
            ln2 = 1.0 + 0.1 * _rand((H,), gen, dev, torch.float32, 1.0)
            gu = _rand((2 * I, H), gen, dev, dt, std)
            down = _rand((H, I), gen, dev, dt, std / math.sqrt(2 * full.num_layers))
            bias = _rand((full.qkv_size,), gen, dev, dt, std) if full.qkv_bias else None
            bias_l = None if bias is None else torch.cat([bias[q0:q1], bias[k0:k0 + kl], bias[v0:v0 + kl]])
            qkv_l = torch.cat([qkv[q0:q1], qkv[k0:k0 + kl], qkv[v0:v0 + kl]]).contiguous()
            o_l = o[:, q0:q1].contiguous()
            gu_l = torch.cat([gu[r * Il:(r + 1) * Il], gu[I + r * Il:I + (r + 1) * Il]]).contiguous()
            down_l = down[:, r * Il:(r + 1) * Il].contiguous()
            del qkv, o, gu, down
            self.layers.append(LlamaLayerWeights(ln1.to(dt), qkv_l, o_l, ln2.to(dt), gu_l, down_l, bias_l))
        gen.manual_seed(seed * 1000003 + 17)
        emb = _rand((full.vocab_size, H), gen, dev, dt, 1.0)
        self.embed = emb
        gen.manual_seed(seed * 1000003 + 23)
        self.norm = (1.0 + 0.1 * _rand((H,), gen, dev, torch.float32, 1.0)).to(dt)
        self.lm_head = emb if full.tie_embeddings else _rand((full.vocab_size, H), gen, dev, dt, std)


class TPEngine(LLMEngine):
    """SPMD engine: one per TP rank, all fed the same requests in the same order."""

    def __init__(self, cfg: EngineConfig, tp_rank: int, tp: int, group=None, model_cfg: Optional[ModelConfig] = None):
        from dgi.models.weights import resolve_checkpoint
        ckpt = resolve_checkpoint(cfg.model, cfg.model_path)
        full = model_cfg or get_config(ckpt or cfg.model)
        full.max_position = max(full.max_position, cfg.max_model_len)
        dev = torch.device(cfg.device)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        model = TPLlamaModel(full, dev, cfg.dtype, tp_rank, tp, group, seed=cfg.seed, checkpoint=ckpt)
        cfg = dataclasses.replace(cfg, device=str(dev))
        if tp > 1:
            # every rank must hold the same page count (block ids are shared): agree on the minimum
            nb = engine_block_budget(cfg, model.cfg, model.num_local_layers, dev)
            t = torch.tensor([nb], dtype=torch.int64, device=dev if dev.type == "cuda" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
            cfg = dataclasses.replace(cfg, num_blocks=int(t.item()))
        super().__init__(cfg, model_cfg=model.cfg, model=model)
        self.tp_rank, self.tp = tp_rank, tp
        self.full_cfg = full
