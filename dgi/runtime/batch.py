"""Per-step attention metadata shared by every layer of one forward pass.

A step's token rows are ordered ``[decode rows | prefill/chunk rows]``: the
first ``num_decode`` rows are single-token decode rows (one per sequence,
paged_decode kernel), the rest are packed prefill chunks (paged_prefill
kernel, which also serves prefix-cache hits and EAGLE tree verification).
All index tensors are int32 on the model device and are built once per step
by the model runner (one pinned H2D copy), then read by all layers.
"""
from __future__ import annotations

import dataclasses
from typing import Optional

import torch


@dataclasses.dataclass
class AttnMeta:
    positions: torch.Tensor                 # [T] int32 rotary positions
    slot_mapping: torch.Tensor              # [T] int32 KV slot (block*bs+off), -1 = don't write
    num_decode: int = 0
    # decode part (rows [0, num_decode))
    dec_block_tables: Optional[torch.Tensor] = None   # [Bd, max_blocks] int32
    dec_context_lens: Optional[torch.Tensor] = None   # [Bd] int32 (including the new token)
    dec_max_splits: int = 1
    dec_part_size: int = 1 << 20
    dec_workspace: Optional[tuple] = None
    # prefill part (rows [num_decode, T))
    num_prefill_tokens: int = 0
    pre_block_tables: Optional[torch.Tensor] = None   # [Bp, max_blocks] int32
    pre_cu_seqlens: Optional[torch.Tensor] = None     # [Bp+1] int32, relative to num_decode
    pre_context_lens: Optional[torch.Tensor] = None   # [Bp] int32 (prefix + this chunk)
    pre_tiles: Optional[torch.Tensor] = None          # [n_tiles, 2] int32
    tree_mask: Optional[torch.Tensor] = None          # [Bp, 64] int64 ancestor bits (EAGLE verify)
    tree_n: int = 0
    # rows whose hidden state feeds the LM head (None = all rows)
    logits_indices: Optional[torch.Tensor] = None

    @property
    def num_tokens(self) -> int:
        return int(self.positions.shape[0])
