"""Paged KV block pool (SURVEY §2.2 ``PagedKVCache``/``KVCachePool`` equivalent).

Physical storage is ONE device tensor ``[L_local, 2, num_blocks, n_kv, bs, hd]``
(bf16) so a block id names the page of every local layer: a sequence needs
``ceil(len/bs)`` ids, not ``L*ceil(len/bs)`` as in the reference's per-layer
pools (worker/distributed/kv_cache.py:250-323).  Allocation is an O(1)
free-list pop with reference counts for prefix sharing (radix cache,
copy-on-write).  Works on CPU too (the reference only allocated on CUDA,
kv_cache.py:130-139, which its own tests contradict).

Sizing for MI355X: ``num_blocks_for_budget`` turns a byte budget (288 GB HBM
minus weights and activation workspace, times ``kv_fraction``) into a block
count.
"""
from __future__ import annotations

from typing import Iterable, Optional

import torch


class OutOfBlocks(RuntimeError):
    pass


def num_blocks_for_budget(budget_bytes: int, num_layers: int, num_kv_heads: int, head_dim: int,
                          block_size: int, dtype_bytes: int = 2) -> int:
    per_block = 2 * num_layers * num_kv_heads * block_size * head_dim * dtype_bytes
    return max(0, int(budget_bytes // per_block))


class BlockPool:
    def __init__(self, num_blocks: int, block_size: int = 16, num_layers: int = 1, num_kv_heads: int = 1,
                 head_dim: int = 128, dtype=torch.bfloat16, device="cpu", allocate: bool = True):
        self.num_blocks = num_blocks
        self.block_size = block_size
        self.num_layers = num_layers
        self.num_kv_heads = num_kv_heads
        self.head_dim = head_dim
        self.dtype = dtype
        self.device = torch.device(device)
        self.kv: Optional[torch.Tensor] = None
        if allocate:
            self.kv = torch.zeros(num_layers, 2, num_blocks, num_kv_heads, block_size, head_dim,
                                  dtype=dtype, device=self.device)
        # block 0 is reserved as a scratch/padding page (graph padding rows write there)
        self._free: list[int] = list(range(num_blocks - 1, 0, -1))
        self.ref = [0] * num_blocks
        self.ref[0] = 1 << 30
        self.evictor = None  # callable(n) -> frees >= n blocks (radix cache LRU)
        self.stats = {"allocs": 0, "frees": 0, "evictions": 0, "cow": 0}

    # ------------------------------------------------------------------ state
    @property
    def num_free(self) -> int:
        return len(self._free)

    @property
    def num_used(self) -> int:
        return self.num_blocks - 1 - len(self._free)

    def page_bytes(self) -> int:
        return 2 * self.num_layers * self.num_kv_heads * self.block_size * self.head_dim * \
            torch.tensor([], dtype=self.dtype).element_size()

    def can_allocate(self, n: int) -> bool:
        return n <= len(self._free) or (self.evictor is not None and n <= len(self._free) + self.evictor(0))

    # ------------------------------------------------------------------ alloc/free
    def allocate(self, n: int) -> list[int]:
        if n > len(self._free) and self.evictor is not None:
            self.evictor(n - len(self._free))
        if n > len(self._free):
            raise OutOfBlocks(f"need {n} blocks, {len(self._free)} free")
        out = [self._free.pop() for _ in range(n)]
        for b in out:
            self.ref[b] = 1
        self.stats["allocs"] += n
        return out

    def incref(self, ids: Iterable[int]) -> None:
        for b in ids:
            self.ref[b] += 1

    def free(self, ids: Iterable[int]) -> None:
        for b in ids:
            r = self.ref[b] - 1
            self.ref[b] = r
            if r == 0:
                self._free.append(b)
                self.stats["frees"] += 1
            elif r < 0:
                raise RuntimeError(f"double free of block {b}")

    def cow(self, block: int) -> int:
        """Copy-on-write: give the caller a private copy of a shared block."""
        if self.ref[block] <= 1:
            return block
        (nb,) = self.allocate(1)
        if self.kv is not None:
            from dgi import ops
            dev = self.kv.device
            ops.kv_copy(self.kv, torch.tensor([block], dtype=torch.int32, device=dev),
                        torch.tensor([nb], dtype=torch.int32, device=dev))
        self.free([block])
        self.stats["cow"] += 1
        return nb

    # ------------------------------------------------------------------ views
    def layer_kv(self, layer: int):
        return self.kv[layer, 0], self.kv[layer, 1]
