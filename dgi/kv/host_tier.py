"""Pinned host-memory KV tier (L2 of the reference's tiered cache,
worker/distributed/kv_cache.py:331-531).

Evicted radix-cache pages are not dropped: their KV (every local layer, K
and V) is gathered on the GPU (``kv_gather`` HIP kernel) into a staging
buffer and copied with async DMA (``hipMemcpyAsync`` via ``copy_(...,
non_blocking=True)`` into page-locked memory) on a dedicated copy stream;
a later prefix hit copies the pages back and scatters them into freshly
allocated blocks (``kv_scatter``) instead of recomputing the prefill.

Host layout is block-major ``[capacity, L, 2, n_kv, bs, hd]`` so one page is
one contiguous DMA (5.2 MB for Llama-3-70B at bs=16).  A 512-token prefix
(32 pages) restores in ~3 ms over the host link, versus ~50 ms to recompute
its prefill on 70B.
"""
from __future__ import annotations

from typing import Optional

import torch

from dgi import ops
from dgi.kv.block_pool import BlockPool


class HostKVTier:
    def __init__(self, pool: BlockPool, capacity_blocks: int, pin: Optional[bool] = None):
        self.pool = pool
        self.capacity = int(capacity_blocks)
        L, two, _nb, nkv, bs, hd = pool.kv.shape
        self.page_shape = (L, two, nkv, bs, hd)
        dev = pool.kv.device
        pin = (dev.type == "cuda") if pin is None else pin
        self.host = torch.empty((self.capacity,) + self.page_shape, dtype=pool.kv.dtype, pin_memory=pin)
        self._free = list(range(self.capacity - 1, -1, -1))
        if dev.type == "cuda":
            from dgi.utils.streams import named_stream
            self.copy_stream = named_stream("kv_host_copy", dev)
        else:
            self.copy_stream = None
        self.stats = {"spilled": 0, "restored": 0, "dropped": 0, "spill_bytes": 0, "restore_bytes": 0}

    @property
    def num_free(self) -> int:
        return len(self._free)

    def page_bytes(self) -> int:
        return self.host[0].numel() * self.host.element_size()

    def alloc(self, n: int) -> list:
        if n > len(self._free):
            raise RuntimeError("host KV tier full")
        return [self._free.pop() for _ in range(n)]

    def release(self, slots) -> None:
        self._free.extend(slots)

    # ------------------------------------------------------------------ movement
    def spill(self, blocks: list) -> list:
        """Copy GPU pages -> host slots (async on the copy stream).  Returns slots."""
        if not blocks:
            return []
        slots = self.alloc(len(blocks))
        dev = self.pool.kv.device
        ids = torch.tensor(blocks, dtype=torch.int32, device=dev)
        staged = ops.kv_gather(self.pool.kv, ids).permute(2, 0, 1, 3, 4, 5).contiguous()   # [n, L, 2, ...]
        if self.copy_stream is not None:
            self.copy_stream.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(self.copy_stream):
                for i, s in enumerate(slots):
                    self.host[s].copy_(staged[i], non_blocking=True)
                staged.record_stream(self.copy_stream)
        else:
            for i, s in enumerate(slots):
                self.host[s].copy_(staged[i])
        self.stats["spilled"] += len(blocks)
        self.stats["spill_bytes"] += len(blocks) * self.page_bytes()
        return slots

    def restore(self, slots: list, blocks: list) -> None:
        """Copy host slots -> GPU pages ``blocks`` (ordered on the compute stream)."""
        if not slots:
            return
        dev = self.pool.kv.device
        if self.copy_stream is not None:
            # the spill of these slots may still be in flight on the copy stream
            torch.cuda.current_stream(dev).wait_stream(self.copy_stream)
        staged = torch.empty((len(slots),) + self.page_shape, dtype=self.host.dtype, device=dev)
        for i, s in enumerate(slots):
            staged[i].copy_(self.host[s], non_blocking=True)
        buf = staged.permute(1, 2, 0, 3, 4, 5).contiguous()                                  # [L, 2, n, ...]
        ops.kv_scatter(self.pool.kv, torch.tensor(blocks, dtype=torch.int32, device=dev), buf)
        self.stats["restored"] += len(slots)
        self.stats["restore_bytes"] += len(slots) * self.page_bytes()
