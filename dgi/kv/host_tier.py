"""Pinned host-memory KV tier (L2 of the reference's tiered cache,
worker/distributed/kv_cache.py:331-531).

Evicted radix-cache pages and the pages of preempted sequences are not dropped:
their KV (every local layer, K and V) moves to page-locked host memory and comes
back by DMA when a prefix hit or a re-admission needs it, instead of being
recomputed by a prefill.

Layout and movement (round 6):

* Host slots are block-major ``[capacity, L, 2, n_kv, bs, hd]``: one slot is one
  page of every layer, contiguous (5.2 MB for Llama-3-70B at bs=16).  The GPU side
  gathers / scatters straight in that layout (``kv_gather`` / ``kv_scatter`` with
  ``block_major``), so there is no permute pass, and slots are handed out lowest
  first so a spill or restore of n pages is usually ONE contiguous run = one
  ``hipMemcpyAsync`` (``runs``) instead of n.
* Both directions run on the tier's copy stream.  A spill gathers on the compute
  stream (ordered after the kernels that wrote the pages) and the copy stream
  waits for it; a restore waits for the compute stream once (the fresh pages'
  previous users), then H2D + scatter on the copy stream, and returns an event
  that the scheduler hangs on the request (``Request.kv_ready``).  The compute
  stream waits for it (``ModelRunner.gate_rows``) only before the first forward
  whose batch contains that request: a GPU-side wait, no host synchronisation.
* Restores therefore run ONE STEP AHEAD of their use: a swapped-out sequence
  re-admitted while step N is scheduled joins step N+1's decode rows, so its DMA
  overlaps step N's forward; ``Scheduler._prefetch`` also starts the restores of
  the sequences at the head of the waiting queue when the step's token budget
  admits no more.  Only a prefix hit on host-resident radix pages is read by the
  step that admits it and gates that step.

The copy stream is FIFO, so a slot released right after its restore was issued
can be refilled by a later spill without a host wait.
"""
from __future__ import annotations

import heapq
from typing import Optional

import torch

from dgi import ops
from dgi.kv.block_pool import BlockPool


def runs(slots: list) -> list:
    """Maximal runs of consecutive slot ids as (index into ``slots``, first slot, length)."""
    out = []
    i = 0
    while i < len(slots):
        j = i + 1
        while j < len(slots) and slots[j] == slots[j - 1] + 1:
            j += 1
        out.append((i, slots[i], j - i))
        i = j
    return out


class HostKVTier:
    def __init__(self, pool: BlockPool, capacity_blocks: int, pin: Optional[bool] = None):
        self.pool = pool
        self.capacity = int(capacity_blocks)
        L, two, _nb, nkv, bs, hd = pool.kv.shape
        self.page_shape = (L, two, nkv, bs, hd)
        dev = pool.kv.device
        pin = (dev.type == "cuda") if pin is None else pin
        self.host = torch.empty((self.capacity,) + self.page_shape, dtype=pool.kv.dtype, pin_memory=pin)
        self._free = list(range(self.capacity))          # min-heap: lowest slots first (contiguous runs)
        if dev.type == "cuda":
            from dgi.utils.streams import named_stream
            self.copy_stream = named_stream("kv_host_copy", dev)
        else:
            self.copy_stream = None
        self.stats = {"spilled": 0, "restored": 0, "dropped": 0, "spill_bytes": 0, "restore_bytes": 0,
                      "spill_dmas": 0, "restore_dmas": 0, "prefetched": 0, "gates": 0}

    @property
    def num_free(self) -> int:
        return len(self._free)

    def page_bytes(self) -> int:
        return self.host[0].numel() * self.host.element_size()

    def alloc(self, n: int) -> list:
        if n > len(self._free):
            raise RuntimeError("host KV tier full")
        return [heapq.heappop(self._free) for _ in range(n)]

    def release(self, slots) -> None:
        for s in slots:
            heapq.heappush(self._free, s)

    # ------------------------------------------------------------------ movement
    def spill(self, blocks: list) -> list:
        """Copy GPU pages -> host slots (async on the copy stream).  Returns slots."""
        if not blocks:
            return []
        slots = self.alloc(len(blocks))
        dev = self.pool.kv.device
        ids = torch.tensor(blocks, dtype=torch.int32, device=dev)
        staged = ops.kv_gather(self.pool.kv, ids, block_major=True)        # [n, L, 2, ...]
        rr = runs(slots)
        if self.copy_stream is not None:
            self.copy_stream.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(self.copy_stream):
                for i, s0, k in rr:
                    self.host[s0:s0 + k].copy_(staged[i:i + k], non_blocking=True)
                staged.record_stream(self.copy_stream)
        else:
            for i, s0, k in rr:
                self.host[s0:s0 + k].copy_(staged[i:i + k])
        self.stats["spilled"] += len(blocks)
        self.stats["spill_dmas"] += len(rr)
        self.stats["spill_bytes"] += len(blocks) * self.page_bytes()
        return slots

    def restore(self, slots: list, blocks: list, prefetch: bool = False):
        """Copy host slots -> GPU pages ``blocks``: H2D + scatter on the copy stream.  Returns
        the event a forward reading ``blocks`` must wait for (None on CPU).  The slots may be
        released as soon as this returns."""
        if not slots:
            return None
        ev = None
        dev = self.pool.kv.device
        rr = runs(slots)
        if self.copy_stream is not None:
            cur = torch.cuda.current_stream(dev)
            # the fresh pages' previous users (kernels already enqueued on the compute stream)
            self.copy_stream.wait_stream(cur)
            with torch.cuda.stream(self.copy_stream):
                staged = torch.empty((len(slots),) + self.page_shape, dtype=self.host.dtype, device=dev)
                for i, s0, k in rr:
                    staged[i:i + k].copy_(self.host[s0:s0 + k], non_blocking=True)
                ops.kv_scatter(self.pool.kv, torch.tensor(blocks, dtype=torch.int32, device=dev), staged,
                               block_major=True)
                ev = torch.cuda.Event()
                ev.record(self.copy_stream)
        else:
            staged = torch.cat([self.host[s0:s0 + k] for _i, s0, k in rr]).to(dev)
            ops.kv_scatter(self.pool.kv, torch.tensor(blocks, dtype=torch.int32, device=dev), staged,
                           block_major=True)
        self.stats["restored"] += len(slots)
        self.stats["restore_dmas"] += len(rr)
        self.stats["restore_bytes"] += len(slots) * self.page_bytes()
        if prefetch:
            self.stats["prefetched"] += len(slots)
        return ev

    def synchronize(self) -> None:
        """Host wait for every copy issued so far (tests, teardown)."""
        if self.copy_stream is not None:
            self.copy_stream.synchronize()
