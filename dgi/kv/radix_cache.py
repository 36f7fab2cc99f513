"""RadixAttention-style prefix cache over paged KV blocks.

The reference keeps a flat prefix-hash index of whole KV tensors
(worker/distributed/kv_cache.py:373-445) and evicts blocks that owners still
reference (Appendix E-12).  Here a radix tree whose edges are full KV blocks
(``block_size`` token ids each) maps token prefixes to block ids:

* ``match(tokens)`` returns the longest cached block chain and pins it
  (``lock``) so eviction cannot free pages an in-flight request reads;
* ``insert(tokens, blocks)`` adopts a finished (or prefilled) sequence's full
  blocks, taking its own pool reference;
* eviction frees least-recently-used *unpinned leaves* only, so a shared
  prefix is never freed under a reader.

Block granularity (not token granularity) matches the paged attention
kernels: a hit skips whole pages of prefill and the partially filled tail
page is always private to its sequence (no copy-on-write needed for it).
"""
from __future__ import annotations

import itertools
import time
from typing import Optional

from dgi.kv.block_pool import BlockPool


class _Node:
    __slots__ = ("key", "block", "children", "parent", "last", "lock")

    def __init__(self, key, block, parent):
        self.key = key
        self.block = block
        self.children: dict = {}
        self.parent = parent
        self.last = time.monotonic()
        self.lock = 0


class RadixCache:
    def __init__(self, pool: BlockPool):
        self.pool = pool
        self.bs = pool.block_size
        self.root = _Node(None, -1, None)
        self.num_nodes = 0
        self.hits_tokens = 0
        self.query_tokens = 0
        self.evicted = 0
        self._clock = itertools.count()
        pool.evictor = self.evict

    # ------------------------------------------------------------------ lookup
    def match(self, tokens: list[int], lock: bool = True) -> tuple[list[int], list]:
        """Longest prefix of full blocks.  Returns (block ids, node path)."""
        node = self.root
        blocks, path = [], []
        bs = self.bs
        now = time.monotonic()
        for i in range(0, len(tokens) - bs + 1, bs):
            key = tuple(tokens[i:i + bs])
            child = node.children.get(key)
            if child is None:
                break
            child.last = now
            blocks.append(child.block)
            path.append(child)
            node = child
        if lock:
            for n in path:
                n.lock += 1
            self.pool.incref(blocks)
        self.query_tokens += len(tokens)
        self.hits_tokens += len(blocks) * bs
        return blocks, path

    def release(self, path: list) -> None:
        for n in path:
            n.lock -= 1

    # ------------------------------------------------------------------ insert
    def insert(self, tokens: list[int], blocks: list[int]) -> int:
        """Adopt the full blocks of ``tokens``; returns how many were new."""
        node = self.root
        bs = self.bs
        n_full = min(len(tokens) // bs, len(blocks))
        new = 0
        now = time.monotonic()
        for j in range(n_full):
            key = tuple(tokens[j * bs:(j + 1) * bs])
            child = node.children.get(key)
            if child is None:
                child = _Node(key, blocks[j], node)
                node.children[key] = child
                self.pool.incref([blocks[j]])
                self.num_nodes += 1
                new += 1
            child.last = now
            node = child
        return new

    # ------------------------------------------------------------------ evict
    def _evictable_leaves(self):
        out = []
        stack = [self.root]
        while stack:
            n = stack.pop()
            for c in n.children.values():
                if c.children:
                    stack.append(c)
                elif c.lock == 0:
                    out.append(c)
        return out

    def evict(self, n: int) -> int:
        """Free >= n blocks from unpinned LRU leaves.  n == 0: report capacity."""
        if n == 0:
            return sum(1 for c in self._evictable_leaves() if self.pool.ref[c.block] == 1)
        freed = 0
        while freed < n:
            leaves = [c for c in self._evictable_leaves()]
            if not leaves:
                break
            leaves.sort(key=lambda c: c.last)
            progressed = False
            for c in leaves:
                if freed >= n:
                    break
                del c.parent.children[c.key]
                self.num_nodes -= 1
                if self.pool.ref[c.block] == 1:
                    freed += 1
                self.pool.free([c.block])
                self.evicted += 1
                progressed = True
            if not progressed:
                break
        self.pool.stats["evictions"] += freed
        return freed

    def hit_rate(self) -> float:
        return self.hits_tokens / self.query_tokens if self.query_tokens else 0.0

    def reset(self) -> None:
        stack = [self.root]
        while stack:
            n = stack.pop()
            for c in n.children.values():
                stack.append(c)
                self.pool.free([c.block])
        self.root = _Node(None, -1, None)
        self.num_nodes = 0
