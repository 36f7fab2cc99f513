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

With a ``HostKVTier`` attached, eviction *spills* LRU pages to pinned host
memory instead of dropping them (the node stays in the tree with
``block == -1``); a later match restores them into fresh GPU pages.  Only
when the host tier is full are host-resident leaves dropped.
"""
from __future__ import annotations

import itertools
import time
from typing import Optional

from dgi.kv.block_pool import BlockPool


class _Node:
    __slots__ = ("key", "block", "host", "children", "parent", "last", "lock")

    def __init__(self, key, block, parent):
        self.key = key
        self.block = block      # GPU page id, -1 while the page lives in the host tier
        self.host = -1          # host-tier slot
        self.children: dict = {}
        self.parent = parent
        self.last = time.monotonic()
        self.lock = 0


class RadixCache:
    def __init__(self, pool: BlockPool, host_tier=None):
        self.pool = pool
        self.host = host_tier
        self.host_hits_blocks = 0
        self.restore_event = None       # event of the last host-tier restore (``take_restore_event``)
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
        if any(n.block < 0 for n in path):
            path = self._restore(path)
            blocks = [n.block for n in path]
        if lock:
            for n in path:
                n.lock += 1
            self.pool.incref(blocks)
        self.query_tokens += len(tokens)
        self.hits_tokens += len(blocks) * bs
        return blocks, path

    def _restore(self, path: list) -> list:
        """Bring host-resident pages of ``path`` back to the GPU (truncating the
        match at the first page that cannot be restored)."""
        for n in path:
            n.lock += 1                      # keep the path out of eviction while allocating
        try:
            need = [n for n in path if n.block < 0]
            try:
                fresh = self.pool.allocate(len(need))
            except Exception:
                cut = path.index(need[0])
                return path[:cut]
            self.restore_event = self.host.restore([n.host for n in need], fresh)
            self.host.release([n.host for n in need])
            for n, b in zip(need, fresh):
                n.block, n.host = b, -1
            self.host_hits_blocks += len(need)
            return path
        finally:
            for n in path:
                n.lock -= 1

    def take_restore_event(self):
        """The event of the restore the last ``match`` issued (None if it issued none)."""
        ev, self.restore_event = self.restore_event, None
        return ev

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
            elif child.block < 0:             # page was spilled: adopt the recomputed copy
                child.block = blocks[j]
                self.pool.incref([blocks[j]])
                self.host.release([child.host])
                child.host = -1
            child.last = now
            node = child
        return new

    def insert_locked(self, tokens: list[int], blocks: list[int]) -> list:
        """``insert`` and return the node path of the inserted full blocks, locked (the caller
        releases it): a request publishes its prompt pages when its prefill completes and
        keeps them pinned while it decodes."""
        self.insert(tokens, blocks)
        node, path = self.root, []
        bs = self.bs
        for j in range(min(len(tokens) // bs, len(blocks))):
            node = node.children.get(tuple(tokens[j * bs:(j + 1) * bs]))
            if node is None:
                break
            node.lock += 1
            path.append(node)
        return path

    # ------------------------------------------------------------------ evict
    def _evictable_leaves(self):
        """Unpinned GPU-resident nodes none of whose children hold a GPU page."""
        out = []
        stack = [self.root]
        while stack:
            n = stack.pop()
            for c in n.children.values():
                if c.children:
                    stack.append(c)
                if c.block >= 0 and c.lock == 0 and all(g.block < 0 for g in c.children.values()):
                    out.append(c)
        return out

    def _drop_host_leaves(self, n: int) -> int:
        """Free host slots by deleting LRU host-resident leaves."""
        cands = []
        stack = [self.root]
        while stack:
            x = stack.pop()
            for c in x.children.values():
                stack.append(c)
                if c.block < 0 and not c.children and c.lock == 0:
                    cands.append(c)
        cands.sort(key=lambda c: c.last)
        dropped = 0
        for c in cands[:n]:
            del c.parent.children[c.key]
            self.host.release([c.host])
            self.num_nodes -= 1
            dropped += 1
        self.host.stats["dropped"] += dropped
        return dropped

    def _evictable_total(self) -> int:
        """GPU pages eviction can free by repeated leaf eviction: every unpinned node whose page
        only the cache holds and whose GPU-resident descendants all qualify too (evicting the
        current leaves turns their parents into leaves).  Counting the current leaves alone
        under-reports a deep tree, and an admission that needs more pages than that waits
        forever while the cache holds them."""
        total = 0
        # post-order over the tree: a node qualifies iff it and its whole GPU-resident subtree do
        stack = [(self.root, False)]
        ok: dict = {}
        while stack:
            n, done = stack.pop()
            if not done:
                stack.append((n, True))
                stack.extend((c, False) for c in n.children.values())
                continue
            sub = all(ok[id(c)] for c in n.children.values())
            if n is self.root:
                break
            if n.block < 0:
                ok[id(n)] = sub
            else:
                ok[id(n)] = sub and n.lock == 0 and (self.pool.ref[n.block] == 1 or self.host is None)
                if ok[id(n)] and self.pool.ref[n.block] == 1:
                    total += 1
        return total

    def evict(self, n: int) -> int:
        """Free >= n GPU blocks from unpinned LRU leaves.  n == 0: report capacity."""
        if n == 0:
            return self._evictable_total()
        freed = 0
        while freed < n:
            leaves = [c for c in self._evictable_leaves() if self.pool.ref[c.block] == 1] if self.host is not None \
                else [c for c in self._evictable_leaves()]
            if not leaves:
                break
            leaves.sort(key=lambda c: c.last)
            victims = leaves[: max(1, n - freed)]
            if self.host is not None:
                if self.host.num_free < len(victims):
                    self._drop_host_leaves(len(victims) - self.host.num_free)
                victims = victims[: self.host.num_free]
            if not victims:
                # host tier cannot take more: fall back to dropping GPU leaves
                victims = [c for c in leaves if not c.children][: max(1, n - freed)]
                if not victims:
                    break
                for c in victims:
                    del c.parent.children[c.key]
                    self.num_nodes -= 1
                    if self.pool.ref[c.block] == 1:
                        freed += 1
                    self.pool.free([c.block])
                    self.evicted += 1
                continue
            if self.host is not None:
                slots = self.host.spill([c.block for c in victims])
                for c, s_ in zip(victims, slots):
                    self.pool.free([c.block])
                    c.block, c.host = -1, s_
                    freed += 1
                    self.evicted += 1
            else:
                for c in victims:
                    del c.parent.children[c.key]
                    self.num_nodes -= 1
                    if self.pool.ref[c.block] == 1:
                        freed += 1
                    self.pool.free([c.block])
                    self.evicted += 1
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
                if c.block >= 0:
                    self.pool.free([c.block])
                elif self.host is not None:
                    self.host.release([c.host])
        self.root = _Node(None, -1, None)
        self.num_nodes = 0
