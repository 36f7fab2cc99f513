"""KV memory: the reference-compatible page API and the native pool/radix cache.

Part 1 mirrors the behaviours the reference checks in
tests/test_worker_distributed_kv_cache.py (CacheLocation, CacheBlock,
PagedKVCache alloc/free/share/LRU, KVCachePool sequences with rollback,
DistributedKVCacheManager tiers, Redis key format, stats) — on CPU, which the
reference's own tests assume but its implementation did not allow (E-9).

Part 2 covers what the serving engine actually uses: ``dgi.kv.BlockPool``
(one id spans every layer, ref counts, copy-on-write) and ``RadixCache``
(block-granular prefix sharing with LRU leaf eviction).
"""
import asyncio
from unittest.mock import AsyncMock

import pytest
import torch

from worker.distributed.kv_cache import (CacheBlock, CacheLocation, DistributedKVCacheManager, KVCachePool,
                                         PagedKVCache)
from dgi.kv.block_pool import BlockPool, OutOfBlocks, num_blocks_for_budget
from dgi.kv.radix_cache import RadixCache


def _paged(max_blocks=10, **kw):
    return PagedKVCache(num_layers=4, num_heads=8, head_dim=64, block_size=16, max_blocks=max_blocks, device="cpu",
                        dtype=kw.get("dtype", torch.float32))


def _mgr(**kw):
    args = dict(num_layers=4, num_heads=8, head_dim=64, gpu_cache_blocks=10, cpu_cache_gb=0.001, redis_client=None,
                block_size=16, device="cpu", dtype=torch.float32)
    args.update(kw)
    return DistributedKVCacheManager(**args)


# ============================================================================= reference-compatible API

def test_cache_location_members():
    assert [c.value for c in CacheLocation] == ["gpu", "cpu", "redis", "remote"]


def test_cache_block_defaults():
    b = CacheBlock(block_id="x")
    assert (b.block_size, b.keys, b.values, b.layer_idx, b.num_tokens, b.ref_count, b.prefix_hash) == \
        (16, None, None, 0, 0, 1, "")
    assert b.location is CacheLocation.GPU


def test_cache_block_custom_and_fullness():
    k = torch.zeros(2, 32, 8)
    b = CacheBlock(block_id="c", block_size=32, keys=k, values=k, layer_idx=5, num_tokens=10, ref_count=2,
                   prefix_hash="abc", location=CacheLocation.CPU)
    assert b.keys is k and b.location is CacheLocation.CPU and b.is_shared
    assert not b.is_full
    b.num_tokens = 32
    assert b.is_full
    b.num_tokens = 40
    assert b.is_full


def test_cache_block_refs_and_touch():
    b = CacheBlock(block_id="r")
    b.add_ref()
    b.add_ref()
    assert b.ref_count == 3
    assert [b.remove_ref(), b.remove_ref(), b.remove_ref(), b.remove_ref()] == [2, 1, 0, 0]
    t = b.last_access
    import time
    time.sleep(0.002)
    b.touch()
    assert b.last_access > t


def test_paged_cache_init_and_stats():
    c = _paged()
    assert (c.num_layers, c.num_heads, c.head_dim, c.block_size, c.max_blocks, c.device) == (4, 8, 64, 16, 10, "cpu")
    s = c.get_stats()
    assert (s["allocations"], s["evictions"], s["hits"], s["misses"]) == (0, 0, 0, 0)


def test_paged_cache_allocates_on_cpu_with_page_views():
    c = _paged()
    b = c.allocate_block(layer_idx=0, prefix_hash="p")
    assert b.layer_idx == 0 and b.prefix_hash == "p" and b.block_id in c._blocks
    assert b.keys.shape == (8, 16, 64) and b.keys.device.type == "cpu"
    b.keys.fill_(3.0)
    assert c.k_pool[b.slot].eq(3.0).all()  # view into the pool, not a copy
    assert c.get_stats()["allocations"] == 1


def test_paged_cache_many_blocks():
    c = _paged()
    blocks = [c.allocate_block(layer_idx=i % 4) for i in range(5)]
    assert all(blocks) and len({b.block_id for b in blocks}) == 5
    s = c.get_stats()
    assert s["allocations"] == 5 and s["total_blocks"] == 5


def test_paged_cache_free_zeroes_and_recycles():
    c = _paged()
    b = c.allocate_block(0)
    b.keys.fill_(1.0)
    c.free_block(b.block_id)
    assert b.block_id not in c._blocks and b.block_id in c._free_blocks
    assert c.k_pool[b.slot].abs().sum() == 0
    again = c.allocate_block(0)
    assert again.block_id == b.block_id


def test_paged_cache_shared_block_needs_two_frees():
    c = _paged()
    b = c.allocate_block(0)
    b.add_ref()
    c.free_block(b.block_id)
    assert b.block_id in c._blocks and b.ref_count == 1
    c.free_block(b.block_id)
    assert b.block_id not in c._blocks


def test_paged_cache_hit_and_miss():
    c = _paged()
    b = c.allocate_block(0)
    assert c.get_block(b.block_id) is b
    assert c.get_block("nope") is None
    s = c.get_stats()
    assert (s["hits"], s["misses"]) == (1, 1)


def test_paged_cache_lru_eviction_picks_oldest_unshared():
    c = _paged(max_blocks=3)
    a, b, d = (c.allocate_block(0) for _ in range(3))
    assert not c._free_blocks
    c.get_block(a.block_id)        # a becomes most recent
    b.add_ref()                    # b is shared: not evictable
    new = c.allocate_block(0)
    assert new is not None and c.get_stats()["evictions"] == 1
    assert d.block_id not in c._blocks or d.block_id == new.block_id
    assert a.block_id in c._blocks and b.block_id in c._blocks


def test_paged_cache_full_of_shared_blocks_returns_none():
    c = _paged(max_blocks=2)
    for _ in range(2):
        c.allocate_block(0).add_ref()
    assert c.allocate_block(0) is None


def test_kv_pool_sequences():
    pool = KVCachePool(num_layers=4, num_heads=8, head_dim=64, block_size=16, max_blocks_per_layer=10, device="cpu",
                       dtype=torch.float32)
    assert (pool.num_layers, pool.num_heads, pool.head_dim, len(pool._layer_caches)) == (4, 8, 64, 4)
    blocks = pool.allocate_sequence(32)
    assert len(blocks) == 4 and all(len(lb) == 2 for lb in blocks)
    assert len(pool.allocate_sequence(20)[0]) == 2   # partial last block
    assert pool.get_total_memory_gb() > 0
    pool.free_sequence(blocks)
    assert all(c.get_stats()["total_blocks"] == 2 for c in pool._layer_caches)


def test_kv_pool_rolls_back_on_failure():
    pool = KVCachePool(num_layers=3, num_heads=2, head_dim=8, block_size=4, max_blocks_per_layer=4, device="cpu",
                       dtype=torch.float32)
    held = pool.allocate_sequence(12)          # 3 of 4 pages per layer, pinned (live sequence)
    with pytest.raises(RuntimeError):
        pool.allocate_sequence(8)              # needs 2 per layer, only 1 free, live pages not evictable
    assert all(c.get_stats()["total_blocks"] == 3 for c in pool._layer_caches)
    pool.free_sequence(held)
    assert len(pool.allocate_sequence(16)[0]) == 4


def test_manager_init_hash_and_initial_stats():
    m = _mgr()
    assert (m.num_layers, m.num_heads, m.head_dim, m.redis) == (4, 8, 64, None)
    h1, h2, h3 = (m.compute_prefix_hash(t) for t in ([1, 2, 3], [1, 2, 3], [1, 2, 4]))
    assert h1 == h2 != h3 and len(h1) == 16
    assert m.compute_prefix_hash([70000, 1]) != m.compute_prefix_hash([70001, 1])
    s = m.get_stats()
    assert (s["l1_hits"], s["l2_hits"], s["l3_hits"], s["misses"], s["total_requests"]) == (0, 0, 0, 0, 0)


async def test_manager_miss_then_l1_hit():
    m = _mgr()
    k, v = torch.randn(8, 16, 64), torch.randn(8, 16, 64)
    calls = []

    async def compute():
        calls.append(1)
        return k, v

    rk, rv = await m.get_or_compute("pfx", 0, compute)
    assert rk.shape == k.shape and torch.equal(rk, k) and torch.equal(rv, v)
    rk2, _ = await m.get_or_compute("pfx", 0, compute)
    assert len(calls) == 1 and torch.equal(rk2, k)
    s = m.get_stats()
    assert s["misses"] == 1 and s["l1_hits"] == 1


async def test_manager_l2_hit_after_l1_loss():
    m = _mgr()
    k, v = torch.randn(8, 16, 64), torch.randn(8, 16, 64)

    async def compute():
        return k, v

    await m.get_or_compute("pfx", 1, compute)
    blk = m._prefix_index["pfx"][1]
    m.gpu_cache.get_layer_cache(1).free_block(blk.block_id)
    rk, _ = await m.get_or_compute("pfx", 1, compute)
    assert torch.equal(rk, k) and m.get_stats()["l2_hits"] == 1


async def test_manager_distinct_prefixes_each_compute():
    m = _mgr(num_layers=2, num_heads=4, head_dim=32)
    n = []

    async def compute():
        n.append(1)
        return torch.randn(4, 16, 32), torch.randn(4, 16, 32)

    for p in ("a", "b", "c"):
        await m.get_or_compute(p, 0, compute)
    assert len(n) == 3


def test_cpu_tier_copies_and_evicts_lru():
    m = _mgr()
    m.cpu_cache_max_items = 3
    src = torch.randn(8, 16, 64)
    m._add_to_cpu_cache("k0", src, src)
    src.zero_()
    assert m.cpu_cache["k0"][0].abs().sum() > 0  # stored a copy
    for i in range(1, 5):
        m._add_to_cpu_cache(f"k{i}", torch.randn(8, 16, 64), torch.randn(8, 16, 64))
    assert list(m.cpu_cache) == ["k2", "k3", "k4"]
    assert m.cpu_cache["k4"][0].device.type == "cpu"


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
def test_kv_blob_roundtrip_is_exact(dtype):
    m = _mgr()
    k, v = torch.randn(8, 16, 64).to(dtype), torch.randn(8, 16, 64).to(dtype)
    rk, rv = m._deserialize_kv(m._serialize_kv(k, v))
    assert rk.dtype == dtype and torch.equal(rk, k) and torch.equal(rv, v)


async def test_redis_absent_returns_none():
    assert await _mgr()._get_from_redis("x") is None


async def test_redis_get_uses_kv_prefix():
    r = AsyncMock()
    r.get.return_value = None
    m = _mgr(redis_client=r)
    assert await m._get_from_redis("test_key") is None
    r.get.assert_called_once_with("kv:test_key")


async def test_redis_write_and_l3_hit():
    store = {}
    r = AsyncMock()

    async def setex(key, ttl, val):
        store[key] = (ttl, val)

    async def get(key):
        return store.get(key, (0, None))[1]

    r.setex.side_effect = setex
    r.get.side_effect = get
    m = _mgr(redis_client=r)
    k, v = torch.randn(8, 16, 64), torch.randn(8, 16, 64)
    await m._write_to_redis("test_key", k, v, ttl=60)
    assert store["kv:test_key"][0] == 60
    # a fresh manager (empty L1/L2) finds it in L3 under the "prefix:layer" key
    await m._write_to_redis("pfx:2", k, v)
    m2 = _mgr(redis_client=r)

    async def never():
        raise AssertionError("should hit L3")

    rk, rv = await m2.get_or_compute("pfx", 2, never)
    assert torch.equal(rk, k) and m2.get_stats()["l3_hits"] == 1


def test_manager_hit_rates():
    m = _mgr()
    m._stats.update(l1_hits=10, l2_hits=5, misses=3)
    s = m.get_stats()
    assert s["total_requests"] == 18
    assert s["l1_hit_rate"] == pytest.approx(10 / 18)
    assert s["overall_hit_rate"] == pytest.approx(15 / 18)


# ============================================================================= native pool + radix cache

def _pool(n=16, bs=4):
    return BlockPool(n, bs, num_layers=2, num_kv_heads=1, head_dim=8, dtype=torch.float32, device="cpu")


def test_block_budget_arithmetic():
    # 70B: 80 layers x 8 kv heads x 128 dims, 16-token pages: 5 MiB per page
    per = 2 * 80 * 8 * 16 * 128 * 2
    assert num_blocks_for_budget(per * 1000 + 5, 80, 8, 128, 16) == 1000


def test_block_pool_reserves_scratch_page_and_counts():
    p = _pool()
    assert p.num_free == 15 and p.num_used == 0
    ids = p.allocate(5)
    assert 0 not in ids and len(set(ids)) == 5 and p.num_used == 5
    p.free(ids)
    assert p.num_free == 15
    with pytest.raises(OutOfBlocks):
        p.allocate(16)


def test_block_pool_refcount_and_double_free():
    p = _pool()
    (b,) = p.allocate(1)
    p.incref([b])
    p.free([b])
    assert p.num_free == 14
    p.free([b])
    assert p.num_free == 15
    with pytest.raises(RuntimeError, match="double free"):
        p.free([b])


def test_block_pool_kv_layout_spans_all_layers():
    p = _pool()
    assert p.kv.shape == (2, 2, 16, 1, 4, 8)
    k0, v0 = p.layer_kv(0)
    assert k0.shape == (16, 1, 4, 8)
    assert p.page_bytes() == 2 * 2 * 1 * 4 * 8 * 4


def test_radix_match_insert_and_sharing():
    p = _pool()
    rc = RadixCache(p)
    toks = list(range(10))           # 2 full pages + 2 tokens
    blocks = p.allocate(3)
    assert rc.insert(toks, blocks) == 2
    got, path = rc.match(list(range(8)) + [99, 98])
    assert got == blocks[:2]
    assert p.ref[blocks[0]] == 3     # owner + tree + this match
    rc.release(path)
    p.free(got)
    miss, _ = rc.match([5, 5, 5, 5], lock=False)
    assert miss == []
    assert 0 < rc.hit_rate() < 1


def test_radix_eviction_frees_lru_unlocked_leaves():
    p = _pool(n=8)
    rc = RadixCache(p)
    a = p.allocate(2)
    rc.insert([1] * 4 + [2] * 4, a)
    b = p.allocate(2)
    rc.insert([3] * 4 + [4] * 4, b)
    p.free(a)
    p.free(b)                        # only the tree holds them now
    assert p.num_free == 3
    _, path = rc.match([3] * 4 + [4] * 4)   # lock prefix b
    got = p.allocate(5)              # needs 2 evictions: must come from prefix a
    assert len(got) == 5
    assert rc.match([1] * 4, lock=False)[0] == []
    assert rc.match([3] * 4 + [4] * 4, lock=False)[0] == b
    rc.release(path)


def test_copy_on_write_duplicates_shared_page():
    p = _pool()
    (b,) = p.allocate(1)
    p.kv[:, :, b] = 7.0
    assert p.cow(b) == b             # private: unchanged
    p.incref([b])
    nb = p.cow(b)
    assert nb != b and p.ref[b] == 1 and p.ref[nb] == 1
    assert torch.equal(p.kv[:, :, nb], p.kv[:, :, b])
