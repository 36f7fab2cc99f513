"""Pinned host KV tier under the radix cache: spill on eviction, restore on hit."""
import pytest
import torch

from dgi.engine import EngineConfig, LLMEngine
from dgi.kv.block_pool import BlockPool
from dgi.kv.host_tier import HostKVTier
from dgi.kv.radix_cache import RadixCache
from dgi.sched.request import SamplingParams


def _pool(nb=9, device="cpu"):
    p = BlockPool(nb, 4, num_layers=2, num_kv_heads=1, head_dim=8, dtype=torch.float32, device=device)
    p.kv.copy_(torch.randn_like(p.kv))
    return p


def test_spill_and_restore_roundtrip():
    pool = _pool()
    tier = HostKVTier(pool, 8)
    rc = RadixCache(pool, tier)
    toks = list(range(16))                       # 4 full blocks
    blocks = pool.allocate(4)
    want = pool.kv[:, :, blocks].clone()
    rc.insert(toks, blocks)
    pool.free(blocks)                            # only the cache holds them now
    assert rc.evict(4) == 4                      # all spilled, GPU pages free
    assert tier.stats["spilled"] == 4 and pool.num_free == 8
    pool.kv.zero_()
    got, path = rc.match(toks + [99])
    assert len(got) == 4 and rc.host_hits_blocks == 4
    assert torch.equal(pool.kv[:, :, got], want)
    rc.release(path)
    pool.free(got)


def test_host_full_drops_lru_leaves():
    pool = _pool()
    tier = HostKVTier(pool, 2)
    rc = RadixCache(pool, tier)
    for base in (0, 100):
        b = pool.allocate(2)
        rc.insert(list(range(base, base + 8)), b)
        pool.free(b)
    assert rc.evict(4) >= 2
    assert tier.num_free >= 0 and pool.num_free >= 6


def test_engine_prefix_reuse_through_host_tier():
    cfg = EngineConfig(model="llama-tiny", device="cpu", max_num_seqs=4, max_num_batched_tokens=128,
                       max_model_len=256, use_graphs=False, num_blocks=24, host_kv_gb=0.01)
    eng = LLMEngine(cfg)
    ref = LLMEngine(EngineConfig(**{**cfg.__dict__, "host_kv_gb": 0.0, "enable_prefix_caching": False}),
                    model=eng.model)
    g = torch.Generator().manual_seed(1)
    shared = torch.randint(5, 500, (64,), generator=g).tolist()
    sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
    a = eng.generate([shared + [7, 8]], sp)[0].output
    # unrelated traffic pushes the shared prefix out of the 24-page GPU pool
    for i in range(6):
        eng.generate([torch.randint(5, 500, (80,), generator=g).tolist()], sp)
    assert eng.host_tier.stats["spilled"] > 0
    b = eng.generate([shared + [9, 10]], sp)[0].output
    assert eng.scheduler.radix.host_hits_blocks > 0
    assert b == ref.generate([shared + [9, 10]], sp)[0].output
    assert a == ref.generate([shared + [7, 8]], sp)[0].output


@pytest.mark.gpu
def test_host_tier_gpu_roundtrip():
    pool = BlockPool(17, 16, num_layers=4, num_kv_heads=8, head_dim=128, dtype=torch.bfloat16, device="cuda")
    pool.kv.copy_(torch.randn_like(pool.kv))
    tier = HostKVTier(pool, 16)
    rc = RadixCache(pool, tier)
    toks = list(range(16 * 6))
    blocks = pool.allocate(6)
    want = pool.kv[:, :, blocks].clone()
    rc.insert(toks, blocks)
    pool.free(blocks)
    assert rc.evict(6) == 6
    pool.kv.zero_()
    got, path = rc.match(toks + [1])
    torch.cuda.synchronize()
    assert torch.equal(pool.kv[:, :, got], want)


@pytest.mark.parametrize("prefix_caching", [False, True])
def test_preemption_swaps_to_host_tier_instead_of_recomputing(prefix_caching):
    """A pool too small for every running sequence forces preemptions: with the
    host tier the victims' pages are swapped out and back, the outputs equal an
    unconstrained engine's, and no prompt token is prefilled twice."""
    base = dict(model="llama-tiny", device="cpu", max_num_seqs=6, max_num_batched_tokens=256,
                max_model_len=256, use_graphs=False, enable_prefix_caching=prefix_caching)
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(5, 500, (20 + 3 * i,), generator=g).tolist() for i in range(6)]
    sp = SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True)
    big = LLMEngine(EngineConfig(**base, num_blocks=256))
    want = [r.output for r in big.generate(prompts, sp)]
    # 6 sequences x up to 59 tokens need ~22 pages of 16; 16 pages force preemption
    eng = LLMEngine(EngineConfig(**base, num_blocks=17, host_kv_gb=0.05), model=big.model)
    got = [r.output for r in eng.generate(prompts, sp)]
    st = eng.scheduler.stats()
    assert got == want
    assert st["preemptions"] > 0 and st["swapped_out"] == st["preemptions"] == st["swapped_in"]
    assert eng.stats["prefill_tokens"] == sum(len(p) for p in prompts)
    if not prefix_caching:          # (the radix cache may keep evicted prefix pages there)
        assert eng.host_tier.num_free == eng.host_tier.capacity


def test_preemption_without_tier_recomputes():
    base = dict(model="llama-tiny", device="cpu", max_num_seqs=6, max_num_batched_tokens=256,
                max_model_len=256, use_graphs=False, enable_prefix_caching=False)
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(5, 500, (20 + 3 * i,), generator=g).tolist() for i in range(6)]
    sp = SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True)
    eng = LLMEngine(EngineConfig(**base, num_blocks=17))
    eng.generate(prompts, sp)
    assert eng.scheduler.stats()["preemptions"] > 0
    assert eng.stats["prefill_tokens"] > sum(len(p) for p in prompts)


def test_auto_host_tier_size_is_half_the_pool_capped_by_ram():
    from dgi.engine import auto_host_kv_gb
    pool = _pool(nb=65)
    gb = auto_host_kv_gb(pool, torch.device("cpu"))
    assert 0 < gb <= pool.page_bytes() * 65 * 0.5 / (1 << 30) + 0.01


@pytest.mark.gpu
def test_streams_created_are_within_the_engine_budget():
    """Every long-lived stream a serving engine really creates (mixed steps with the
    side attention stream, host tier spills) is in its stream budget, and the
    budget fits the hardware queues of one priority class."""
    from dgi.parallel.fabric import GPU_HW_QUEUES
    from dgi.utils.streams import created, engine_streams
    eng = LLMEngine(EngineConfig(model="llama-tiny-hd128", device="cuda", max_num_seqs=6, max_num_batched_tokens=256,
                                 max_model_len=256, use_graphs=False, enable_prefix_caching=False, num_blocks=17,
                                 host_kv_gb=0.05))
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(5, 500, (20 + 3 * i,), generator=g).tolist() for i in range(6)]
    sp = SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True)
    for p in prompts[:3]:
        eng.add_request(p, sp)
    for _ in range(2):
        eng.step()
    for p in prompts[3:]:                 # admitted while the first three decode: mixed steps
        eng.add_request(p, sp)
    while eng.has_unfinished():
        eng.step()
    torch.cuda.synchronize()
    assert eng.scheduler.stats()["swapped_out"] > 0            # the copy stream was used
    budget = engine_streams(eng)
    have = created(torch.cuda.current_device())
    assert set(have["normal"]) - {"capture"} <= set(budget), (have, budget)
    assert "attn_side" in have["normal"] and "kv_host_copy" in have["normal"]
    assert len(budget) <= GPU_HW_QUEUES and len(have["high"]) <= GPU_HW_QUEUES - 1


def test_slot_runs_batch_contiguous_dmas():
    from dgi.kv.host_tier import runs
    assert runs([3, 4, 5, 9, 10, 2]) == [(0, 3, 3), (3, 9, 2), (5, 2, 1)]
    assert runs([]) == []
    pool = _pool(nb=17)
    tier = HostKVTier(pool, 16)
    blocks = pool.allocate(6)
    want = pool.kv[:, :, blocks].clone()
    slots = tier.spill(blocks)
    assert slots == list(range(6)) and tier.stats["spill_dmas"] == 1         # lowest slots first: one run
    fresh = pool.allocate(6)
    tier.restore(slots, fresh)
    tier.release(slots)
    assert tier.stats["restore_dmas"] == 1
    assert torch.equal(pool.kv[:, :, fresh], want)


def test_prompt_pages_are_shared_while_the_first_request_decodes():
    """A prompt's full pages are published in the radix cache when its prefill completes
    (not only when it finishes): a second request with the same prefix, admitted while
    the first still decodes, reuses them, and its output equals a cold engine's."""
    cfg = EngineConfig(model="llama-tiny", device="cpu", max_num_seqs=4, max_num_batched_tokens=128,
                       max_model_len=256, use_graphs=False, num_blocks=64)
    eng = LLMEngine(cfg)
    cold = LLMEngine(EngineConfig(**{**cfg.__dict__, "enable_prefix_caching": False}), model=eng.model)
    g = torch.Generator().manual_seed(5)
    shared = torch.randint(5, 500, (48,), generator=g).tolist()
    sp = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True)
    r1 = eng.add_request(shared + [1, 2], sp)
    eng.step()                        # r1's prefill
    eng.step()                        # r1 decodes
    r2 = eng.add_request(shared + [3, 4, 5], sp)
    while eng.has_unfinished():
        eng.step()
    assert r2.num_cached == 48 and r1.num_cached == 0
    assert [r1.output, r2.output] == [r.output for r in cold.generate([shared + [1, 2], shared + [3, 4, 5]], sp)]


def _gpu_prompts(n, seed, base=20, step=3):
    g = torch.Generator().manual_seed(seed)
    return [torch.randint(5, 500, (base + step * i,), generator=g).tolist() for i in range(n)]


@pytest.mark.gpu
def test_gpu_prefix_hits_with_graphs_are_token_identical():
    """prefix-hit prefill chunks under the captured decode graphs, with
    the host tier spilling and restoring shared pages (a pool too small for every prefix).
    Greedy outputs equal an engine without prefix caching on the same weights."""
    base = dict(model="llama-tiny-hd128", device="cuda", max_num_seqs=8, max_num_batched_tokens=256,
                max_model_len=512, use_graphs=True)
    g = torch.Generator().manual_seed(11)
    shared = [torch.randint(5, 500, (64,), generator=g).tolist() for _ in range(3)]
    prompts = [shared[i % 3] + torch.randint(5, 500, (5 + i,), generator=g).tolist() for i in range(12)]
    # unrelated long prompts between the waves push the cached prefixes out of the 40-page pool
    filler = [torch.randint(5, 500, (150,), generator=g).tolist() for _ in range(4)]
    order = prompts[:8] + filler + prompts[8:]
    sp = SamplingParams(max_tokens=16, temperature=0.0, ignore_eos=True)
    cold = LLMEngine(EngineConfig(**base, enable_prefix_caching=False, num_blocks=256))
    want = [r.output for r in cold.generate(order, sp)]
    eng = LLMEngine(EngineConfig(**base, enable_prefix_caching=True, num_blocks=40, host_kv_gb=0.05),
                    model=cold.model)
    eng.warmup()
    got = []
    for i in range(0, len(order), 4):  # waves: later waves hit pages published / spilled by earlier ones
        got += [r.output for r in eng.generate(order[i:i + 4], sp)]
    torch.cuda.synchronize()
    assert got == want
    st = eng.scheduler.stats()
    assert st["prefix_hit_rate"] > 0.2, st
    assert eng.runner.graphs is not None and eng.runner.graphs.captured
    assert eng.host_tier.stats["spilled"] > 0 and eng.scheduler.radix.host_hits_blocks > 0, eng.host_tier.stats


@pytest.mark.gpu
@pytest.mark.parametrize("prefix_caching", [False, True])
def test_gpu_swap_in_feeds_captured_decode(prefix_caching):
    """preemption swaps sequences to the pinned host tier and back
    (restored one step ahead on the copy stream, gated by an event) and the re-admitted
    rows decode in the captured graphs: token-identical to an unconstrained engine, no
    prompt recomputed, restores batched into contiguous DMAs."""
    base = dict(model="llama-tiny-hd128", device="cuda", max_num_seqs=6, max_num_batched_tokens=256,
                max_model_len=256, use_graphs=True, enable_prefix_caching=prefix_caching)
    prompts = _gpu_prompts(6, 3)
    sp = SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True)
    big = LLMEngine(EngineConfig(**base, num_blocks=256))
    want = [r.output for r in big.generate(prompts, sp)]
    eng = LLMEngine(EngineConfig(**base, num_blocks=17, host_kv_gb=0.05), model=big.model)
    eng.warmup()
    got = [r.output for r in eng.generate(prompts, sp)]
    torch.cuda.synchronize()
    st, ts = eng.scheduler.stats(), eng.host_tier.stats
    assert got == want
    assert st["swapped_out"] > 0 and st["swapped_in"] == st["swapped_out"]
    assert eng.stats["prefill_tokens"] == sum(len(p) for p in prompts)
    assert ts["restore_dmas"] < ts["restored"] or ts["restored"] <= st["swapped_in"], ts
    assert ts["gates"] > 0


@pytest.mark.parametrize("host_kv_gb", [0.0, 0.05])
def test_admission_evicts_whole_cached_chains(host_kv_gb):
    """A prompt needing more pages than the radix tree's current leaves hold is admitted by
    evicting chain after chain (leaves first, then the parents they expose) — the capacity
    check counts every page repeated leaf eviction frees, so the engine cannot stall with
    nothing running while the cache holds the pages."""
    base = dict(model="llama-tiny", device="cpu", max_num_seqs=8, max_num_batched_tokens=256,
                max_model_len=512, use_graphs=False)
    g = torch.Generator().manual_seed(11)
    shared = [torch.randint(5, 500, (64,), generator=g).tolist() for _ in range(3)]
    prompts = [shared[i % 3] + torch.randint(5, 500, (5 + i,), generator=g).tolist() for i in range(12)]
    filler = [torch.randint(5, 500, (150,), generator=g).tolist() for _ in range(4)]
    order = prompts[:8] + filler + prompts[8:]
    sp = SamplingParams(max_tokens=16, temperature=0.0, ignore_eos=True)
    cold = LLMEngine(EngineConfig(**base, enable_prefix_caching=False, num_blocks=256))
    want = [r.output for r in cold.generate(order, sp)]
    eng = LLMEngine(EngineConfig(**base, enable_prefix_caching=True, num_blocks=40, host_kv_gb=host_kv_gb),
                    model=cold.model)
    got = []
    for i in range(0, len(order), 4):
        got += [r.output for r in eng.generate(order[i:i + 4], sp)]
    assert got == want
    assert eng.scheduler.stats()["prefix_hit_rate"] > 0.1
    if host_kv_gb:
        assert eng.host_tier.stats["spilled"] > 0 and eng.scheduler.radix.host_hits_blocks > 0
