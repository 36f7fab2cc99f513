"""EAGLE-3 speculative decoding: lossless vs plain greedy, draft training raises
acceptance, and the reference-compatible ``worker.engines.speculative`` API
(mirrors reference tests/test_worker_engines_speculative.py)."""
import asyncio

import pytest
import torch
import torch.nn as nn

from dgi.engine import EngineConfig, LLMEngine
from dgi.sched.request import SamplingParams
from dgi.spec.eagle3 import SpecConfig, SpecEngine, kv_slot_copy, train_draft


def _engines(model="llama-tiny", device="cpu", spec=None):
    spec = spec or SpecConfig(depth=3, width=2, topk=3, auto_off=False, adaptive_depth=False)
    cfg = EngineConfig(model=model, device=device, max_num_seqs=8, max_num_batched_tokens=256, max_model_len=512,
                       use_graphs=False)
    base = LLMEngine(cfg)
    se = SpecEngine(cfg, spec)
    se.model.copy_from(base.model)
    return base, se


def _prompts(n=3, V=500):
    g = torch.Generator().manual_seed(0)
    return [torch.randint(5, V, (L,), generator=g).tolist() for L in (7, 20, 33, 12)[:n]]


def test_spec_is_lossless_and_training_raises_acceptance():
    base, se = _engines()
    sp = SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True)
    ref = [r.output for r in base.generate(_prompts(), sp)]
    assert [r.output for r in se.generate(_prompts(), sp)] == ref
    before = se.acceptance()["mean_accepted"]
    info = train_draft(se, steps=60, batch=8, prompt_len=16, gen_len=48, num_seqs=16)
    assert info["loss_last"] < info["loss_first"]
    se.spec_stats.update(spec_steps=0, spec_rows=0, accepted=0, spec_tokens=0)
    assert [r.output for r in se.generate(_prompts(), sp)] == ref
    after = se.acceptance()
    assert after["mean_accepted"] > before + 0.5 and after["tokens_per_step"] > 1.5


def test_spec_mixed_greedy_and_sampled_requests():
    base, se = _engines()
    g = SamplingParams(max_tokens=10, temperature=0.0, ignore_eos=True)
    s = SamplingParams(max_tokens=10, temperature=0.8, top_k=0, top_p=1.0, ignore_eos=True, seed=7)
    p = _prompts(2)
    r0 = se.add_request(p[0], g)
    r1 = se.add_request(p[1], s)
    while se.has_unfinished():
        se.step()
    assert r0.output == base.generate([p[0]], g)[0].output
    assert len(r1.output) == 10


def _sampled(i, n=24):
    return SamplingParams(max_tokens=n, temperature=0.9, top_k=20, top_p=0.9, ignore_eos=True, seed=100 + i)


def _gen(eng, prompts, mk):
    reqs = [eng.add_request(p, mk(i)) for i, p in enumerate(prompts)]
    while eng.has_unfinished():
        eng.step()
    return [r.output for r in reqs]


def test_spec_sampled_requests_are_identical_to_plain_sampling():
    """Coupled verification: every tree node is checked against the target's own
    seeded sample for that output index, so speculative sampled decoding emits
    exactly the tokens plain sampled decoding emits."""
    base, se = _engines()
    train_draft(se, steps=60, batch=8, prompt_len=16, gen_len=48, num_seqs=16)
    ref = _gen(base, _prompts(), _sampled)
    se.spec_stats.update(spec_steps=0, spec_rows=0, accepted=0, spec_tokens=0)
    assert _gen(se, _prompts(), _sampled) == ref
    assert se.spec_stats["spec_steps"] > 0 and se.spec_stats["accepted"] > 0


def test_sampler_distribution_chi_square():
    """The Gumbel-max sampler (the draw plain and speculative decoding share)
    follows softmax(logits / T) renormalised over the top-k / top-p set."""
    from scipy.stats import chisquare

    from dgi import ops
    logits = torch.tensor([[2.0, 1.5, 1.0, 0.5, 0.0, -0.5, -1.0, -3.0]])
    n = 20000
    lg = logits.expand(n, -1).contiguous()
    temps = torch.full((n,), 0.8)
    seeds = torch.arange(n)
    for k, p in ((0, 1.0), (5, 1.0), (0, 0.8)):
        tk, tp = torch.full((n,), k), torch.full((n,), p)
        out = ops.sample(lg, temps, seeds, 3, top_k=tk, top_p=tp)
        kept = torch.isfinite(ops.apply_top_k_top_p(logits, tk[:1], tp[:1], temps[:1]))[0]
        prob = torch.softmax(torch.where(kept, logits[0] / 0.8, torch.tensor(-float("inf"))), -1)
        obs = torch.bincount(out, minlength=8).double()
        assert int(obs[~kept].sum()) == 0
        exp = prob[kept].double()
        exp = (exp / exp.sum() * obs[kept].sum()).numpy()
        stat, pval = chisquare(obs[kept].numpy(), exp)
        assert pval > 1e-3, (k, p, stat, pval)


def test_adaptive_depth_follows_acceptance():
    """Reference _adapt_depth: depth shrinks under min_accept_rate, grows over 0.7."""
    base, se = _engines(spec=SpecConfig(depth=4, width=2, topk=3, auto_off=False, adaptive_depth=True))
    sp = SamplingParams(max_tokens=30, temperature=0.0, ignore_eos=True)
    prompts = _prompts(2)
    ref = [r.output for r in base.generate(prompts, sp)]
    # oracle drafts that are always right: depth stays at the maximum
    se.oracle, se.oracle_accept = {}, 1.0
    reqs = [se.add_request(p, sp) for p in prompts]
    for r, o in zip(reqs, ref):
        se.oracle[r.rid] = o
    while se.has_unfinished():
        se.step()
    assert [r.output for r in reqs] == ref and se.cur_depth == 4
    # oracle drafts that are always wrong: depth falls to 1
    se.oracle_accept = 0.0
    reqs = [se.add_request(p, sp) for p in prompts]
    for r, o in zip(reqs, ref):
        se.oracle[r.rid] = o
    while se.has_unfinished():
        se.step()
    assert [r.output for r in reqs] == ref and se.cur_depth == 1
    assert se.spec_stats["depth_changes"] >= 3


def test_auto_off_switches_to_plain_when_speculation_is_slower():
    base, se = _engines(spec=SpecConfig(depth=3, width=2, topk=3, auto_off=True, adaptive_depth=False,
                                        probe_every=12))
    sp = SamplingParams(max_tokens=40, temperature=0.0, ignore_eos=True)
    prompts = _prompts(2)
    ref = [r.output for r in base.generate(prompts, sp)]
    real = se._record
    # make speculation look 3x as expensive per token as plain decoding

    def rec(mode, R, seconds, tokens):
        real(mode, R, seconds * (3.0 if mode == "spec" else 1.0) * tokens / max(1, tokens), tokens)
    se._record = rec
    reqs = [se.add_request(p, sp) for p in prompts]
    modes = []
    while se.has_unfinished():
        se.step()
        modes.append(se.spec_on)
    assert [r.output for r in reqs] == ref                       # lossless in both modes
    assert se.spec_stats["plain_steps"] > 0 and se.spec_stats["switches_off"] >= 1
    assert modes.count(False) > modes.count(True)


def test_controller_ignores_single_outliers_and_capture_steps():
    """One low-acceptance step does not move the depth (EMA, >= 2 steps per depth);
    a step that captured a graph is no cost sample, so it cannot switch speculation
    off; reset_controller() restores full depth and forgets the costs."""
    _, se = _engines(spec=SpecConfig(depth=4, width=2, topk=3, auto_off=True, adaptive_depth=True))
    se._adapt_depth(0.9)
    se._adapt_depth(0.0)                  # outlier: EMA 0.54, stays
    assert se.cur_depth == 4
    for _ in range(2):
        se._adapt_depth(0.0)
    assert se.cur_depth == 3 and se.spec_stats["depth_changes"] == 1
    se._adapt_depth(0.0)                  # first sample at the new depth never moves it
    assert se.cur_depth == 3
    # auto-off: speculation steps without a clean cost sample keep speculation on
    se._record("plain", 4, 0.010, 4)
    for _ in range(6):
        se._control(4)
    assert se.spec_on
    se._period_acc = [8, 4]               # 2 drafts accepted per row: depth 3 is already long enough
    se._record("spec", 4, 0.030, 4)       # now measurably slower than plain
    se._control(4)
    assert se.spec_on                     # one sample does not decide
    se._record("spec", 4, 0.030, 4)
    se._control(4)
    # slower than plain at depth 3: a shallower tree is tried first
    assert se.spec_on and se.cur_depth == 2 and se.spec_stats["switches_off"] == 0
    for _ in range(2):
        se._record("spec", 4, 0.030, 4)
        se._control(4)
    assert se.spec_on and se.cur_depth == 1
    for _ in range(2):
        se._record("spec", 4, 0.030, 4)
        se._control(4)
    assert not se.spec_on and se.spec_stats["switches_off"] == 1
    # losing re-probes back off: 48, then 96 plain steps
    for wait in (48, 96):
        for _ in range(wait - 1):
            se._control(4)
        assert not se.spec_on
        se._control(4)
        assert se.spec_on
        se._record("spec", 4, 0.030, 4)
        se._control(4)
        se._record("spec", 4, 0.030, 4)
        se._control(4)
        assert not se.spec_on
    assert se._backoff == 4
    se.reset_controller(keep_plain_costs=True)
    assert se.spec_on and se.cur_depth == 4 and list(se._cost) == [("plain", 4)]
    se.reset_controller()
    assert not se._cost
    assert se.warmup_spec([1, 2]) == 0    # CPU: no graphs to capture


def test_kv_slot_copy():
    kv = torch.randn(3, 2, 5, 2, 4, 8)
    ref = kv.clone()
    src, dst = torch.tensor([9, 13]), torch.tensor([5, 6])
    kv_slot_copy(kv, src, dst, 4)
    for s_, d_ in zip(src.tolist(), dst.tolist()):
        ref[:, :, d_ // 4, :, d_ % 4] = ref[:, :, s_ // 4, :, s_ % 4]
    assert torch.equal(kv, ref)


@pytest.mark.gpu
def test_kv_slot_copy_kernel_matches_reference_on_chains():
    """HIP slot copy (gather then scatter) == the torch advanced-index copy, including move
    chains where one move's source slot is another's destination, across pages and sequences."""
    g = torch.Generator().manual_seed(3)
    kv = torch.randn(4, 2, 9, 8, 16, 128, generator=g).to(torch.bfloat16)
    src = torch.tensor([18, 20, 21, 37, 50, 17], dtype=torch.int32)
    dst = torch.tensor([17, 18, 19, 33, 34, 16], dtype=torch.int32)   # 18 -> 17 while 20 -> 18, ...
    ref = kv.clone()
    c = ref.view(8, 9, 8, 16, 128)
    vals = c[:, src.long() // 16, :, src.long() % 16]
    c[:, dst.long() // 16, :, dst.long() % 16] = vals
    gk = kv.cuda()
    kv_slot_copy(gk, src.cuda(), dst.cuda(), 16)
    assert torch.equal(gk.cpu(), ref)


@pytest.mark.gpu
def test_spec_gpu_greedy_trajectory():
    """Spec output is a greedy trajectory of the target.  Plain decode (decode
    kernel) and verification (prefill kernel) may order bf16 near-ties
    differently, so exact equality is checked via the teacher-forced gap."""
    from dgi.spec.eagle3 import greedy_gap
    base, se = _engines("llama-tiny-hd128", "cuda", SpecConfig(depth=4, width=3, topk=4, auto_off=False,
                                                               adaptive_depth=False))
    sp = SamplingParams(max_tokens=32, temperature=0.0, ignore_eos=True)
    prompts = _prompts(4, 1000)
    train_draft(se, steps=80, batch=8, prompt_len=32, gen_len=96, num_seqs=32, random_seqs=32)
    se.spec_stats.update(spec_steps=0, spec_rows=0, accepted=0, spec_tokens=0)
    outs = [r.output for r in se.generate(prompts, sp)]
    for p, o in zip(prompts, outs):
        assert len(o) == 32 and greedy_gap(se, p, o) < 0.07   # bf16 logit resolution near |logit|~8
    assert se.acceptance()["tokens_per_step"] > 1.3


@pytest.mark.gpu
def test_spec_verify_graph_matches_eager():
    """The hipGraph verify pass (static buffers, padded batch bucket) gives the
    same tokens and acceptance as the eager verify pass, bit for bit (controller
    off: its timing-driven decisions would route the two engines differently)."""
    import dataclasses
    spec = SpecConfig(depth=4, width=3, topk=4, auto_off=False, adaptive_depth=False)
    base, sg = _engines("llama-tiny-hd128", "cuda", spec)
    se = SpecEngine(EngineConfig(model="llama-tiny-hd128", device="cuda", max_num_seqs=8, max_num_batched_tokens=256,
                                 max_model_len=512, use_graphs=False), dataclasses.replace(spec, graphs=False))
    se.model.copy_from(base.model)
    sp = SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True)
    prompts = _prompts(3, 1000)                        # R=3 -> bucket 4 with one padding row
    ref = [r.output for r in base.generate(prompts, sp)]
    outs = []
    for eng in (sg, se):
        eng.oracle, eng.oracle_accept = {}, 0.7
        rs = [eng.add_request(p, sp) for p in prompts]
        for r, o in zip(rs, ref):
            eng.oracle[r.rid] = o
        while eng.has_unfinished():
            eng.step()
        outs.append(([r.output for r in rs], eng.spec_stats["accepted"]))
    assert sg._vgraphs and not se._vgraphs
    assert outs[0] == outs[1]
    assert outs[0][1] > 0


# ------------------------------------------------------------------ reference-compatible API
def test_compat_config_output_defaults():
    from worker.engines.speculative import SpeculativeConfig, SpeculativeOutput
    c = SpeculativeConfig()
    assert (c.draft_model_id, c.use_self_draft, c.draft_head_hidden_size, c.num_speculative_tokens) == \
        (None, True, 1024, 5)
    assert (c.tree_width, c.tree_depth, c.temperature, c.top_p, c.min_accept_rate, c.adaptive_depth) == \
        (3, 5, 0.0, 1.0, 0.3, True)
    nc = c.to_native()
    assert nc.width == 3 and nc.depth == 5 and nc.num_nodes <= 64
    o = SpeculativeOutput([1, 2], 0.5, 4, 2, 1.0)
    assert o.accepted_tokens == 2


def test_compat_draft_head_tree_buffer_medusa():
    from worker.engines.speculative import DraftHead, MedusaHead, TreeDraftBuffer
    d = DraftHead(hidden_size=64, vocab_size=100, num_layers=2, hidden_dim=32)
    assert d.token_embedding is None
    with pytest.raises(RuntimeError, match="Token embedding not set"):
        d(torch.randn(1, 3, 64), torch.randint(0, 100, (1, 3)))
    d.set_token_embedding(nn.Embedding(100, 64))
    assert d(torch.randn(2, 5, 64), torch.randint(0, 100, (2, 5))).shape == (2, 5, 64)
    b = TreeDraftBuffer(3, 5, "cpu")
    b.add_candidates(torch.tensor([1, 2]), torch.tensor([-0.1, -0.2]), torch.tensor([-1, -1]))
    b.add_candidates(torch.tensor([3, 4]), torch.tensor([-0.3, -0.4]), torch.tensor([0, 1]))
    assert b.layer_offsets == [0, 2] and b.get_tree_tokens().tolist() == [1, 2, 3, 4]
    m = b.get_tree_attention_mask(5)
    assert m.shape == (4, 9) and m[:, :5].all() and m[2, 5] and not m[2, 6] and m[3, 6]
    b.nodes = [(1, -0.1, -1), (2, -0.2, 0), (3, -0.3, 1), (4, -0.4, 2)]
    assert b.trace_accepted_path(torch.tensor([True, True, False, False])) == [1, 2]
    assert b.trace_accepted_path(torch.tensor([False, False, False, False])) == []
    mh = MedusaHead(64, 100, num_heads=3, hidden_dim=16)
    outs = mh(torch.randn(2, 4, 64))
    assert len(outs) == 3 and outs[0].shape == (2, 4, 100)


def test_compat_speculative_decoder_loop_and_stats():
    from worker.engines.speculative import SpeculativeConfig, SpeculativeDecoder

    class Tiny(nn.Module):
        def __init__(self):
            super().__init__()
            self.model = nn.Module()
            self.model.embed_tokens = nn.Embedding(50, 32)
            self.lm_head = nn.Linear(32, 50)

        def forward(self, input_ids, output_hidden_states=True, use_cache=False):
            h = self.model.embed_tokens(input_ids).cumsum(1)
            return type("O", (), {"logits": self.lm_head(h), "hidden_states": (h,)})()
    torch.manual_seed(0)
    tgt = Tiny()
    dec = SpeculativeDecoder(tgt, SpeculativeConfig(tree_width=1, tree_depth=3), device="cpu")
    dec.setup_draft_head(32, 50)
    ids = torch.randint(0, 50, (1, 6))
    out = asyncio.run(dec.generate(ids, max_new_tokens=8))
    # lossless: equals plain greedy decoding of the target
    cur = ids
    ref = []
    for _ in range(8):
        nxt = tgt(cur).logits[0, -1].argmax()
        ref.append(int(nxt))
        cur = torch.cat([cur, nxt.view(1, 1)], 1)
    assert out.tokens == ref
    st = dec.get_stats()
    assert st["total_steps"] >= 1 and st["speedup_estimate"] >= 1.0
    dec._current_depth = 1
    dec._adapt_depth(0.05)
    assert dec._current_depth == 1


def test_oracle_chain_acceptance_ceiling():
    """With the known greedy continuation as the first chain, every depth is accepted."""
    base, se = _engines(spec=SpecConfig(depth=4, width=2, topk=3, auto_off=False))
    sp = SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True)
    prompts = _prompts()
    ref = [r.output for r in base.generate(prompts, sp)]
    se.oracle, se.oracle_accept = {}, 1.0
    rs = [se.add_request(p, sp) for p in prompts]
    for r, o in zip(rs, ref):
        se.oracle[r.rid] = o
    while se.has_unfinished():
        se.step()
    assert [r.output for r in rs] == ref
    assert se.acceptance()["mean_accepted"] > 3.0


def test_draft_vocabulary_keeps_spec_lossless_and_restricts_proposals():
    """EAGLE-3 draft vocabulary: the draft scores only the target's most frequent choices
    (a [V', H] head per depth instead of [V, H]); outputs stay identical to plain greedy
    decoding and every drafted token is a member of the draft vocabulary."""
    from dgi.spec.eagle3 import hot_vocab_from_targets
    t = torch.tensor([[5, 5, 7, 9, 9, 9, 3]])
    assert hot_vocab_from_targets(t, 16, 2).tolist() == [5, 9]
    assert hot_vocab_from_targets(t, 16, 10).tolist()[:4] == [0, 3, 5, 7] or \
        set(hot_vocab_from_targets(t, 16, 10).tolist()) >= {3, 5, 7, 9}
    base, se = _engines()
    sp = SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True)
    ref = [r.output for r in base.generate(_prompts(), sp)]
    info = train_draft(se, steps=40, batch=8, prompt_len=16, gen_len=48, num_seqs=16, draft_vocab=96)
    assert info["draft_vocab"]["size"] == 96 and 0 < info["draft_vocab"]["target_tokens_covered"] <= 1
    hot = set(se.draft.hot.tolist())
    assert se.draft.hot_head.shape == (96, se.model_cfg.hidden_size)
    seen = []
    orig = se._draft_tree_eager

    def spy(*a, **k):
        tok, par = orig(*a, **k)
        seen.append(tok[:, 1:].reshape(-1).tolist())
        return tok, par
    se._draft_tree_eager = spy
    assert [r.output for r in se.generate(_prompts(), sp)] == ref
    assert seen and all(t in hot for s in seen for t in s)


def test_auto_draft_vocabulary_picks_the_smallest_covering_size():
    """draft_vocab=-1: the smallest candidate size whose most frequent target tokens cover 99 % of
    the training corpus; the whole vocabulary when the target's choices are spread out."""
    from dgi.spec.eagle3 import auto_draft_vocab
    V = 1000
    g = torch.Generator().manual_seed(0)
    peaked = torch.randint(0, 40, (5000,), generator=g)             # 40 distinct tokens
    assert auto_draft_vocab(peaked, V, sizes=(16, 64, 256)) == 64
    spread = torch.randint(0, V, (5000,), generator=g)
    assert auto_draft_vocab(spread, V, sizes=(16, 64, 256)) == 0
    assert auto_draft_vocab(torch.zeros(0, dtype=torch.long), V) == 0


@pytest.mark.gpu
def test_spec_whole_step_graph_matches_staged_path():
    """the whole speculative step as one captured graph (draft catch-up, tree
    drafting, verify, accept, KV compaction, feature gather) runs in the steady state (R = 3:
    a padded bucket of 4), stays a greedy trajectory of the target, and accepts like the staged
    path (separate draft / verify graphs, host compaction) on the same draft."""
    import dataclasses
    from dgi.spec.eagle3 import greedy_gap
    spec = SpecConfig(depth=4, width=3, topk=4, auto_off=False, adaptive_depth=False)
    base, whole = _engines("llama-tiny-hd128", "cuda", spec)
    train_draft(whole, steps=80, batch=8, prompt_len=32, gen_len=96, num_seqs=32, random_seqs=32)
    staged = SpecEngine(EngineConfig(model="llama-tiny-hd128", device="cuda", max_num_seqs=8,
                                     max_num_batched_tokens=256, max_model_len=512, use_graphs=False),
                        dataclasses.replace(spec), model=whole.model, draft=whole.draft)
    staged.whole_step = False
    sp = SamplingParams(max_tokens=32, temperature=0.0, ignore_eos=True)
    prompts = _prompts(3, 1000)
    res = {}
    for name, eng in (("whole", whole), ("staged", staged)):
        eng.spec_stats.update(spec_steps=0, spec_rows=0, accepted=0, spec_tokens=0, whole_steps=0)
        outs = [r.output for r in eng.generate(prompts, sp)]
        for p, o in zip(prompts, outs):
            assert len(o) == 32 and greedy_gap(eng, p, o) < 0.07
        res[name] = (outs, eng.acceptance())
    assert res["whole"][1]["whole_steps"] > 0 and res["staged"][1]["whole_steps"] == 0
    assert whole._sgraphs and not staged._sgraphs
    tw, ts = res["whole"][1]["tokens_per_step"], res["staged"][1]["tokens_per_step"]
    assert tw > 1.3 and abs(tw - ts) < 0.35 * ts
    # sampled requests take the graph too (coupled verification with the per-node seeds)
    spt = SamplingParams(max_tokens=16, temperature=0.8, top_k=50, top_p=0.9, ignore_eos=True, seed=3)
    n0 = whole.spec_stats["whole_steps"]
    outs = [r.output for r in whole.generate(prompts, spt)]
    assert all(len(o) == 16 for o in outs) and whole.spec_stats["whole_steps"] > n0


def test_token_range_equals_slicing_the_full_token_list_cpu():
    """_whole_step slices each sequence's catch-up window without building prompt + output."""
    import types
    from dgi.spec.eagle3 import _token_range
    r = types.SimpleNamespace(prompt=list(range(10)), output=list(range(100, 105)))
    full = r.prompt + r.output
    for a in range(len(full) + 2):
        for b in range(a, len(full) + 2):
            assert _token_range(r, a, b) == full[a:b]


def test_step_graph_metadata_fill_matches_the_per_row_rule_cpu():
    """_StepGraph._fill (vectorized) against the per-row rule it encodes: catch-up rows p0 .. p0+C-1
    (past nv, or past the live batch: scratch slots on page 0), draft depths at n - 1 + depth with
    slots n .., verify nodes at n - 1 + depth(k) with slots n - 1 + k; padding rows on page 0."""
    import types
    import numpy as np
    import torch
    from dgi.spec.eagle3 import _StepGraph
    rng = np.random.default_rng(3)
    bs, maxw = 16, 12
    for _ in range(50):
        Rb, C = int(rng.integers(1, 6)), int(rng.integers(2, 6))
        depth = np.array([0] + sorted(rng.integers(1, 4, size=int(rng.integers(2, 7))).tolist()), dtype=np.int64)
        N = len(depth)
        lv, tot = [], Rb * maxw + 2 * Rb * C + 2 * Rb
        for m in range(2, min(N, 4)):
            lv.append((tot, m))
            tot += 2 * Rb * m + Rb
        o_v = tot
        tot += 2 * Rb * N + Rb
        g = object.__new__(_StepGraph)
        g.Rb, g.C, g.N, g.maxw = Rb, C, N, maxw
        g.eng = types.SimpleNamespace(pool=types.SimpleNamespace(block_size=bs))
        g.host = torch.full((tot,), -7, dtype=torch.int32)
        g.o_bt, g.o_c, g.o_v, g.lv, g.depth_np = 0, Rb * maxw, o_v, lv, depth
        R = int(rng.integers(0, Rb + 1))
        n_vec = rng.integers(C + 1, 150, size=R)
        nv_vec = rng.integers(1, C + 1, size=R)
        p0_vec = n_vec - nv_vec
        brows = [rng.integers(1, 500, size=maxw).tolist() for _ in range(R)]
        g._fill(n_vec, p0_vec, brows, nv_vec)
        h = g.host.numpy()

        def slot(i, p):
            return brows[i][p // bs] * bs + p % bs
        o = Rb * maxw
        for i in range(Rb):
            for k in range(C):
                pos, sl = h[o + i * C + k], h[o + Rb * C + i * C + k]
                if i < R:
                    assert pos == p0_vec[i] + k
                    assert sl == (slot(i, p0_vec[i] + k) if k < nv_vec[i] else k % bs)
                else:
                    assert pos == k and sl == k % bs
            assert h[o + 2 * Rb * C + i] == (p0_vec[i] if i < R else 0) + C
            assert h[o + 2 * Rb * C + Rb + i] == (nv_vec[i] - 1 if i < R else 0)
        for i in range(Rb):
            for k in range(N):
                pos, sl = h[o_v + i * N + k], h[o_v + Rb * N + i * N + k]
                if i < R:
                    assert pos == n_vec[i] - 1 + depth[k] and sl == slot(i, n_vec[i] - 1 + k)
                else:
                    assert pos == k and sl == k % bs
            assert h[o_v + 2 * Rb * N + i] == (n_vec[i] - 1 + N if i < R else N)
