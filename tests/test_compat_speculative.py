"""Speculative decoding compatibility layer (worker/engines/speculative.py).

Behavioural parity with the reference's
tests/test_worker_engines_speculative.py: config/output dataclasses,
DraftHead, TreeDraftBuffer (candidates, layer offsets, tokens, attention
mask, accepted-path tracing), SpeculativeDecoder (draft head set-up,
adaptive depth bounds, stats) and MedusaHead.  Beyond the reference: the
tree mask must encode ancestry (the reference's mask allowed sibling
attention, E-15), and the device-side tree ops (``dgi.ops.tree_mask`` /
``tree_verify``) are checked against brute-force definitions on CPU.
"""
import asyncio

import pytest
import torch
import torch.nn as nn

from worker.engines.speculative import (DraftHead, MedusaHead, SpeculativeConfig, SpeculativeDecoder,
                                        SpeculativeOutput, TreeDraftBuffer)
from dgi import ops


class _Target(nn.Module):
    """HF-shaped toy causal LM: embeddings -> running sum -> lm_head."""

    def __init__(self, vocab=50, hidden=32):
        super().__init__()
        self.model = nn.Module()
        self.model.embed_tokens = nn.Embedding(vocab, hidden)
        self.lm_head = nn.Linear(hidden, vocab)

    def forward(self, input_ids, output_hidden_states=True, use_cache=False):
        h = self.model.embed_tokens(input_ids).cumsum(1)
        return type("Out", (), {"logits": self.lm_head(h), "hidden_states": (h,)})()


@pytest.fixture
def buf():
    return TreeDraftBuffer(tree_width=3, tree_depth=5, device="cpu")


@pytest.fixture
def dec():
    torch.manual_seed(0)
    return SpeculativeDecoder(_Target(), SpeculativeConfig(tree_width=3, tree_depth=3, adaptive_depth=True),
                              device="cpu")


# ----------------------------------------------------------------------------- dataclasses

def test_config_defaults():
    c = SpeculativeConfig()
    assert (c.draft_model_id, c.use_self_draft, c.draft_head_hidden_size, c.num_speculative_tokens) == \
        (None, True, 1024, 5)
    assert (c.tree_width, c.tree_depth, c.temperature, c.top_p, c.min_accept_rate, c.adaptive_depth) == \
        (3, 5, 0.0, 1.0, 0.3, True)


def test_config_custom_and_native_mapping():
    c = SpeculativeConfig(draft_model_id="small", use_self_draft=False, draft_head_hidden_size=512,
                          num_speculative_tokens=10, tree_width=5, tree_depth=8, temperature=0.5,
                          min_accept_rate=0.5, adaptive_depth=False)
    assert (c.draft_model_id, c.tree_width, c.tree_depth, c.adaptive_depth) == ("small", 5, 8, False)
    n = c.to_native()
    assert (n.width, n.depth) == (5, 8)


def test_output_fields():
    o = SpeculativeOutput(tokens=[1, 2, 3, 4], accept_rate=0.8, draft_tokens=5, accepted_tokens=4, latency_ms=10.5)
    assert (o.tokens, o.accept_rate, o.draft_tokens, o.accepted_tokens, o.latency_ms) == ([1, 2, 3, 4], 0.8, 5, 4,
                                                                                          10.5)


# ----------------------------------------------------------------------------- draft head

def test_draft_head_init_and_embedding():
    d = DraftHead(hidden_size=64, vocab_size=100, num_layers=2, hidden_dim=32)
    assert (d.hidden_size, d.vocab_size, d.token_embedding) == (64, 100, None)
    assert d.feature_predictor is not None
    e = nn.Embedding(100, 64)
    d.set_token_embedding(e)
    assert d.token_embedding is e


def test_draft_head_requires_embedding():
    d = DraftHead(64, 100)
    with pytest.raises(RuntimeError, match="Token embedding not set"):
        d(torch.randn(1, 3, 64), torch.randint(0, 100, (1, 3)))


@pytest.mark.parametrize("b,s", [(1, 1), (2, 5), (1, 100)])
def test_draft_head_shapes(b, s):
    d = DraftHead(64, 100, num_layers=3, hidden_dim=16)
    d.set_token_embedding(nn.Embedding(100, 64))
    assert d(torch.randn(b, s, 64), torch.randint(0, 100, (b, s))).shape == (b, s, 64)


# ----------------------------------------------------------------------------- tree buffer

def test_buffer_init_and_reset(buf):
    assert (buf.tree_width, buf.tree_depth, buf.device) == (3, 5, "cpu")
    assert buf.nodes == [] and buf.layer_offsets == []
    buf.nodes.append((1, 0.5, -1))
    buf.layer_offsets.append(0)
    buf.reset()
    assert buf.nodes == [] and buf.layer_offsets == []


def test_buffer_add_candidates(buf):
    buf.add_candidates(torch.tensor([1, 2, 3]), torch.tensor([-0.1, -0.2, -0.3]), torch.tensor([0, 0, 0]))
    assert [n[0] for n in buf.nodes] == [1, 2, 3] and [n[2] for n in buf.nodes] == [0, 0, 0]
    assert buf.nodes[1][1] == pytest.approx(-0.2)
    assert buf.layer_offsets == [0]


def test_buffer_layers_and_tokens(buf):
    buf.add_candidates(torch.tensor([10, 20]), torch.tensor([-0.1, -0.2]), torch.tensor([-1, -1]))
    buf.add_candidates(torch.tensor([30, 40]), torch.tensor([-0.3, -0.4]), torch.tensor([0, 1]))
    assert buf.layer_offsets == [0, 2]
    assert buf.get_tree_tokens().tolist() == [10, 20, 30, 40]


def test_buffer_mask_sees_prefix_self_and_ancestors_only(buf):
    buf.add_candidates(torch.tensor([1, 2]), torch.tensor([-0.1, -0.2]), torch.tensor([-1, -1]))
    buf.add_candidates(torch.tensor([3, 4]), torch.tensor([-0.3, -0.4]), torch.tensor([0, 1]))
    m = buf.get_tree_attention_mask(5).bool()
    assert m.shape == (4, 9)
    assert m[:, :5].all()                       # whole prefix
    tree = m[:, 5:]
    expect = torch.tensor([[1, 0, 0, 0], [0, 1, 0, 0], [1, 0, 1, 0], [0, 1, 0, 1]], dtype=torch.bool)
    assert torch.equal(tree, expect)            # no sibling / cousin attention


def test_buffer_roots_only_mask(buf):
    buf.add_candidates(torch.tensor([1, 2]), torch.tensor([-0.1, -0.2]), torch.tensor([-1, -1]))
    m = buf.get_tree_attention_mask(5)
    assert m.shape == (2, 7) and int(m[:, :5].sum()) == 10


@pytest.mark.parametrize("mask,path", [([1, 1, 1], [1, 2, 3]), ([1, 1, 0], [1, 2]), ([0, 0, 0], []),
                                       ([1, 0, 1], [1])])
def test_trace_accepted_chain(buf, mask, path):
    buf.nodes = [(1, -0.1, -1), (2, -0.2, 0), (3, -0.3, 1)]
    assert buf.trace_accepted_path(torch.tensor(mask, dtype=torch.bool)) == path


def test_trace_accepted_branching_prefers_longest(buf):
    # two roots; the second root has the deeper accepted chain
    buf.nodes = [(1, -0.1, -1), (2, -0.2, -1), (3, -0.3, 0), (4, -0.4, 1), (5, -0.5, 3)]
    mask = torch.tensor([True, True, False, True, True])
    assert buf.trace_accepted_path(mask) == [2, 4, 5]


# ----------------------------------------------------------------------------- decoder

def test_decoder_init_and_draft_head(dec):
    assert dec.draft_head is None and dec.draft_model is None and dec._current_depth == 3
    d = dec.setup_draft_head(hidden_size=32, vocab_size=50)
    assert isinstance(d, DraftHead) and dec.draft_head is d and d.hidden_size == 32
    assert d.token_embedding is dec.target.model.embed_tokens   # shares the target's embedding


@pytest.mark.parametrize("start,rate,end", [(5, 0.1, 4), (1, 0.05, 1), (2, 0.8, 3), (3, 0.95, 3), (2, 0.5, 2)])
def test_adapt_depth(dec, start, rate, end):
    dec._current_depth = start
    dec._adapt_depth(accept_rate=rate)
    assert dec._current_depth == end


def test_adaptive_depth_off_keeps_depth_during_generation(dec):
    dec.config.adaptive_depth = False
    dec.setup_draft_head(32, 50)
    dec._current_depth = 2
    asyncio.run(dec.generate(torch.randint(0, 50, (1, 4)), max_new_tokens=6))
    assert dec._current_depth == 2


def test_gpt_style_target_embedding_is_shared():
    t = nn.Module()
    t.transformer = nn.Module()
    t.transformer.wte = nn.Embedding(50, 32)
    t.lm_head = nn.Linear(32, 50)
    d = SpeculativeDecoder(t, SpeculativeConfig(), device="cpu").setup_draft_head(32, 50)
    assert d.token_embedding is t.transformer.wte


def test_stats_initial_and_estimate(dec):
    s = dec.get_stats()
    assert (s["total_steps"], s["total_draft_tokens"], s["total_accepted_tokens"], s["avg_accept_rate"]) == \
        (0, 0, 0, 0.0)
    assert s["speedup_estimate"] >= 1.0
    dec._stats.update(total_steps=10, total_draft_tokens=50, total_accepted_tokens=35, avg_accept_rate=0.7)
    dec._current_depth = 4
    s = dec.get_stats()
    assert s["total_steps"] == 10 and s["current_depth"] == 4
    assert s["speedup_estimate"] == pytest.approx(2.8)


def test_generate_is_lossless_against_greedy(dec):
    dec.setup_draft_head(32, 50)
    ids = torch.randint(0, 50, (1, 6))
    out = asyncio.run(dec.generate(ids, max_new_tokens=10))
    cur, ref = ids, []
    for _ in range(10):
        nxt = dec.target(cur).logits[0, -1].argmax()
        ref.append(int(nxt))
        cur = torch.cat([cur, nxt.view(1, 1)], 1)
    assert out.tokens == ref
    assert 0.0 <= out.accept_rate <= 1.0 and out.draft_tokens >= out.accepted_tokens


# ----------------------------------------------------------------------------- medusa

def test_medusa_heads_and_shapes():
    m = MedusaHead(hidden_size=64, vocab_size=100, num_heads=4, hidden_dim=16)
    assert m.num_heads == 4 and len(m.heads) == 4
    outs = m(torch.randn(2, 10, 64))
    assert len(outs) == 4 and all(o.shape == (2, 10, 100) for o in outs)


@pytest.mark.parametrize("nh,b", [(1, 1), (2, 4), (8, 8)])
def test_medusa_variants(nh, b):
    outs = MedusaHead(64, 100, num_heads=nh, hidden_dim=16)(torch.randn(b, 5, 64))
    assert len(outs) == nh and all(o.shape[0] == b for o in outs)


def test_draft_head_feeds_tree_buffer():
    d = DraftHead(64, 100)
    d.set_token_embedding(nn.Embedding(100, 64))
    h = d(torch.randn(1, 5, 64), torch.randint(0, 100, (1, 5)))
    assert h.shape == (1, 5, 64)
    lp, idx = torch.topk(torch.randn(1, 100), k=3)
    b = TreeDraftBuffer(3, 3, "cpu")
    b.add_candidates(idx.squeeze(), lp.squeeze(), torch.zeros(3, dtype=torch.long))
    assert b.get_tree_tokens().shape == (3,)


# ----------------------------------------------------------------------------- device tree ops (CPU path)

def _brute_ancestors(parent):
    n = len(parent)
    anc = torch.zeros(n, n, dtype=torch.bool)
    for i in range(n):
        j = i
        while j >= 0:
            anc[i, j] = True
            j = parent[j]
    return anc


def test_tree_mask_op_matches_brute_force():
    # node 0 is the root (last accepted token); the rest is a drafted tree
    parent = [-1, 0, 0, 1, 1, 2, 5]
    anc_bits, depth = ops.tree_mask(torch.tensor([parent], dtype=torch.int32))
    brute = _brute_ancestors(parent)
    got = torch.tensor([[bool((int(anc_bits[0, i]) >> j) & 1) for j in range(len(parent))]
                        for i in range(len(parent))])
    assert torch.equal(got, brute)
    assert depth[0].tolist() == [0, 1, 1, 2, 2, 2, 3]


def test_tree_verify_op_accepts_longest_matching_path():
    parent = torch.tensor([[-1, 0, 0, 1, 2, 4]], dtype=torch.int32)
    draft = torch.tensor([[0, 11, 12, 13, 14, 15]])
    # target's greedy choice after each node: root->12, node2->14, node4->99 (rejects 15)
    target = torch.tensor([[12, 0, 14, 0, 99, 0]])
    anc, depth = ops.tree_mask(parent)
    acc, path, toks = ops.tree_verify(parent, draft, target, anc, depth, max_path=4)
    assert int(acc[0]) == 2
    assert path[0, :3].tolist() == [0, 2, 4]
    assert toks[0, :3].tolist() == [12, 14, 99]   # two accepted drafts + the bonus token
