"""CPU behaviour of dgi.ops: reference implementations (the GPU tests' oracles)
and the dispatch rules that decide which native kernel a GPU call takes."""
import math

import pytest

import torch
import torch.nn.functional as F

from dgi import ops


def test_linear_cpu_falls_back_to_torch():
    x = torch.randn(3, 64)
    w = torch.randn(32, 64)
    b = torch.randn(32)
    torch.testing.assert_close(ops.linear(x, w, b), F.linear(x, w, b))
    x3 = torch.randn(2, 3, 64)                       # non-2-D activations keep torch semantics
    torch.testing.assert_close(ops.linear(x3, w), F.linear(x3, w))
    out = torch.empty(3, 32)
    assert ops.linear(x, w, out=out) is out


def test_skinny_dispatch_follows_the_measured_table():
    # 8B-class projections at decode M: qkv, o, gate_up
    assert ops._use_skinny(1, 6144, 4096) and ops._use_skinny(8, 28672, 4096)
    assert ops._use_skinny(16, 4096, 4096) and not ops._use_skinny(32, 4096, 4096)
    assert not ops._use_skinny(16, 6144, 4096)       # above M = 8 only the square o-proj
    # hipBLASLt already streams these at 4.5-5.7 TB/s
    assert not ops._use_skinny(1, 4096, 14336)        # 8B down
    assert not ops._use_skinny(1, 128256, 4096)       # vocab head
    assert not ops._use_skinny(1, 10240, 8192)        # 70B qkv
    # shapes the kernel cannot tile
    assert not ops._use_skinny(1, 4096, 896) and not ops._use_skinny(1, 4104, 4096)


def test_rmsnorm_and_silu_mul_references():
    x = torch.randn(5, 256, dtype=torch.bfloat16)
    w = torch.randn(256, dtype=torch.bfloat16)
    xf = x.float()
    ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    torch.testing.assert_close(ops.rmsnorm(x, w, 1e-5).float(), ref, atol=2e-2, rtol=2e-2)
    gu = torch.randn(4, 2 * 96, dtype=torch.bfloat16)
    g, u = gu.float()[:, :96], gu.float()[:, 96:]
    torch.testing.assert_close(ops.silu_mul(gu).float(), F.silu(g) * u, atol=2e-2, rtol=2e-2)


def test_tree_mask_reference_marks_ancestors_and_depth():
    # root 0 -> 1, 2 ; 1 -> 3 ; 3 -> 4
    parent = torch.tensor([[-1, 0, 0, 1, 3]], dtype=torch.int32)
    anc, depth = ops.tree_mask(parent)
    assert depth[0].tolist() == [0, 1, 1, 2, 3]
    want = {0: {0}, 1: {0, 1}, 2: {0, 2}, 3: {0, 1, 3}, 4: {0, 1, 3, 4}}
    for n, s in want.items():
        row = int(anc[0, n])
        assert {i for i in range(5) if row >> i & 1} == s


def _brute_threshold(row, T, k, p):
    """Literal per-element definition of the top-k / top-p keep rule."""
    vals = [float(v) for v in row]
    in_k = [v for v in vals if sum(1 for u in vals if u > v) < k]
    z_k = sum(math.exp((v - max(vals)) / T) for v in in_k)      # nucleus mass renormalised over top-k
    kept = [v for v in in_k
            if sum(math.exp((u - max(vals)) / T) for u in vals if u > v) <= p * z_k]
    return min(kept) if len(kept) < len(vals) else float("-inf")


def test_topkp_threshold_reference_matches_definition():
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(6, 40, generator=g) * 2
    logits[3, :10] = logits[3, 10]        # ties straddling the cut
    temps = torch.tensor([1.0, 0.7, 1.3, 1.0, 0.5, 2.0])
    ks = torch.tensor([5, 0, 12, 3, 40, 0])
    ps = torch.tensor([1.0, 0.9, 0.5, 0.8, 0.95, 1.0])
    th = ops.topkp_threshold(logits, temps, ks, ps)
    for b in range(6):
        k = int(ks[b]) if int(ks[b]) > 0 else 10 ** 9
        want = _brute_threshold(logits[b].tolist(), float(temps[b]), k, float(ps[b]))
        if b == 5:
            want = float("-inf")                # top_k off and top_p = 1: no filter
        assert float(th[b]) == want, (b, float(th[b]), want)
    # top_k alone keeps exactly k distinct values; masking and greedy rows
    masked = ops.apply_top_k_top_p(logits, ks, ps, temps)
    assert int(torch.isfinite(masked[0]).sum()) == 5
    th0 = ops.topkp_threshold(logits, torch.zeros(6), ks, ps)
    assert torch.isinf(th0).all()


def test_sample_with_filter_stays_inside_the_kept_set():
    g = torch.Generator().manual_seed(1)
    logits = torch.randn(16, 300, generator=g)
    temps = torch.full((16,), 0.8)
    ks = torch.full((16,), 7)
    ps = torch.full((16,), 0.9)
    th = ops.topkp_threshold(logits, temps, ks, ps)
    out = ops.sample(logits, temps, torch.arange(16), 2, top_k=ks, top_p=ps)
    picked = logits.gather(1, out[:, None]).squeeze(1)
    assert bool((picked >= th).all())


def test_topkp_matches_hf_topk_then_topp_warpers():
    """Literal HF order: TopKLogitsWarper, then TopPLogitsWarper on the masked
    (renormalised) scores.  The flat row is where renormalising matters: top-50
    of 100 near-equal logits hold ~half the mass, so a full-vocab nucleus rule
    would keep all 50 while HF keeps ~45."""
    from transformers.generation.logits_process import TopKLogitsWarper, TopPLogitsWarper

    g = torch.Generator().manual_seed(3)
    logits = torch.randn(5, 100, generator=g) * 1.5
    logits[0] = torch.linspace(0.0, 0.01, 100)          # flat row
    temps = torch.tensor([1.0, 0.8, 1.0, 1.2, 0.6])
    ks = torch.tensor([50, 50, 10, 0, 20])
    ps = torch.tensor([0.9, 0.9, 0.5, 0.7, 0.99])
    masked = ops.apply_top_k_top_p(logits, ks, ps, temps)
    for b in range(5):
        sc = (logits[b: b + 1] / temps[b]).double()
        if int(ks[b]) > 0:
            sc = TopKLogitsWarper(int(ks[b]))(None, sc)
        sc = TopPLogitsWarper(float(ps[b]))(None, sc)
        want = torch.isfinite(sc[0])
        got = torch.isfinite(masked[b])
        assert torch.equal(got, want), (b, int(got.sum()), int(want.sum()))
    assert int(torch.isfinite(masked[0]).sum()) < 50


def test_running_set_is_an_ordered_o1_set():
    from dgi.sched.request import Request, SamplingParams
    from dgi.sched.scheduler import RunningSet
    rs = RunningSet()
    reqs = [Request([1, 2, 3], SamplingParams()) for _ in range(5)]
    for r in reqs:
        rs.append(r)
    rs.remove(reqs[1])
    rs.discard(reqs[1])
    assert list(rs) == [reqs[0], reqs[2], reqs[3], reqs[4]] and len(rs) == 4
    assert list(reversed(rs))[0] is reqs[4] and reqs[2] in rs and reqs[1] not in rs
    for r in rs:                      # iteration is a snapshot: removal inside the loop is safe
        rs.remove(r)
    assert not rs


def test_debug_modes_are_opt_in(monkeypatch):
    from dgi.utils import debug
    monkeypatch.delenv("DGI_DEBUG_SYNC", raising=False)
    monkeypatch.delenv("DGI_DEBUG_STREAMS", raising=False)
    assert not debug.sync_enabled() and debug.stream_checker() is None
    debug.after_op("noop")                         # no GPU / disabled: a no-op
    monkeypatch.setenv("DGI_DEBUG_STREAMS", "1")
    chk = debug.stream_checker()
    t = torch.zeros(4)
    rec = chk.on_send(t)
    chk.on_complete(rec)                           # untouched buffer: fine
    rec = chk.on_send(t)
    t.add_(1)
    with pytest.raises(debug.StreamOrderError):
        chk.on_complete(rec)
    monkeypatch.setenv("HIP_LAUNCH_BLOCKING", "0")
    monkeypatch.setenv("DGI_DEBUG_SYNC", "0")
    monkeypatch.setenv("AMD_SERIALIZE_KERNEL", "0")
    monkeypatch.delenv("AMD_SERIALIZE_KERNEL")
    debug.enable_serialized()
    import os
    assert os.environ["DGI_DEBUG_SYNC"] == "1" and os.environ["AMD_SERIALIZE_KERNEL"] == "3"


def test_fused_decode_layers_match_unfused_on_cpu():
    """The fused decode layer wiring (norm prologue, ping-pong residual, RoPE/KV and
    SwiGLU epilogues) computes exactly the unfused layer on the reference ops."""
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.models.config import get_config
    from dgi.models.llama import LlamaModel
    from dgi.sched.request import SamplingParams
    for name, mix in (("llama-tiny-hd128", (True, True)), ("qwen-tiny", (True, False)), ("glm-tiny", (True, True)),
                      ("llama-tiny-hd128", (False, True))):
        mc = get_config(name)
        outs, logits = [], []
        for fused in (False, True):
            m = LlamaModel(mc, "cpu", torch.float32, seed=11)
            m.force_fused = fused
            if fused:
                m._fused_decode = lambda h, meta, mix=mix: mix if meta.num_prefill_tokens == 0 else (False, False)
            calls = []
            real_fused = m._forward_layers_fused

            def count(*a, real_fused=real_fused, calls=calls):
                calls.append(1)
                return real_fused(*a)
            m._forward_layers_fused = count
            e = LLMEngine(EngineConfig(model=name, device="cpu", dtype=torch.float32, num_blocks=64, max_num_seqs=4,
                                       max_model_len=256, max_num_batched_tokens=64, use_graphs=False,
                                       enable_prefix_caching=False), model_cfg=mc, model=m)
            got = []
            orig = m.compute_logits

            def spy(h, r, idx, orig=orig, got=got):
                o = orig(h, r, idx)
                got.append(o.detach().clone())
                return o
            m.compute_logits = spy
            reqs = e.generate([[1, 5, 9, 300, 17], [1, 2, 3]], SamplingParams(max_tokens=6, temperature=0.0,
                                                                              ignore_eos=True))
            outs.append([r.output for r in reqs])
            logits.append(got)
            assert (len(calls) >= 5) == fused, (name, fused, len(calls))
        assert outs[0] == outs[1], name
        for a, b in zip(*logits):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)


def test_fused_layers_take_small_prefill_steps(monkeypatch):
    """Steps of <= 16 rows with prefill tokens (short prompts, an EAGLE tree verify) run
    the fused decode layers (per-row norm / RoPE / KV-write epilogues, attention split into
    decode and prefill rows) and produce the unfused model's logits; larger prefill steps
    stay unfused."""
    import dgi.models.llama as llama
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.models.config import get_config
    from dgi.models.llama import LlamaModel
    from dgi.sched.request import SamplingParams
    mc = get_config("llama-tiny-hd128")
    res = {}
    for flag in (False, True):
        monkeypatch.setattr(llama, "FUSED_SMALL_PREFILL", flag)
        m = LlamaModel(mc, "cpu", torch.float32, seed=11)
        m.force_fused = flag
        rows = []
        real = m._forward_layers_fused
        m._forward_layers_fused = lambda h, meta, *a, real=real, rows=rows: (
            rows.append((h.shape[0], meta.num_prefill_tokens)) or real(h, meta, *a))
        e = LLMEngine(EngineConfig(model="llama-tiny-hd128", device="cpu", dtype=torch.float32, num_blocks=64,
                                   max_num_seqs=4, max_model_len=256, max_num_batched_tokens=16, use_graphs=False,
                                   enable_prefix_caching=False), model_cfg=mc, model=m)
        got = []
        orig = m.compute_logits
        m.compute_logits = lambda h, r, idx, orig=orig, got=got: got.append(orig(h, r, idx).detach().clone()) or got[-1]
        reqs = e.generate([[1, 5, 9, 300, 17], [1, 2, 3], list(range(7, 47))],
                          SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))
        res[flag] = ([r.output for r in reqs], got, rows)
    outs0, logits0, rows0 = res[False]
    outs1, logits1, rows1 = res[True]
    assert not rows0
    assert any(p > 0 for t, p in rows1)        # chunked prefill steps of <= 16 rows went fused
    assert outs0 == outs1
    for a, b in zip(logits0, logits1):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)


def test_mlp_pad_table_picks_cheapest_rows_and_reports_impl():
    from dgi.runtime.gemm_pad import MlpPadTable
    grid = [512, 544, 576, 608]
    t = MlpPadTable(grid, [10.0, 12.0, 9.0, 11.0], 32,
                    impls=[(False, False), (True, False), (True, True), (False, True)])
    assert t.pad(520) == 576          # within +15 %: the 576-row run is the cheapest
    assert t.pad(100) == 100          # below the table: no say
    assert t.impl(576) == (True, True) and t.impl(544) == (True, False)
    assert t.impl(550) == (False, False) and t.impl(4096) == (False, False)


def test_layer_truncated_model_name():
    from dgi.models.config import get_config
    c = get_config("llama3-70b@L8")
    full = get_config("llama3-70b")
    assert c.num_layers == 8 and c.hidden_size == full.hidden_size and c.num_kv_heads == full.num_kv_heads


def test_trimmed_last_layer_matches_full(monkeypatch):
    """Prefill steps run the last layer's o-proj + MLP only on the rows that
    produce logits; the sampled tokens and logits equal the untrimmed model's."""
    import dgi.models.llama as llama
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.sched.request import SamplingParams
    cfg = EngineConfig(model="llama-tiny", device="cpu", max_num_seqs=4, max_num_batched_tokens=64,
                       max_model_len=256, use_graphs=False, num_blocks=64)
    g = torch.Generator().manual_seed(5)
    prompts = [torch.randint(5, 500, (n,), generator=g).tolist() for n in (37, 20, 51)]
    sp = SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True)
    outs = {}
    for flag in (True, False):
        monkeypatch.setattr(llama, "TRIM_LAST_LAYER", flag)
        eng = LLMEngine(cfg)
        outs[flag] = [r.output for r in eng.generate(prompts, sp)]
    assert outs[True] == outs[False]


def test_fused_decode_honours_trim_last_on_padded_batch():
    """A padded pure-decode batch (pipeline stage without graphs: T = bucket > nlog
    rows) through the fused decode layers returns exactly nlog logits rows — the
    sampler's per-row views are nlog long (llama.py fused early return)."""
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.sched.request import SamplingParams
    e = LLMEngine(EngineConfig(model="llama-tiny-hd128", device="cpu", dtype=torch.float32, num_blocks=64,
                               max_num_seqs=4, max_model_len=256, max_num_batched_tokens=64, use_graphs=False,
                               enable_prefix_caching=False))
    for p in ([1, 5, 9, 300, 17], [1, 2, 3]):
        e.add_request(p, SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True))
    e.step()                                   # both prompts prefilled: the next batch is pure decode
    sb = e.scheduler.schedule()
    assert len(sb.decode) == 2 and not sb.prefill
    r = e.runner
    flat, hdr, sampled = r.build_host(sb, pad_decode_to=4)
    ids, meta, samp = r.meta_from_device(r.to_device(flat), hdr)
    ref = e.model.forward(meta, input_ids=ids)
    e.model.force_fused = True
    calls = []
    real = e.model._forward_layers_fused
    e.model._forward_layers_fused = lambda *a: calls.append(1) or real(*a)
    got = e.model.forward(meta, input_ids=ids)
    assert calls and got.shape[0] == len(sampled) == 2
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)
    assert samp.sample(got).shape[0] == 2


def test_gemm_table_decides_with_margin_and_round_trips_json(tmp_path):
    """The routing table keeps the raw per-implementation times: the MFMA kernel is chosen
    only where it beats hipBLASLt by >= 3 % (near-ties stay on hipBLASLt, so passes agree),
    the median of several passes decides the shipped table, and a table written to JSON
    loads back with the same choices."""
    import json
    from dgi.runtime.gemm_pad import MlpPadTable, RAW_KEYS

    def pt(front, front_m, back, back_m, pq=(1.0, None), po=(1.0, None)):
        r = dict.fromkeys(RAW_KEYS)
        r.update(front=front, front_mfma=front_m, back=back, back_mfma=back_m, pq_blas=pq[0], pq_mfma=pq[1],
                 po_blas=po[0], po_mfma=po[1])
        return r
    grid = [512, 544]
    raw = [pt(10.0, 9.8, 5.0, 4.0, pq=(2.0, 1.5)), pt(10.0, 9.0, 5.0, 4.9, po=(1.0, 0.5))]
    t = MlpPadTable.decide(grid, raw, 32)
    assert t.impl(512) == (False, True)            # 2 % faster gate_up: not enough; down 20 %: MFMA
    assert t.impl(544) == (True, False)            # 10 % vs 2 %
    assert t.proj_impl(512) == (True, False) and t.proj_impl(544) == (False, True)
    assert t.times == [10.0 + 4.0, 9.0 + 5.0]
    runs = [raw, [pt(10.0, 9.0, 5.0, 4.0), pt(10.0, 9.0, 5.0, 4.9)], [pt(10.0, 9.9, 5.0, 4.0), pt(10.0, 9.1, 5.0, 4.9)]]
    med = MlpPadTable.median_raw(runs)
    assert med[0]["front_mfma"] == 9.8 and med[1]["front_mfma"] == 9.0
    p = tmp_path / "t.json"
    p.write_text(json.dumps(t.to_json({"k": 1})))
    back = MlpPadTable.from_json(json.loads(p.read_text()))
    assert back.impls == t.impls and back.proj_impls == t.proj_impls and back.source == "shipped"


@pytest.mark.parametrize("name", ["llama-tiny-hd128", "llama-tiny-tp"])
def test_fused_norm_layer_composition_matches_unfused_cpu(monkeypatch, name):
    """The fused-norm layer composition (gains folded into the weights, residual + row
    statistics from the o / down epilogues, rstd applied by qkv / gate_up) through the fp32
    reference ops equals the unfused layers: whole-sequence logits, the trimmed last layer and
    the EAGLE-3 feature taps."""
    from dgi.models import llama
    from dgi.models.config import get_config
    from dgi.models.llama import LlamaModel
    from dgi.runtime.batch import AttnMeta
    mc = get_config(name)            # tiny-tp (2 kv heads): the qkv GEMM also takes the RoPE + KV epilogue
    ref = LlamaModel(mc, "cpu", torch.float32, seed=9)
    fold = LlamaModel(mc, "cpu", torch.float32, init="empty").copy_from(ref)
    fold.fold_norms()
    assert fold.norms_folded and torch.equal(fold.layers[0].in_norm, torch.ones_like(fold.layers[0].in_norm))
    T = 37
    ids = torch.randint(3, 1000, (T,), generator=torch.Generator().manual_seed(2))
    outs = {}
    for name, m, mode in (("ref", ref, "0"), ("fold", fold, "force-cpu")):
        monkeypatch.setattr(llama, "NORM_FOLD", mode)
        monkeypatch.setattr(llama, "NORM_FOLD_MIN_ROWS", 1)
        nb = 8
        m.kv_cache = torch.zeros(mc.num_layers, 2, nb, mc.num_kv_heads, 16, mc.head_dim)
        meta = AttnMeta(positions=torch.arange(T), slot_mapping=torch.arange(16, 16 + T), num_decode=0,
                        num_prefill_tokens=T, pre_block_tables=torch.arange(1, nb, dtype=torch.int32)[None],
                        pre_cu_seqlens=torch.tensor([0, T], dtype=torch.int32),
                        pre_context_lens=torch.tensor([T], dtype=torch.int32), logits_indices=torch.tensor([T - 1]))
        m.capture_layers, m.captured = (0, mc.num_layers - 1), {}
        full = m.forward(AttnMeta(**{**meta.__dict__, "logits_indices": None}), input_ids=ids)
        feats = {k: v.clone() for k, v in m.captured.items()}
        m.capture_layers, m.captured = (), {}
        last = m.forward(meta, input_ids=ids)          # trimmed last layer
        outs[name] = (full, last, feats)
    (f0, l0, c0), (f1, l1, c1) = outs["ref"], outs["fold"]
    assert torch.allclose(f0, f1, atol=1e-3, rtol=1e-3)
    assert torch.allclose(l0, l1, atol=1e-3, rtol=1e-3) and torch.allclose(l1[-1], f1[-1], atol=1e-3, rtol=1e-3)
    for k in (0, mc.num_layers - 1):
        assert torch.allclose(c0[k], c1[k], atol=1e-3, rtol=1e-3)
