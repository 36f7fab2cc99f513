"""Numerics of every HIP kernel against its plain-PyTorch fp32 reference.

Run on an MI355X (``pytest -m gpu``).  Shapes cover GQA 8:1 (Llama-3),
ragged contexts, block tables with holes/out-of-order pages, chunked prefill
over a cached prefix, split-KV decode, and EAGLE tree masks.
"""
import math
import random

import pytest
import torch

from dgi import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _native():
    ops.load_native(required=True)


def _bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("T,H", [(1, 4096), (7, 8192), (33, 1024), (5, 768)])
def test_rmsnorm(T, H):
    x = _bf(T, H)
    w = _bf(H)
    out = ops.rmsnorm(x, w, 1e-5)
    ref = ops.rmsnorm_ref(x, w, 1e-5)
    torch.testing.assert_close(out.float(), ref.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("T,H", [(3, 4096), (16, 8192)])
def test_fused_add_rmsnorm(T, H):
    x = _bf(T, H)
    r = _bf(T, H)
    w = _bf(H)
    x2, r2 = x.clone(), r.clone()
    ops.fused_add_rmsnorm(x, r, w, 1e-5)
    ops.fused_add_rmsnorm_ref(x2, r2, w, 1e-5)
    torch.testing.assert_close(r.float(), r2.float(), atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(x.float(), x2.float(), atol=3e-2, rtol=3e-2)


def _make_cache(nblocks, nkv, bs, hd):
    k = _bf(nblocks, nkv, bs, hd)
    v = _bf(nblocks, nkv, bs, hd)
    return k, v


@pytest.mark.parametrize("nh,nkv,hd,rd,mode", [(32, 8, 128, 128, 0), (8, 1, 64, 64, 0), (64, 8, 128, 128, 0),
                                               (32, 2, 128, 64, 1), (8, 2, 128, 128, 1), (16, 4, 128, 64, 0)])
def test_rope_cache(nh, nkv, hd, rd, mode):
    """NeoX (mode 0) and interleaved GLM-style (mode 1) pairing, full and partial rotary dims."""
    T, bs, nb = 19, 16, 40
    qkv = _bf(T, (nh + 2 * nkv) * hd)
    pos = torch.randint(0, 4000, (T,), device=DEV, dtype=torch.int32)
    slots = torch.randperm(nb * bs, device=DEV)[:T].to(torch.int32)
    slots[3] = -1
    cs = ops.rope_cos_sin(rd, 4096, 500000.0 if mode == 0 else 10000.0, device=DEV)
    k1, v1 = _make_cache(nb, nkv, bs, hd)
    k2, v2 = k1.clone(), v1.clone()
    q1, q2 = qkv.clone(), qkv.clone()
    ops.rope_cache(q1, pos, cs, nh, nkv, hd, slots, k1, v1, mode)
    ops.rope_cache_ref(q2, pos, cs, nh, nkv, hd, slots, k2, v2, mode)
    torch.testing.assert_close(q1[:, : nh * hd].float(), q2[:, : nh * hd].float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(k1.float(), k2.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(v1.float(), v2.float(), atol=0, rtol=0)


def _block_tables(ctx_lens, bs, nblocks, maxw):
    ids = list(range(1, nblocks))
    random.Random(0).shuffle(ids)
    bt = torch.zeros(len(ctx_lens), maxw, dtype=torch.int32)
    k = 0
    for b, c in enumerate(ctx_lens):
        n = (c + bs - 1) // bs
        bt[b, :n] = torch.tensor(ids[k:k + n], dtype=torch.int32)
        k += n
    return bt.to(DEV)


@pytest.mark.parametrize("nh,nkv,hd", [(32, 8, 128), (64, 8, 128), (8, 1, 64), (8, 8, 128), (28, 4, 128),
                                       (14, 2, 64)])
@pytest.mark.parametrize("ctx_lens", [[1], [17, 300, 64, 1000], [4097, 33]])
def test_paged_decode(nh, nkv, hd, ctx_lens):
    """Every plan: one split, split + reduce kernel, fixed parts, device-side plan + ticket reduce."""
    _paged_decode_case(nh, nkv, hd, ctx_lens)


@pytest.mark.parametrize("bs", [8, 32, 64])
def test_paged_decode_block_sizes(bs):
    """32-token tiles over 4 / 1 / half a block of the paged pool."""
    _paged_decode_case(32, 8, 128, [1, 33, 700, 2100], bs=bs)


def _paged_decode_case(nh, nkv, hd, ctx_lens, bs=16):
    maxw = max(300, max((c + bs - 1) // bs for c in ctx_lens))
    nblocks = sum((c + bs - 1) // bs for c in ctx_lens) + 8
    kc, vc = _make_cache(nblocks, nkv, bs, hd)
    bt = _block_tables(ctx_lens, bs, nblocks, maxw)
    ctx = torch.tensor(ctx_lens, dtype=torch.int32, device=DEV)
    B = len(ctx_lens)
    qkv = _bf(B, (nh + 2 * nkv) * hd)
    scale = 1 / math.sqrt(hd)
    ref = ops.paged_decode_ref(qkv, kc, vc, bt, ctx, nh, nkv, scale)
    # single split
    out1 = ops.paged_decode(qkv, kc, vc, bt, ctx, nh, nkv, scale, 1, 1 << 20)
    torch.testing.assert_close(out1.float(), ref.float(), atol=2e-2, rtol=2e-2)
    # split-KV
    splits, part = ops.decode_split_plan(B, max(ctx_lens), nkv)
    out2 = ops.paged_decode(qkv, kc, vc, bt, ctx, nh, nkv, scale, splits, part)
    torch.testing.assert_close(out2.float(), ref.float(), atol=2e-2, rtol=2e-2)
    # fixed part 128 with many splits (graph style: empty splits exit)
    out3 = ops.paged_decode(qkv, kc, vc, bt, ctx, nh, nkv, scale, (max(ctx_lens) + 127) // 128 + 3, 128)
    torch.testing.assert_close(out3.float(), ref.float(), atol=2e-2, rtol=2e-2)
    # separate reduce kernel (no ticket counters in the workspace)
    ws2 = (torch.empty(B * nh * splits * hd, device=DEV), torch.empty(B * nh * splits, device=DEV))
    out4 = ops.paged_decode(qkv, kc, vc, bt, ctx, nh, nkv, scale, splits, part, workspace=ws2)
    torch.testing.assert_close(out4.float(), ref.float(), atol=2e-2, rtol=2e-2)
    # device-side dynamic plan (graphs): up to S parts of >= 64 tokens, in-kernel reduce;
    # the ticket counters must be back to zero after every launch
    for S in (1, 3, 16, 64):
        ws = (torch.empty(B * nh * S * hd, device=DEV), torch.empty(B * nh * S, device=DEV),
              torch.zeros(B * nkv, dtype=torch.int32, device=DEV))
        for _ in range(2):
            out5 = ops.paged_decode(qkv, kc, vc, bt, ctx, nh, nkv, scale, S, -64, workspace=ws)
            torch.testing.assert_close(out5.float(), ref.float(), atol=2e-2, rtol=2e-2)
        assert int(ws[2].abs().sum()) == 0


@pytest.mark.parametrize("nh,nkv,hd", [(32, 8, 128), (64, 8, 128), (8, 1, 128), (28, 4, 128), (32, 8, 64),
                                       (14, 2, 64)])
@pytest.mark.parametrize("qlens,ctxs", [([5], [5]), ([130, 1, 64], [130, 40, 600]), ([512], [512]),
                                        ([300, 77], [1000, 77])])
@pytest.mark.parametrize("tile,db", [(128, 1), (128, 0), (256, 1)])
def test_paged_prefill(nh, nkv, hd, qlens, ctxs, tile, db, monkeypatch):
    monkeypatch.setattr(ops, "PREFILL_TILE", tile)
    monkeypatch.setattr(ops, "PREFILL_DB", db)
    bs = 16
    maxw = 80
    nblocks = sum((c + bs - 1) // bs for c in ctxs) + 4
    kc, vc = _make_cache(nblocks, nkv, bs, hd)
    bt = _block_tables(ctxs, bs, nblocks, maxw)
    cu = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0).tolist()), dtype=torch.int32, device=DEV)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    T = sum(qlens)
    q = _bf(T, (nh + 2 * nkv) * hd)
    scale = 1 / math.sqrt(hd)
    ref = ops.paged_prefill_ref(q, kc, vc, bt, cu, ctx, nh, nkv, scale)
    out = ops.paged_prefill(q, kc, vc, bt, cu, ctx, nh, nkv, scale)
    torch.testing.assert_close(out.float(), ref.float(), atol=2e-2, rtol=2e-2)


def test_paged_prefill_tree_mask():
    nh, nkv, hd, bs = 32, 8, 128, 16
    # 2 sequences with cached prefixes 40 / 100 and a 7-node draft tree each
    par = torch.tensor([[-1, 0, 0, 1, 1, 2, 3], [-1, 0, 1, 1, 0, 4, 5]], dtype=torch.int32)
    anc, _ = ops.tree_mask_ref(par)
    N = 7
    ctxs = [40 + N, 100 + N]
    nblocks = 20
    kc, vc = _make_cache(nblocks, nkv, bs, hd)
    bt = _block_tables(ctxs, bs, nblocks, 16)
    cu = torch.tensor([0, N, 2 * N], dtype=torch.int32, device=DEV)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    q = _bf(2 * N, (nh + 2 * nkv) * hd)
    scale = 1 / math.sqrt(hd)
    tm = anc.to(DEV)
    ref = ops.paged_prefill_ref(q, kc, vc, bt, cu, ctx, nh, nkv, scale, tm, N)
    out = ops.paged_prefill(q, kc, vc, bt, cu, ctx, nh, nkv, scale, tree_mask=tm, tree_n=N)
    torch.testing.assert_close(out.float(), ref.float(), atol=2e-2, rtol=2e-2)
    # a plain causal run differs (the mask matters)
    plain = ops.paged_prefill(q, kc, vc, bt, cu, ctx, nh, nkv, scale)
    assert (plain.float() - ref.float()).abs().max() > 1e-2


@pytest.mark.parametrize("T,I", [(1, 14336), (9, 28672), (64, 3072)])
def test_silu_mul(T, I):
    gu = _bf(T, 2 * I)
    torch.testing.assert_close(ops.silu_mul(gu).float(), ops.silu_mul_ref(gu).float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [1, 3, 16, 17, 32])
@pytest.mark.parametrize("N,K,cfg", [(6144, 4096, 0), (4096, 14336, 0), (1152, 1024, 1), (256, 1024, 4),
                                     (512, 2048, 2), (1024, 2048, 5), (512, 4096, 6), (96, 1024, 3),
                                     (512, 4096, 7), (256, 14336, 8), (512, 2048, 9), (256, 3072, 10),
                                     (512, 4096, 11), (128, 1024, 11)])
def test_skinny_gemm(M, N, K, cfg):
    if N % (16 * {2: 2, 3: 2, 5: 4, 6: 2}.get(cfg, 1)):
        pytest.skip("column tiles do not divide N")
    x = _bf(M, K)
    w = _bf(N, K, scale=0.05)
    b = _bf(N)
    ref = (x.float() @ w.float().t() + b.float())
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    torch.ops.dgi.skinny_gemm(out, x, w, b, cfg)
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=2e-2)
    # strided activation rows (a view into a wider buffer), no bias, via ops.linear
    xs = _bf(M, K + 64)[:, :K]
    y = ops.linear(xs, w)
    torch.testing.assert_close(y.float(), xs.float() @ w.float().t(), atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_sample_greedy_and_topk(dtype):
    B, V = 7, 128256
    logits = torch.randn(B, V, device=DEV).to(dtype)
    out = ops.sample(logits)
    assert torch.equal(out.cpu(), logits.float().argmax(-1).cpu())
    v, i = ops.topk(logits, 8)
    rv, ri = logits.float().topk(8, dim=-1)
    torch.testing.assert_close(v.cpu(), rv.cpu())
    # bf16 logits tie often: indices must point at the reported values, all distinct
    torch.testing.assert_close(logits.float().gather(1, i).cpu(), v.cpu())
    assert all(len(set(r)) == 8 for r in i.cpu().tolist())


@pytest.mark.parametrize("B,V,k", [(3, 128256, 4), (48, 128256, 8), (5, 32768, 1), (2, 1000, 8), (1, 8200, 2),
                                   (4, 128256, 12)])
def test_topk_logprobs_matches_log_softmax_topk(B, V, k):
    """Fused top-k of log_softmax (chunked HIP kernels straight from bf16 logits) against
    torch: same values to fp32 logsumexp rounding, indices pointing at the reported values,
    lower index first among equal logits (bf16 rows tie often)."""
    logits = (torch.randn(B, V, device=DEV) * 3).to(torch.bfloat16)
    v, i = ops.topk_logprobs(logits, k)
    ref = torch.log_softmax(logits.float(), dim=-1)
    rv, _ri = ref.topk(k, dim=-1)
    torch.testing.assert_close(v.cpu(), rv.cpu(), atol=2e-5, rtol=1e-5)
    torch.testing.assert_close(ref.gather(1, i).cpu(), v.cpu(), atol=2e-5, rtol=1e-5)
    il = i.cpu().tolist()
    assert all(len(set(r)) == k for r in il)
    lf = logits.float().cpu()
    for b in range(B):                   # ties: the lowest index of a tied value comes first
        for j in range(k - 1):
            if lf[b, il[b][j]] == lf[b, il[b][j + 1]]:
                assert il[b][j] < il[b][j + 1]
    # a strided row view (logits of a wider buffer)
    wide = torch.randn(B, V + 8, device=DEV).to(torch.bfloat16)
    v2, i2 = ops.topk_logprobs(wide[:, :V], k)
    rv2 = torch.log_softmax(wide[:, :V].float(), dim=-1).topk(k, dim=-1).values
    torch.testing.assert_close(v2.cpu(), rv2.cpu(), atol=2e-5, rtol=1e-5)


@pytest.mark.parametrize("V", [128256, 151936, 32000])
def test_sample_split_rows_match_one_workgroup_per_row(V):
    """Batches of <= 32 rows split each row over workgroups of 8192 logits (sample_part_kernel +
    sample_final_kernel); 33+ rows take one workgroup per row.  A row's pick depends only on its
    logits, seed and step, so the first rows of a 40-row call (unsplit) must equal an 8-row call
    of the same rows (split): greedy, Gumbel-sampled, and with top-k / top-p thresholds."""
    B = 40
    logits = (torch.randn(B, V, device=DEV) * 2).to(torch.bfloat16)
    temps = torch.rand(B, device=DEV) + 0.3
    temps[::3] = 0.0                                          # greedy rows mixed in
    seeds = torch.arange(B, device=DEV, dtype=torch.long) * 7 + 1
    ks = torch.tensor([0, 5, 50, 0] * (B // 4), device=DEV, dtype=torch.long)
    ps = torch.tensor([1.0, 1.0, 0.9, 0.7] * (B // 4), device=DEV)
    for kw in ({}, {"top_k": ks, "top_p": ps}):
        full = ops.sample(logits, temps, seeds, 5, **kw)
        for n in (1, 8, 32):
            kn = {k: v[:n] for k, v in kw.items()}
            part = ops.sample(logits[:n], temps[:n], seeds[:n], 5, **kn)
            assert torch.equal(part.cpu(), full[:n].cpu()), (n, kw.keys())
    assert torch.equal(ops.sample(logits[:4]).cpu(), logits[:4].float().argmax(-1).cpu())
    wide = torch.randn(4, V + 8, device=DEV).to(torch.bfloat16)     # strided rows
    assert torch.equal(ops.sample(wide[:, :V]).cpu(), wide[:, :V].float().argmax(-1).cpu())


def test_sample_temperature_distribution():
    V = 8
    logits = torch.log(torch.tensor([[0.5, 0.25, 0.125, 0.125, 1e-9, 1e-9, 1e-9, 1e-9]], device=DEV)).repeat(4096, 1)
    temps = torch.ones(4096, device=DEV)
    seeds = torch.arange(4096, device=DEV, dtype=torch.long)
    out = ops.sample(logits, temps, seeds, step=3)
    freq = torch.bincount(out.cpu(), minlength=V).float() / 4096
    assert abs(freq[0] - 0.5) < 0.05 and abs(freq[1] - 0.25) < 0.05 and freq[4:].sum() < 0.01


def test_kv_gather_scatter_copy():
    L, NB, nkv, bs, hd = 3, 20, 8, 16, 128
    cache = _bf(L, 2, NB, nkv, bs, hd)
    ids = torch.tensor([5, 1, 17], dtype=torch.int32, device=DEV)
    g = ops.kv_gather(cache, ids)
    assert torch.equal(g, cache[:, :, ids.long()])
    c2 = torch.zeros_like(cache)
    ops.kv_scatter(c2, ids, g)
    assert torch.equal(c2[:, :, ids.long()], g)
    src = torch.tensor([2, 3], dtype=torch.int32, device=DEV)
    dst = torch.tensor([10, 11], dtype=torch.int32, device=DEV)
    ops.kv_copy(cache, src, dst)
    assert torch.equal(cache[:, :, 10], cache[:, :, 2]) and torch.equal(cache[:, :, 11], cache[:, :, 3])
    # block-major (host KV tier slot layout): [n, L, 2, page], no permute pass
    gb = ops.kv_gather(cache, ids, block_major=True)
    assert gb.shape == (3, L, 2, nkv, bs, hd)
    assert torch.equal(gb, cache[:, :, ids.long()].permute(2, 0, 1, 3, 4, 5))
    c3 = torch.zeros_like(cache)
    ops.kv_scatter(c3, ids, gb, block_major=True)
    assert torch.equal(c3[:, :, ids.long()], cache[:, :, ids.long()])
    assert int((c3 != 0).sum()) == int((cache[:, :, ids.long()] != 0).sum())     # nothing else written


def test_tree_mask_verify():
    par = torch.tensor([[-1, 0, 0, 1, 1, 2, 3, 6]], dtype=torch.int32)
    anc_r, dep_r = ops.tree_mask_ref(par)
    anc, dep = ops.tree_mask(par.to(DEV))
    assert torch.equal(anc.cpu(), anc_r) and torch.equal(dep.cpu(), dep_r)
    draft = torch.tensor([[9, 11, 12, 13, 14, 15, 16, 17]], dtype=torch.long)
    # target argmax at each node: node0 -> 11 (accept node1), node1 -> 13 (accept node3),
    # node3 -> 16 (accept node6), node6 -> 17 (accept node7), node7 -> 99 (bonus)
    target = torch.tensor([[11, 13, 0, 16, 0, 0, 17, 99]], dtype=torch.long)
    acc_r, path_r, tok_r = ops.tree_verify_ref(par, draft, target, anc_r, dep_r, 6)
    acc, path, tok = ops.tree_verify(par.to(DEV), draft.to(DEV), target.to(DEV), anc, dep, 6)
    assert acc.item() == 4 == acc_r.item()
    assert torch.equal(path.cpu(), path_r) and torch.equal(tok.cpu(), tok_r)
    assert tok_r[0, :5].tolist() == [11, 13, 16, 17, 99]


def test_model_decode_matches_eager_and_graph():
    """Native GPU engine (eager and hipGraph) vs the pure-torch CPU engine, same weights."""
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.models.config import get_config
    from dgi.models.llama import LlamaModel
    from dgi.sched.request import SamplingParams
    mc = get_config("llama-tiny-hd128")
    cpu_model = LlamaModel(mc, "cpu", seed=3)
    prompts = [[1] + list(range(3, 3 + n)) for n in (5, 40, 130, 7)]
    sp = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True)
    outs = []
    for graphs in (False, True):
        gm = LlamaModel(mc, "cuda", init="empty").copy_from(cpu_model)
        e = LLMEngine(EngineConfig(model="llama-tiny-hd128", device="cuda", num_blocks=256, max_num_seqs=8,
                                   max_model_len=512, max_num_batched_tokens=256, use_graphs=graphs),
                      model_cfg=mc, model=gm)
        outs.append([r.output for r in e.generate(prompts, sp)])
    assert outs[0] == outs[1]
    # per step: the token the GPU chose is an argmax of the fp32 CPU model's logits for
    # the same prefix (teacher forced), up to a bf16 tolerance
    f32 = LlamaModel(mc, "cpu", torch.float32, init="empty").copy_from(cpu_model)
    ref_eng = LLMEngine(EngineConfig(model="llama-tiny-hd128", device="cpu", dtype=torch.float32, num_blocks=256,
                                     max_num_seqs=8, max_model_len=512, max_num_batched_tokens=256,
                                     use_graphs=False, enable_prefix_caching=False), model_cfg=mc, model=f32)
    got = {}
    orig = ref_eng.model.compute_logits

    def spy(h, residual, idx):
        out = orig(h, residual, idx)
        got["l"] = out[-1].detach().float()
        return out
    ref_eng.model.compute_logits = spy
    one = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
    for p, toks in zip(prompts, outs[0]):
        for t, tok in enumerate(toks):
            ref_eng.generate([p + toks[:t]], one)
            r = got["l"]
            tol = 0.03 * float(r.abs().max()) + 0.02
            assert float(r[tok]) >= float(r.max()) - tol, (len(p), t, tok, int(r.argmax()))


def _teacher_forced_ok(name, src_model, prompts, gpu_outs, rel=0.03, abs_=0.02):
    """Every token the GPU chose is an argmax of the fp32 CPU model's logits for the same
    prefix (teacher forced), up to a bf16 tolerance — per step, every prompt."""
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.models.llama import LlamaModel
    from dgi.sched.request import SamplingParams
    mc = src_model.cfg
    f32 = LlamaModel(mc, "cpu", torch.float32, init="empty").copy_from(src_model)
    ref = LLMEngine(EngineConfig(model=name, device="cpu", dtype=torch.float32, num_blocks=256, max_num_seqs=8,
                                 max_model_len=512, max_num_batched_tokens=256, use_graphs=False,
                                 enable_prefix_caching=False), model_cfg=mc, model=f32)
    got = {}
    orig = ref.model.compute_logits

    def spy(h, residual, idx):
        out = orig(h, residual, idx)
        got["l"] = out[-1].detach().float()
        return out
    ref.model.compute_logits = spy
    one = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
    checked = 0
    for p, toks in zip(prompts, gpu_outs):
        for t, tok in enumerate(toks):
            ref.generate([p + toks[:t]], one)
            r = got["l"]
            tol = rel * float(r.abs().max()) + abs_
            assert float(r[tok]) >= float(r.max()) - tol, (name, len(p), t, tok, int(r.argmax()))
            checked += 1
    return checked


def _teacher_forced_topk_ok(name, src_model, prompts, gpu_outs, k, rel=0.03, abs_=0.02):
    """Sampled runs: every token the GPU drew is inside the fp32 model's top-k for the
    same prefix (teacher forced), up to a bf16 tolerance — per step, every prompt."""
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.models.llama import LlamaModel
    from dgi.sched.request import SamplingParams
    mc = src_model.cfg
    f32 = LlamaModel(mc, "cpu", torch.float32, init="empty").copy_from(src_model)
    ref = LLMEngine(EngineConfig(model=name, device="cpu", dtype=torch.float32, num_blocks=256, max_num_seqs=8,
                                 max_model_len=512, max_num_batched_tokens=256, use_graphs=False,
                                 enable_prefix_caching=False), model_cfg=mc, model=f32)
    got = {}
    orig = ref.model.compute_logits

    def spy(h, residual, idx):
        out = orig(h, residual, idx)
        got["l"] = out[-1].detach().float()
        return out
    ref.model.compute_logits = spy
    one = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
    checked = 0
    for p, toks in zip(prompts, gpu_outs):
        for t, tok in enumerate(toks):
            ref.generate([p + toks[:t]], one)
            r = got["l"]
            kth = float(r.topk(k).values[-1])
            tol = rel * float(r.abs().max()) + abs_
            assert float(r[tok]) >= kth - tol, (name, len(p), t, tok, kth, float(r[tok]))
            checked += 1
    return checked


def test_qwen2_engine_gpu_matches_cpu():
    """Qwen2 family (biased QKV, GQA 7:1) through the native kernels vs the CPU engine."""
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.models.config import get_config
    from dgi.models.llama import LlamaModel
    from dgi.sched.request import SamplingParams
    mc = get_config("qwen-tiny")
    cpu_model = LlamaModel(mc, "cpu", seed=5)
    prompts = [[1] + list(range(7, 7 + n)) for n in (3, 60, 150)]
    sp = SamplingParams(max_tokens=10, temperature=0.0, ignore_eos=True)
    gm = LlamaModel(mc, "cuda", init="empty").copy_from(cpu_model)
    ge = LLMEngine(EngineConfig(model="qwen-tiny", device="cuda", num_blocks=128, max_num_seqs=4, max_model_len=512,
                                max_num_batched_tokens=256, use_graphs=True), model_cfg=mc, model=gm)
    gpu = [r.output for r in ge.generate(prompts, sp)]
    assert _teacher_forced_ok("qwen-tiny", cpu_model, prompts, gpu) == 30


def test_glm_engine_gpu_matches_cpu():
    """GLM-4 family (biased QKV, half-dim interleaved RoPE) through the native kernels vs the CPU engine."""
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.models.config import get_config
    from dgi.models.llama import LlamaModel
    from dgi.sched.request import SamplingParams
    mc = get_config("glm-tiny")
    cpu_model = LlamaModel(mc, "cpu", seed=7)
    prompts = [[1] + list(range(9, 9 + n)) for n in (4, 70, 140)]
    sp = SamplingParams(max_tokens=10, temperature=0.0, ignore_eos=True)
    gm = LlamaModel(mc, "cuda", init="empty").copy_from(cpu_model)
    ge = LLMEngine(EngineConfig(model="glm-tiny", device="cuda", num_blocks=128, max_num_seqs=4, max_model_len=512,
                                max_num_batched_tokens=256, use_graphs=True), model_cfg=mc, model=gm)
    gpu = [r.output for r in ge.generate(prompts, sp)]
    assert _teacher_forced_ok("glm-tiny", cpu_model, prompts, gpu) == 30


def test_mlp_row_padding_matches_unpadded():
    """Padding the MLP rows (o-proj into a padded buffer, gate_up/down on extra
    zero rows) leaves every real row's result unchanged."""
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.sched.request import SamplingParams
    e = LLMEngine(EngineConfig(model="llama-tiny-hd128", device=DEV, max_num_seqs=8, max_num_batched_tokens=2048,
                               max_model_len=1024, use_graphs=False))
    tab = e.mlp_pad_table
    assert tab is not None
    for T in (512, 700, 1500, 2048):
        p = tab.pad(T)
        assert T <= p <= T * 1.15 + 32 and p % 32 == 0
    g = torch.Generator().manual_seed(11)
    prompts = [torch.randint(5, 1000, (n,), generator=g).tolist() for n in (130, 257, 301, 90)]
    sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
    e.model.mlp_pad = None
    ref = [r.output for r in e.generate(prompts, sp)]
    e.model.mlp_pad = lambda T: T + 40 if T >= 64 else T
    out = [r.output for r in e.generate(prompts, sp)]
    assert out == ref


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_topkp_threshold_kernel_matches_reference(dtype):
    B, V = 24, 128256
    g = torch.Generator(device="cpu").manual_seed(5)
    logits = (torch.randn(B, V, generator=g) * 3).to(dtype)
    logits[7, 1000:] = float("-inf")                       # masked vocab tail
    logits[5] = 1.0                                        # constant row
    temps = torch.tensor([0.0, 1.0, 0.7, 1.5] * 6)
    ks = torch.tensor([0, 50, 1, 2000, 0, 50] * 4)
    ps = torch.tensor([0.9, 1.0, 0.95, 0.5, 0.8, 0.999] * 4)
    ref = ops.topkp_threshold(logits, temps, ks, ps)       # CPU reference (sort based)
    lg = logits.to(DEV)
    th = ops.topkp_threshold(lg, temps.to(DEV), ks.to(DEV), ps.to(DEV)).cpu()
    kept_ref = (logits.float() >= ref[:, None]).sum(-1)
    kept = (logits.float() >= th[:, None]).sum(-1)
    for b in range(B):
        # same set up to fp32 summation order at the nucleus boundary
        assert abs(int(kept[b]) - int(kept_ref[b])) <= max(2, int(0.002 * int(kept_ref[b]))), \
            (b, int(kept[b]), int(kept_ref[b]), float(th[b]), float(ref[b]))
    # sampling stays inside the cut; unfiltered rows match the plain sampler
    seeds = torch.arange(B, device=DEV)
    out = ops.sample(lg, temps.to(DEV), seeds, 3, top_k=ks.to(DEV), top_p=ps.to(DEV))
    picked = lg.float().gather(1, out[:, None]).squeeze(1).cpu()
    assert bool((picked >= th).all())
    off = torch.zeros(B, dtype=torch.long, device=DEV), torch.ones(B, device=DEV)
    a = ops.sample(lg, temps.to(DEV), seeds, 3, top_k=off[0], top_p=off[1])
    assert torch.equal(a, ops.sample(lg, temps.to(DEV), seeds, 3))


def test_topkp_sampling_distribution():
    V = 8
    probs = torch.tensor([0.4, 0.3, 0.2, 0.05, 0.05, 0, 0, 0]) + 1e-9
    logits = torch.log(probs)[None].repeat(8192, 1).to(DEV)
    temps = torch.ones(8192, device=DEV)
    seeds = torch.arange(8192, device=DEV)
    ks = torch.full((8192,), 0, dtype=torch.long, device=DEV)
    ps = torch.full((8192,), 0.6, device=DEV)               # nucleus = {0, 1} (0.4 <= 0.6 < 0.7)
    out = ops.sample(logits, temps, seeds, 1, top_k=ks, top_p=ps).cpu()
    freq = torch.bincount(out, minlength=V).float() / 8192
    assert freq[2:].sum() == 0
    assert abs(freq[0] - 4 / 7) < 0.03


def test_graph_decode_with_top_k_one_matches_greedy():
    """Filtered requests run inside the captured decode graph: temperature 1 with
    top_k = 1 collapses to the argmax (up to bf16 ties at the max)."""
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.models.config import get_config
    from dgi.models.llama import LlamaModel
    from dgi.sched.request import SamplingParams
    mc = get_config("llama-tiny-hd128")
    gm = LlamaModel(mc, "cuda", seed=11)
    e = LLMEngine(EngineConfig(model="llama-tiny-hd128", device="cuda", num_blocks=256, max_num_seqs=8,
                               max_model_len=512, max_num_batched_tokens=256, use_graphs=True),
                  model_cfg=mc, model=gm)
    prompts = [[1] + list(range(5, 5 + n)) for n in (6, 33, 90, 12)]
    greedy = [r.output for r in e.generate(prompts, SamplingParams(max_tokens=10, temperature=0.0, ignore_eos=True))]
    topk1 = [r.output for r in e.generate(prompts, SamplingParams(max_tokens=10, temperature=1.0, top_k=1,
                                                                  top_p=1.0, ignore_eos=True))]
    assert sum(a == b for a, b in zip(greedy, topk1)) >= 3, (greedy, topk1)
    assert e.runner.graphs is not None and e.runner.graphs.captured


@pytest.mark.parametrize("pro,epi", [(0, 0), (1, 0), (2, 0), (2, 1), (1, 2), (2, 2)])
@pytest.mark.parametrize("M", [1, 5, 16])
def test_fused_skinny_matches_reference(pro, epi, M):
    """Fused decode GEMM (RMSNorm prologue, SwiGLU / RoPE+KV epilogue) vs the
    unfused reference ops in fp32 on the same bf16 inputs."""
    _fused_skinny_case(pro, epi, M, None)


@pytest.mark.parametrize("pro,epi", [(0, 0), (2, 0), (2, 1), (1, 2), (2, 2)])
def test_fused_skinny_every_launch_config(pro, epi):
    """Every fused_decode.hip launch config (waves, K-steps per group, one- or
    two-tile workgroups, load ring depth, persistent one-ring workgroups) against
    the reference, at M = 1 and 3."""
    for cfg in range(27):
        for M in (1, 3):
            _fused_skinny_case(pro, epi, M, cfg)


@pytest.mark.parametrize("pro,epi,R", [(2, 1, 2 * 14336), (2, 0, 8192), (0, 0, 8224), (2, 2, None)])
def test_fused_skinny_persistent_multi_tile(pro, epi, R):
    """Persistent configs (whole pair tiles: 12-16; quarter pairs: 22-26) at sizes where
    each workgroup streams several tiles through one ring (8B gate_up: 7 tiles per workgroup; 8192 rows: 2; 8224: 3 with a 1-tile
    last workgroup; qkv: 2), including the tile-parity double-buffered reduce."""
    for cfg in (12, 13, 14, 15, 16, 22, 23, 24, 25, 26):
        for M in (1, 4):
            _fused_skinny_case(pro, epi, M, cfg, R)


@pytest.mark.parametrize("pro,epi,R", [(2, 2, None), (0, 0, 2080), (2, 1, 2 * 1040)])
def test_fused_skinny_split_k(pro, epi, R):
    """Split-K configs (two workgroups per pair tile, last arriver reduces): against the
    reference, bit-identical on a repeat (the tile counters reset themselves, the parts are
    summed in part order), on XCD-paired grids (qkv: 384 tiles) and on grids that are not a
    multiple of 16 workgroups (2080 rows, 1040 gate rows: 130 tiles each)."""
    for cfg in (17, 18, 19, 20, 21):
        for M in (1, 4):
            y1 = _fused_skinny_case(pro, epi, M, cfg, R)
            y2 = _fused_skinny_case(pro, epi, M, cfg, R)
            assert torch.equal(y1, y2), cfg


def _fused_skinny_case(pro, epi, M, cfg, R=None):
    torch.manual_seed(M * 10 + pro * 3 + epi)
    K = 4096
    nh, nkv, bs, nb = 32, 8, 16, 64
    if epi == 2:
        R = (nh + 2 * nkv) * 128
    elif R is not None:
        pass
    elif epi == 1:
        R = 2 * 1024
    else:
        R = 2048
    x = (torch.randn(M, K, device=DEV) * 0.5).bfloat16()
    res = (torch.randn(M, K, device=DEV)).bfloat16() if pro == 2 else None
    gamma = (1 + 0.1 * torch.randn(K, device=DEV)).bfloat16() if pro else None
    w = (torch.randn(R, K, device=DEV) * 0.02).bfloat16()
    bias = (torch.randn(R, device=DEV) * 0.1).bfloat16() if epi != 1 else None
    N = R // 2 if epi == 1 else R
    pos = torch.randint(0, 1000, (M,), device=DEV, dtype=torch.int32)
    inv = 1.0 / (10000 ** (torch.arange(0, 64, device=DEV).float() / 64))
    ang = torch.arange(2048, device=DEV).float()[:, None] * inv[None]
    cos_sin = torch.cat([ang.cos(), ang.sin()], dim=1).contiguous()
    slots = torch.randperm(nb * bs, device=DEV)[:M].int()
    if M > 2:
        slots[1] = -1                      # padding row: no cache write
    kc = torch.zeros(nb, nkv, bs, 128, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    kc_r, vc_r = kc.clone(), vc.clone()
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    y_r = torch.empty_like(y)
    ro = torch.empty_like(x) if pro == 2 else None
    ro_r = torch.empty_like(x) if pro == 2 else None
    ops.fused_skinny(y, x, res, ro, gamma, 1e-5, w, bias, pro, epi, pos, cos_sin, slots, kc, vc, nh, nkv, cfg=cfg)
    ops.fused_skinny_ref(y_r, x, res, ro_r, gamma, 1e-5, w, bias, pro, epi, pos, cos_sin, slots, kc_r, vc_r,
                         nh, nkv)
    torch.cuda.synchronize()
    if pro == 2:
        assert torch.equal(ro, ro_r)
    scale = float(y_r.float().abs().max()) + 1e-3
    assert float((y.float() - y_r.float()).abs().max()) <= 0.02 * scale, (cfg, float((y.float() - y_r.float()).abs().max()))
    if epi == 2:
        for a_, b_ in ((kc, kc_r), (vc, vc_r)):
            s2 = float(b_.float().abs().max()) + 1e-3
            assert float((a_.float() - b_.float()).abs().max()) <= 0.02 * s2
        if M > 2:
            assert int((kc.view(-1, 128).abs().sum(1) > 0).sum()) == (M - 1) * nkv
    return y


def test_fused_decode_model_matches_unfused():
    """Engine decode with the fused layer path vs the unfused kernels (same GPU weights)."""
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.models.config import get_config
    from dgi.models.llama import LlamaModel
    from dgi.sched.request import SamplingParams
    mc = get_config("llama-tiny-hd128")
    src = LlamaModel(mc, "cpu", seed=4)
    prompts = [[1] + list(range(3, 3 + n)) for n in (5, 40, 130, 7)]
    sp = SamplingParams(max_tokens=16, temperature=0.0, ignore_eos=True)
    outs = []
    old = ops.FUSED_DECODE
    try:
        for mode in ("0", "1"):
            ops.FUSED_DECODE = mode
            gm = LlamaModel(mc, "cuda", init="empty").copy_from(src)
            e = LLMEngine(EngineConfig(model="llama-tiny-hd128", device="cuda", num_blocks=256, max_num_seqs=8,
                                       max_model_len=512, max_num_batched_tokens=256, use_graphs=True),
                          model_cfg=mc, model=gm)
            outs.append([r.output for r in e.generate(prompts, sp)])
    finally:
        ops.FUSED_DECODE = old
    # both paths pick, at every step, an argmax of the fp32 model's logits (up to bf16 tolerance)
    for o in outs:
        assert _teacher_forced_ok("llama-tiny-hd128", src, prompts, o) == 64


def test_mall_prefetch_reads_only():
    """The MALL warm-up kernel reads the listed rows and writes nothing (sink stays zero)."""
    ops.load_native(required=True)
    w = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    ref = w.clone()
    rows = torch.tensor([0, 17, 4095, 2048], dtype=torch.int32, device="cuda")
    for kw in ({}, {"nrows": 100}, {"rows": rows}, {"blocks": 7}):
        ops.mall_prefetch(w, **kw)
    torch.cuda.synchronize()
    assert torch.equal(w, ref)
    assert int(ops._PREFETCH_SINKS[w.device].abs().sum()) == 0


@pytest.mark.parametrize("sampled", [False, True])
def test_decode_lookahead_matches_plain_decode(sampled, monkeypatch):
    """Decode lookahead (step N+1 launched before step N's tokens are back) gives the same
    tokens as plain graph decoding, with length stops at different steps, an EOS stop that
    lands while the next step is already in flight, and seeded sampling."""
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.models.config import get_config
    from dgi.models.llama import LlamaModel
    from dgi.sched.request import SamplingParams
    mc = get_config("llama-tiny-hd128")
    src = LlamaModel(mc, "cuda", seed=7)
    prompts = [[1] + list(range(3, 3 + n)) for n in (5, 40, 130, 7)]

    def sp(i, eos_ok):
        return SamplingParams(max_tokens=9 + 4 * i, temperature=0.8 if sampled else 0.0, top_k=20 if sampled else 0,
                              seed=100 + i, ignore_eos=not eos_ok)

    def run(lookahead, eos=None):
        cfg = EngineConfig(model="llama-tiny-hd128", device="cuda", num_blocks=256, max_num_seqs=8, max_model_len=512,
                           max_num_batched_tokens=512, use_graphs=True, decode_lookahead=lookahead)
        e = LLMEngine(cfg, model_cfg=get_config("llama-tiny-hd128"), model=src)
        if eos is not None:
            e.model_cfg.eos_token_id = eos
        reqs = [e.add_request(p, sp(i, eos is not None)) for i, p in enumerate(prompts)]
        while e.has_unfinished():
            e.step()
        return [r.output for r in reqs], [r.finish_reason for r in reqs]

    plain, _ = run(False)
    la, _ = run(True)
    assert la == plain
    eos = plain[2][5]                       # the third prompt's 6th token ends it (and maybe others)
    p2, f2 = run(False, eos)
    l2, g2 = run(True, eos)
    assert l2 == p2 and g2 == f2 and "stop" in f2


@pytest.mark.parametrize("K,N", [(4096, 4096), (1024, 8192), (8192, 8192)])
def test_decode_proj_matches_linear_without_bias(K, N):
    """decode_proj at M = 1 (the persistent fused GEMV, config 16, no prologue / epilogue / bias)
    vs ops.linear and the fp32 reference, on the 8B o-proj, a TP-sharded o-proj and the 70B o-proj;
    a non-contiguous weight falls back to ops.linear."""
    torch.manual_seed(K + N)
    x = (torch.randn(1, K, device=DEV) * 0.5).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    y = ops.decode_proj(x, w)
    ref = x.float() @ w.float().t()
    lin = ops.linear(x, w)
    torch.cuda.synchronize()
    scale = float(ref.abs().max()) + 1e-3
    assert float((y.float() - ref).abs().max()) <= 0.02 * scale
    assert float((y.float() - lin.float()).abs().max()) <= 0.02 * scale
    wt = torch.empty(K, N, device=DEV, dtype=torch.bfloat16).t()      # [N, K] view, not contiguous
    wt.copy_(w)
    y2 = ops.decode_proj(x, wt)
    assert float((y2.float() - ref).abs().max()) <= 0.02 * scale


def test_decode_lookahead_admission_abort_and_page_exhaustion():
    """A lookahead chain broken by a request admitted mid-chain (add_request and
    import_prefilled), an abort while a launch is in flight, and a pool too small for the
    lookahead page growth: every output equals plain (non-lookahead) decoding, nothing
    stays in flight once the work is done, and every page returns to the pool."""
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.models.config import get_config
    from dgi.models.llama import LlamaModel
    from dgi.sched.request import SamplingParams
    mc = get_config("llama-tiny-hd128")
    src = LlamaModel(mc, "cuda", seed=9)
    prompts = [[1] + list(range(3, 3 + n)) for n in (5, 40, 17, 7)]
    sp = SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True)

    def run(lookahead, num_blocks=256):
        cfg = EngineConfig(model="llama-tiny-hd128", device="cuda", num_blocks=num_blocks, max_num_seqs=8,
                           max_model_len=512, max_num_batched_tokens=512, use_graphs=True, decode_lookahead=lookahead,
                           enable_prefix_caching=False)
        e = LLMEngine(cfg, model_cfg=get_config("llama-tiny-hd128"), model=src)
        free0 = e.pool.num_free
        reqs = [e.add_request(p, sp) for p in prompts[:2]]
        for _ in range(6):
            e.step()
        reqs.append(e.add_request(prompts[2], sp))          # admitted while a launch may be in flight
        for _ in range(4):
            e.step()
        victim = reqs[0]
        e.abort(victim.rid)                                  # aborted with a step in flight
        for _ in range(3):
            e.step()
        # a sequence prefilled elsewhere joins the running set mid-chain
        donor = LLMEngine(EngineConfig(model="llama-tiny-hd128", device="cuda", num_blocks=64, max_num_seqs=2,
                                       max_model_len=512, max_num_batched_tokens=512, use_graphs=False,
                                       enable_prefix_caching=False), model_cfg=get_config("llama-tiny-hd128"),
                          model=src)
        got = []
        donor.first_token_hook = lambda r: got.append(donor.export_request_kv(r))   # before its pages are freed
        d = donor.add_request(prompts[3], SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))
        donor.step()
        kv = got[0]
        reqs.append(e.import_prefilled(prompts[3], d.output[0], kv, sp))
        while e.has_unfinished():
            e.step()
        assert e._la is None
        assert e.pool.num_free == free0, (e.pool.num_free, free0)
        return [r.output for r in reqs[1:]]

    plain = run(False)
    assert run(True) == plain
    # a pool with barely enough pages: lookahead growth runs out and falls back to plain steps
    need = sum((len(p) + 24 + 15) // 16 for p in prompts) + 1
    assert run(True, num_blocks=need) == run(False, num_blocks=need) == plain


@pytest.mark.parametrize("rows", [768, 1024])
def test_two_batch_overlap_decode_step_matches_one_batch(rows, monkeypatch):
    """Two-batch overlap (CU-masked GEMM and attention streams, dgi.models.llama
    _forward_layers_tbo) on a pure-decode step gives the logits of the one-batch step
    (same KV, same rows) up to GEMM blocking, and both are within bf16 tolerance of the
    fp32 CPU model on a sample of rows."""
    import random
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.models import llama
    from dgi.models.config import get_config
    from dgi.models.llama import LlamaModel
    from dgi.parallel.probe import _adopt
    mc = get_config("llama-tiny-hd128")
    src = LlamaModel(mc, "cpu", seed=21)
    gm = LlamaModel(mc, "cuda", init="empty").copy_from(src)
    eng = LLMEngine(EngineConfig(model="llama-tiny-hd128", device="cuda", num_blocks=rows * 8 + 16,
                                 max_num_seqs=rows, max_model_len=512, max_num_batched_tokens=2048, use_graphs=False,
                                 enable_prefix_caching=False), model_cfg=mc, model=gm)
    torch.manual_seed(5)
    eng.pool.kv.normal_(0, 1)
    _adopt(eng, rows, 90, random.Random(1))
    sb = eng.scheduler.schedule()
    assert len(sb.decode) == rows and not sb.prefill
    flat, hdr, _ = eng.runner.build_host(sb)
    ids, meta, _ = eng.runner.meta_from_device(eng.runner.to_device(flat), hdr)
    monkeypatch.setattr(llama, "TBO", False)
    ref = eng.model.forward(meta, input_ids=ids).float()
    monkeypatch.setattr(llama, "TBO", True)
    assert eng.model._tbo_ok(torch.empty(rows, 8, device="cuda", dtype=torch.bfloat16), meta, None) == \
        llama.tbo_split(rows)
    got = eng.model.forward(meta, input_ids=ids).float()
    torch.cuda.synchronize()
    scale = float(ref.abs().max())
    assert float((got - ref).abs().max()) <= 0.02 * scale
    # a sample of rows against the fp32 CPU model over the same KV pages
    pick = [0, 1, rows // 2, rows - 1]
    kv_cpu = eng.pool.kv.float().cpu()
    for r in pick:
        req = sb.decode[r]
        ctx = req.num_computed + 1
        blocks = req.blocks[: (ctx + 15) // 16]
        lg = _cpu_decode_row(src, kv_cpu, blocks, ctx, int(ids[r]))
        assert float((got[r].cpu() - lg).abs().max()) <= 0.03 * float(lg.abs().max()) + 0.03


def _cpu_decode_row(model, kv, blocks, ctx, tok):
    """fp32 CPU logits of one decode row at position ctx - 1 over paged KV ``kv`` (pages
    ``blocks``; the row's own K/V is computed here, the rest read from the pages)."""
    import math as _m
    c = model.cfg
    x = model.embed[tok].float()[None]
    pos = torch.tensor([ctx - 1])
    cs = ops.rope_cos_sin(c.rope_dim, c.max_position, c.rope_theta, c.rope_scaling)
    res = None
    for i, L in enumerate(model.layers):
        if res is None:
            res = x
            h = ops.rmsnorm_ref(x, L.in_norm.float(), c.rms_eps)
        else:
            res = x + res
            h = ops.rmsnorm_ref(res, L.in_norm.float(), c.rms_eps)
        qkv = h @ L.qkv.float().t()
        nh, nkv, hd = c.num_heads, c.num_kv_heads, c.head_dim
        q = qkv[:, : nh * hd].view(1, nh, hd)
        k = qkv[:, nh * hd:(nh + nkv) * hd].view(1, nkv, hd)
        v = qkv[:, (nh + nkv) * hd:].view(1, nkv, hd)
        q = ops._rope(q, cs[pos], 0)
        k = ops._rope(k, cs[pos], 0)
        K = kv[i, 0][blocks].permute(0, 2, 1, 3).reshape(-1, nkv, hd)[:ctx].clone()
        V = kv[i, 1][blocks].permute(0, 2, 1, 3).reshape(-1, nkv, hd)[:ctx].clone()
        K[ctx - 1], V[ctx - 1] = k[0], v[0]
        G = nh // nkv
        s = torch.einsum("hgd,thd->hgt", q.view(nkv, G, hd), K) / _m.sqrt(hd)
        o = torch.einsum("hgt,thd->hgd", torch.softmax(s, -1), V).reshape(1, nh * hd)
        x = o @ L.o.float().t()
        res = x + res
        h = ops.rmsnorm_ref(res, L.post_norm.float(), c.rms_eps)
        gu = h @ L.gate_up.float().t()
        I = gu.shape[1] // 2
        x = (torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]) @ L.down.float().t()
    h = ops.rmsnorm_ref(x + res, model.norm.float(), c.rms_eps)
    return (h @ model.lm_head.float().t())[0]


@pytest.mark.parametrize("sampled,eos", [(False, False), (True, False), (False, True)])
def test_mixed_step_lookahead_matches_plain_steps(sampled, eos):
    """Mixed-step lookahead (step N+1 scheduled and launched before step N's tokens are back,
    its input tokens read on the device): staggered arrivals, chunked prefill across steps,
    length stops at different steps, seeded sampling and an EOS stop that lands while the
    next step is in flight give exactly the outputs of plain steps; the chain really ran."""
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.models.config import get_config
    from dgi.models.llama import LlamaModel
    from dgi.sched.request import SamplingParams
    mc = get_config("llama-tiny-hd128")
    src = LlamaModel(mc, "cuda", seed=13)
    g = torch.Generator().manual_seed(2)
    prompts = [torch.randint(5, 900, (n,), generator=g).tolist() for n in (40, 75, 9, 130, 22, 61)]

    def sp(i, eos_ok):
        return SamplingParams(max_tokens=7 + 3 * i, temperature=0.8 if sampled else 0.0, top_k=20 if sampled else 0,
                              seed=50 + i, ignore_eos=not eos_ok)

    def run(mixed, eos_tok=None):
        cfg = EngineConfig(model="llama-tiny-hd128", device="cuda", num_blocks=256, max_num_seqs=8, max_model_len=512,
                           max_num_batched_tokens=64, use_graphs=True, enable_prefix_caching=False)
        e = LLMEngine(cfg, model_cfg=get_config("llama-tiny-hd128"), model=src)
        e.mixed_lookahead = mixed
        if eos_tok is not None:
            e.model_cfg.eos_token_id = eos_tok
        reqs = []
        for i, p in enumerate(prompts):
            reqs.append(e.add_request(p, sp(i, eos_tok is not None)))
            e.step()
        while e.has_unfinished():
            e.step()
        assert e._mx is None and e.pool.num_free == 255
        return [r.output for r in reqs], [r.finish_reason for r in reqs], e.mixed_chained

    plain, pf, n0 = run(False)
    la, lf, n1 = run(True)
    assert la == plain and lf == pf and n0 == 0 and n1 > 0
    if eos:
        tok = plain[3][4]
        p2, f2, _ = run(False, tok)
        l2, g2, _ = run(True, tok)
        assert l2 == p2 and g2 == f2 and "stop" in f2


@pytest.mark.parametrize("graphs", [False, True])
@pytest.mark.parametrize("name", ["llama-tiny-hd128", "llama-tiny-tp"])
def test_fused_norm_layers_match_fp32(monkeypatch, graphs, name):
    """The fused-norm layers (gains folded into qkv / gate_up, residual + row statistics in the
    o / down epilogues, rstd in the qkv / gate_up epilogues) on every step — prefill chunks,
    mixed steps and captured decode graphs: each generated token is an argmax of the fp32 CPU
    model (teacher forced), and the path really ran."""
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.models import llama
    from dgi.models.config import get_config
    from dgi.models.llama import LlamaModel
    from dgi.sched.request import SamplingParams
    monkeypatch.setattr(llama, "NORM_FOLD", "force")
    monkeypatch.setattr(llama, "NORM_FOLD_MIN_ROWS", 1)
    mc = get_config(name)             # tiny-tp: 2 kv heads, so the qkv GEMM also takes the RoPE + KV epilogue
    cpu_model = LlamaModel(mc, "cpu", seed=5)
    prompts = [[1] + list(range(3, 3 + n)) for n in (5, 40, 200, 7)]     # (the fp32 oracle prefills in one chunk)
    gm = LlamaModel(mc, "cuda", init="empty").copy_from(cpu_model)
    calls = [0]
    orig = gm._forward_layers_folded

    def spy(*a, **k):
        calls[0] += 1
        return orig(*a, **k)
    gm._forward_layers_folded = spy
    e = LLMEngine(EngineConfig(model=name, device="cuda", num_blocks=256, max_num_seqs=8,
                               max_model_len=512, max_num_batched_tokens=256, use_graphs=graphs),
                  model_cfg=mc, model=gm)
    assert gm.norms_folded
    outs = [r.output for r in e.generate(prompts, SamplingParams(max_tokens=10, temperature=0.0, ignore_eos=True))]
    torch.cuda.synchronize()
    assert calls[0] > 0
    assert _teacher_forced_ok(name, cpu_model, prompts, outs) == 40
