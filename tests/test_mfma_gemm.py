"""LDS-tiled MFMA GEMM (dgi/csrc/mfma_gemm.hip) against a plain fp32 PyTorch
reference: plain store and fused SwiGLU epilogues, M tails (rows clamped on
load, skipped on store), several tile counts so the XCD-aware block map covers
grids that are and are not multiples of 8."""
import pytest
import torch

from dgi import ops


def _rand(*shape, device, scale=1.0, seed=0):
    g = torch.Generator(device=device).manual_seed(seed)
    return ((torch.rand(*shape, generator=g, device=device) * 2 - 1) * scale).to(torch.bfloat16)


def test_split_timeout_counter_is_zero_without_a_gpu_cpu():
    assert ops.gemm_split_timeouts() == 0


def test_reference_swiglu_matches_silu_mul_cpu():
    x = _rand(7, 64, device="cpu")
    w = _rand(512, 64, device="cpu", seed=1)
    a = ops.mfma_gemm(x, w, 1)                      # CPU: reference path
    b = ops.silu_mul_ref((x.float() @ w.float().t()).to(torch.bfloat16))
    assert a.shape == (7, 256)
    assert torch.allclose(a.float(), b.float(), atol=0.1, rtol=0.05)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(1, 256, 64), (100, 512, 256), (256, 256, 128), (300, 768, 512),
                                   (1000, 1024, 1024), (2048, 2560, 4096), (513, 256, 8192)])
@pytest.mark.parametrize("epi", [0, 1])
@pytest.mark.parametrize("sched", [0, 1, 2, 3])
def test_mfma_gemm_matches_fp32(M, N, K, epi, sched):
    ops.load_native(required=True)
    x = _rand(M, K, device="cuda", seed=M + K)
    w = _rand(N, K, device="cuda", scale=0.05, seed=N)
    ref = ops.mfma_gemm_ref(x, w, epi).float()
    got = ops.mfma_gemm(x, w, epi, sched=sched)
    torch.cuda.synchronize()
    assert got.shape == ref.shape
    err = (got.float() - ref).abs()
    tol = 2e-2 * ref.abs().max().item() + 1e-3
    assert err.max().item() <= tol, (err.max().item(), tol)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(1, 256, 64), (100, 512, 256), (128, 256, 128), (300, 768, 512),
                                   (512, 1280, 1024), (777, 512, 8192), (512, 10240, 512)])
def test_mfma_gemm_half_tile_matches_fp32(M, N, K):
    """Schedule 4: the 128 x 128 half-tile kernel (plain GEMM) against fp32, M tails included."""
    ops.load_native(required=True)
    x = _rand(M, K, device="cuda", seed=M + K)
    w = _rand(N, K, device="cuda", scale=0.05, seed=N)
    ref = ops.mfma_gemm_ref(x, w, 0).float()
    got = ops.mfma_gemm(x, w, 0, sched=4)
    torch.cuda.synchronize()
    err = (got.float() - ref).abs()
    tol = 2e-2 * ref.abs().max().item() + 1e-3
    assert err.max().item() <= tol, (err.max().item(), tol)


@pytest.mark.gpu
@pytest.mark.parametrize("sched", [0, 1, 2, 3, 4])
def test_mfma_gemm_strided_rows_and_asymmetric_operands(sched):
    """A = row slice of a wider buffer (ldx > K) and an asymmetric W: catches
    row/column swaps in the C write and ldx handling."""
    ops.load_native(required=True)
    K = 256
    buf = _rand(384, K + 64, device="cuda", seed=5)
    x = buf[:, :K]
    w = (torch.arange(512 * K, device="cuda", dtype=torch.float32).reshape(512, K) % 7 - 3).to(torch.bfloat16)
    got = ops.mfma_gemm(x, w, 0, sched=sched)
    ref = ops.mfma_gemm_ref(x, w, 0).float()
    assert (got.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(2048, 1024, 256), (1920, 2560, 1024), (4096, 512, 8192), (2048, 16384, 512),
                                   (2000, 16384, 512)])
@pytest.mark.parametrize("epi", [0, 1])
@pytest.mark.parametrize("phases", [4, 2])
def test_mfma_gemm_pingpong_bitwise_stable(M, N, K, epi, phases):
    """Race screen for the ping-pong schedule (sched 3): it accumulates in the same
    order as sched 1, so every one of repeated launches must match sched 1 bit for
    bit -- a slab read before its load landed (or overwritten before every wave
    read it) shows up as a mismatch on some launch.  N = 16384 at M = 2048 is two
    whole waves of tiles: the persistent launch whose next tile's staging loads are
    issued under the current tile's epilogue (M = 2000: the last row tile has a tail
    and is not overlapped)."""
    ops.load_native(required=True)
    x = _rand(M, K, device="cuda", seed=M)
    w = _rand(N, K, device="cuda", scale=0.05, seed=K)
    ref = ops.mfma_gemm(x, w, epi, sched=1)
    for _ in range(12):
        got = ops.mfma_gemm(x, w, epi, sched=3, streamk=1, phases=phases)
        assert torch.equal(got, ref)
    assert torch.equal(ops.mfma_gemm(x, w, epi, sched=3, streamk=1, phases=phases, overlap=False), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(2048, 2560, 512), (1920, 10240, 8192), (1000, 768, 2048), (2432, 8192, 1024),
                                   (300, 57344 // 8, 4096), (2048, 19200, 1024), (512, 10240, 8192),
                                   (512, 57344, 1024), (200, 57344, 1024), (1000, 48896, 1024)])
@pytest.mark.parametrize("epi", [0, 1])
@pytest.mark.parametrize("streamk", [0, 2])
@pytest.mark.parametrize("phases", [4, 2])
def test_mfma_gemm_splitk_matches_fp32_and_is_deterministic(M, N, K, epi, streamk, phases):
    """Hybrid split-K of the last partial wave (persistent launch, 2-4 K pieces per
    remainder tile reduced by the last arriving block through fp32 slabs; uneven
    piece lengths at K = 512; N = 19200 at M = 2048: a split piece, then two whole
    tiles whose second loads under the first's epilogue; N = 57344 at M = 512 / 200 and
    N = 48896 at M = 1000: a last wave more than half full, no split): matches the fp32
    reference, and repeated launches agree bit for bit (slabs are summed in piece order
    whichever piece arrives last)."""
    ops.load_native(required=True)
    x = _rand(M, K, device="cuda", seed=M + 1)
    w = _rand(N, K, device="cuda", scale=0.05, seed=N + 1)
    ref = ops.mfma_gemm_ref(x, w, epi).float()
    got = ops.mfma_gemm(x, w, epi, sched=3, streamk=streamk, phases=phases)
    torch.cuda.synchronize()
    err = (got.float() - ref).abs()
    tol = 2e-2 * ref.abs().max().item() + 1e-3
    assert err.max().item() <= tol, (err.max().item(), tol)
    for _ in range(6):
        assert torch.equal(ops.mfma_gemm(x, w, epi, sched=3, streamk=streamk, phases=phases), got)
    assert ops.gemm_split_timeouts(reset=True) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("cus,N", [(160, 10240), (192, 8192), (128, 4096)])
def test_mfma_gemm_splitk_on_a_cu_limited_grid(cus, N):
    """Split-K on a grid sized for fewer CUs (``set_gemm_cus``, what a CU-masked two-batch-overlap
    stream uses): 2 / 3 / 4 pieces per tile, the "written" counters at [P + t] of a smaller P, the
    last piece's registers folded in piece order.  Matches fp32, bit-identical on repeats, and the
    counters are back to zero for the next full-grid launch."""
    ops.load_native(required=True)
    x = _rand(512, 2048, device="cuda", seed=11)
    w = _rand(N, 2048, device="cuda", scale=0.05, seed=12)
    ref = ops.mfma_gemm_ref(x, w, 0).float()
    ops.set_gemm_cus(cus)
    try:
        got = ops.mfma_gemm(x, w, 0, sched=3)
        again = [ops.mfma_gemm(x, w, 0, sched=3) for _ in range(4)]
    finally:
        ops.set_gemm_cus(0)
    full = ops.mfma_gemm(x, w, 0, sched=3)
    torch.cuda.synchronize()
    tol = 2e-2 * ref.abs().max().item() + 1e-3
    assert (got.float() - ref).abs().max().item() <= tol
    assert all(torch.equal(a, got) for a in again)
    assert (full.float() - ref).abs().max().item() <= tol
    assert ops.gemm_split_timeouts(reset=True) == 0        # no last piece's wait ran out


# ---------------------------------------------------------------------------
# fused RMSNorm epilogues (EPI 2 residual + row statistics, 3 / 4 rstd-scaled plain / SwiGLU)

def _norm_case(M, N, K, kind, device, phases=0):
    x = _rand(M, K, device=device, seed=M + K)
    w = _rand(N, K, device=device, scale=0.05, seed=N)
    if kind == ops.NORM_RES:
        res = _rand(M, N, device=device, seed=7)
        ss = torch.full((M, N // 256), -1.0, device=device)
        want_res = res.clone()
        want_ss = torch.empty_like(ss)
        ops.mfma_gemm_norm_ref(x, w, kind, want_ss, 1e-5, want_res)
        ops.mfma_gemm_norm(x, w, kind, ss, 1e-5, out=res, phases=phases)
        return (res, ss), (want_res, want_ss)
    ss = (torch.rand(M, 8, generator=torch.Generator().manual_seed(M + N)) * K * 0.1).to(device)
    want = ops.mfma_gemm_norm_ref(x, w, kind, ss, 1e-5)
    got = ops.mfma_gemm_norm(x, w, kind, ss, 1e-5, phases=phases)
    return (got,), (want,)


def test_norm_fold_reference_equals_rmsnorm_then_gemm_cpu():
    """Gain folded into the weights + rstd in the epilogue == rmsnorm(x) * gamma @ W^T."""
    x = _rand(9, 512, device="cpu", seed=3)
    w = _rand(768, 512, device="cpu", scale=0.05, seed=4)
    gamma = (1 + 0.1 * torch.randn(512)).to(torch.bfloat16)
    want = ops.rmsnorm_ref(x, gamma, 1e-5).float() @ w.float().t()
    ss = torch.zeros(9, 2)
    ops.row_sumsq(x, ss)
    wf = (w.float() * gamma.float()[None]).to(torch.bfloat16)
    got = ops.mfma_gemm_norm_ref(x, wf, ops.NORM_PLAIN, ss, 1e-5)
    assert torch.allclose(got.float(), want, atol=2e-2 * want.abs().max().item())
    # the residual kind's statistics feed the next norm exactly like row_sumsq of its output
    res = _rand(9, 768, device="cpu", seed=5)
    ss2 = torch.zeros(9, 3)
    ops.mfma_gemm_norm_ref(x, w, ops.NORM_RES, ss2, 1e-5, res)
    ref = torch.zeros(9, 3)
    ops.row_sumsq(res, ref)
    assert torch.allclose(ss2.sum(-1), ref.sum(-1), rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(1, 256, 256), (100, 512, 256), (300, 768, 512), (512, 2560, 1024),
                                   (513, 1024, 8192), (2048, 2560, 4096), (512, 57344, 1024)])
@pytest.mark.parametrize("kind", [2, 3, 4])
@pytest.mark.parametrize("phases", [2, 4])
def test_mfma_gemm_norm_matches_fp32(M, N, K, kind, phases):
    ops.load_native(required=True)
    got, want = _norm_case(M, N, K, kind, "cuda", phases)
    torch.cuda.synchronize()
    for g, w in zip(got, want):
        err = (g.float() - w.float()).abs()
        tol = 2e-2 * w.float().abs().max().item() + 1e-3
        assert err.max().item() <= tol, (err.max().item(), tol)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,kind", [(1000, 8192, 1024, 2), (512, 57344, 1024, 4)])
def test_mfma_gemm_norm_is_deterministic(M, N, K, kind):
    """The row statistics are reduced in a fixed order (no atomics), split-K slabs in piece order:
    repeated runs are bit-identical."""
    ops.load_native(required=True)
    outs = []
    for _ in range(4):
        got, _w = _norm_case(M, N, K, kind, "cuda")
        outs.append([t.clone() for t in got])
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert all(torch.equal(a, b) for a, b in zip(outs[0], o))


def _rope_case(M, nh, nkv, K, device, phases=0, seed=0):
    g = torch.Generator().manual_seed(seed)
    N = (nh + 2 * nkv) * 128
    x = _rand(M, K, device=device, seed=M + K)
    w = _rand(N, K, device=device, scale=0.05, seed=N)
    ss = (torch.rand(M, 8, generator=g) * K * 0.1).to(device)
    cs = ops.rope_cos_sin(128, 4096, 500000.0, device=device)
    pos = torch.randint(0, 4000, (M,), generator=g, dtype=torch.int32).to(device)
    nb, bs = (M + 15) // 16 + 4, 16
    slots = torch.randperm(nb * bs, generator=g)[:M].to(torch.int32)
    slots[::7] = -1                                   # rows with no cache slot (graph padding)
    slots = slots.to(device)
    caches = []
    for _ in range(2):
        kc = torch.zeros(nb, nkv, bs, 128, dtype=torch.bfloat16, device=device)
        vc = torch.zeros_like(kc)
        caches.append((kc, vc))
    want = ops.mfma_gemm_norm_rope_ref(x, w, ss, 1e-5, pos, cs, slots, *caches[0], nh, nkv)
    got = ops.mfma_gemm_norm_rope(x, w, ss, 1e-5, pos, cs, slots, *caches[1], nh, nkv, phases=phases)
    return (got[:, : nh * 128], caches[1][0], caches[1][1]), (want[:, : nh * 128], caches[0][0], caches[0][1])


def test_norm_rope_reference_composes_norm_then_rope_cpu():
    got, want = _rope_case(37, 4, 2, 256, "cpu")
    for g, w in zip(got, want):
        assert torch.equal(g, w)


@pytest.mark.gpu
@pytest.mark.parametrize("M,nh,nkv,K", [(1, 2, 2, 256), (100, 4, 2, 512), (300, 8, 2, 1024), (513, 64, 8, 1024),
                                        (1024, 16, 2, 2048)])
@pytest.mark.parametrize("phases", [2, 4])
def test_mfma_gemm_norm_rope_matches_fp32(M, nh, nkv, K, phases):
    """EPI 5: rotated q columns, rotated k and plain v in the paged caches (rows with slot -1 write
    nothing) against the fp32 norm-then-rope reference."""
    ops.load_native(required=True)
    got, want = _rope_case(M, nh, nkv, K, "cuda", phases)
    torch.cuda.synchronize()
    for g, w in zip(got, want):
        err = (g.float() - w.float()).abs()
        tol = 2e-2 * w.float().abs().max().item() + 1e-3
        assert err.max().item() <= tol, (err.max().item(), tol)
