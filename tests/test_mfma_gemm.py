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
                                   (300, 57344 // 8, 4096), (2048, 19200, 1024)])
@pytest.mark.parametrize("epi", [0, 1])
@pytest.mark.parametrize("streamk", [0, 2])
@pytest.mark.parametrize("phases", [4, 2])
def test_mfma_gemm_splitk_matches_fp32_and_is_deterministic(M, N, K, epi, streamk, phases):
    """Hybrid split-K of the last partial wave (persistent launch, 2-4 K pieces per
    remainder tile reduced by the last arriving block through fp32 slabs; uneven
    piece lengths at K = 512; N = 19200 at M = 2048: a split piece, then two whole
    tiles whose second loads under the first's epilogue): matches the fp32 reference,
    and repeated launches agree bit for bit (slabs are summed in piece order)."""
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
