"""CPU behaviour of dgi.ops: reference implementations (the GPU tests' oracles)
and the dispatch rules that decide which native kernel a GPU call takes."""
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
