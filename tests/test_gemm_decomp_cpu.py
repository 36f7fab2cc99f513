"""CPU model of the ping-pong GEMM's persistent work decomposition (``dgi/csrc/mfma_gemm.hip``,
``drive()`` / ``launch_pp``, hybrid split-K): the same integer formulas, checked for every launch
shape the host can pick.  Every (tile, 128-deep K unit) must be computed exactly once, every tile
cut into pieces must have np pieces numbered 0..np-1 in K order (the last arriving piece folds
them in that order), each piece's fp32 slab must be its own, and the tile's counters must stay
inside the workspace.  A mistake here is a wrong tile or a bounded wait on the GPU, so it is
pinned on the CPU first.  (A column-group stream-K variant was modelled and measured too: no
gain, removed; profiles/r6_splitk/README.md.)"""
import itertools

import pytest


def hybrid_items(P, total, nt2, cap=4):
    """Hybrid split-K (whole-K pieces of the last partial wave, one piece per block; at most
    ``cap`` pieces per tile)."""
    full, rem = divmod(total, P)
    splits = min(cap, P // rem) if rem else 0
    assert splits >= 2
    items = []
    for g in range(P):
        if g < rem * splits:
            j = g // rem
            u0, u1 = j * nt2 // splits, (j + 1) * nt2 // splits
            t = g - j * rem
            items.append(dict(g=g, t=t, u0=u0, u1=u1, piece=True, own=j, np=splits, slab=j * rem + t))
        for k in range(full):
            items.append(dict(g=g, t=rem + k * P + g, u0=0, u1=nt2, piece=False))
    return items


def check(items, P, total, nt2):
    cover = {}
    for it in items:
        for u in range(it["u0"], it["u1"]):
            key = (it["t"], u)
            assert key not in cover, ("unit computed twice", key)
            cover[key] = it
        assert it["u1"] > it["u0"]
    assert len(cover) == total * nt2, "some (tile, unit) never computed"
    pieces = {}
    for it in items:
        if it["piece"]:
            pieces.setdefault(it["t"], []).append(it)
    slabs = set()
    for t, ps in pieces.items():
        assert t < P, "counter index outside the workspace"
        ps.sort(key=lambda x: x["u0"])
        np_ = ps[0]["np"]
        assert len(ps) == np_ and 2 <= np_ <= 4
        assert [p["own"] for p in ps] == list(range(np_)), "pieces not numbered in K order"
        for p in ps:
            assert 0 <= p["slab"] < 2 * P
            assert p["slab"] not in slabs, "two pieces share a slab"
            slabs.add(p["slab"])
    return pieces


@pytest.mark.parametrize("P", [256, 248, 64])
@pytest.mark.parametrize("cap", [4])
def test_hybrid_split_decomposition(P, cap):
    for total, nt2 in itertools.product(range(1, 2 * P + 3, 3), (4, 5, 64)):
        full, rem = divmod(total, P)
        if rem and min(cap, P // rem) >= 2 and nt2 >= min(cap, P // rem):
            check(hybrid_items(P, total, nt2, cap), P, total, nt2)
