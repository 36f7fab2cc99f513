"""CPU model of the ping-pong GEMM's persistent work decomposition (``dgi/csrc/mfma_gemm.hip``,
``drive()`` / ``launch_pp``): the same integer formulas, checked for every launch shape the host
can pick.  Every (tile, 128-deep K unit) must be computed exactly once, every tile cut into pieces
must have np pieces numbered 0..np-1 in K order, each piece's fp32 slab must be its own (two per
block), and the tile's counters must stay inside the workspace.  A mistake here is a wrong tile
or a bounded wait on the GPU, so it is pinned on the CPU first."""
import itertools

import pytest


def hybrid_items(P, total, nt2, cap=4):
    """Hybrid split-K (whole-K pieces of the last partial wave, one piece per block; at most
    ``cap`` pieces per tile, DGI_GEMM_MAX_SPLITS)."""
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


def group_items(P, tiles_m, tiles_n, nt2):
    """Column-group stream-K: groups of G = tiles_m blocks share each column's K range."""
    G = tiles_m
    NG = P // G
    full, rem = divmod(tiles_n, NG)
    R = rem * nt2
    items = []

    def piece_info(t, g):
        c = t // tiles_m
        g0 = ((c * nt2 + 1) * NG - 1) // R
        g1 = ((c + 1) * nt2 * NG - 1) // R
        return g0, g // G - g0, g1 - g0 + 1

    def slab_of(t, g0, jj):
        og = g0 + jj
        c = t // tiles_m
        return (og * G + (t - c * tiles_m)) * 2 + (0 if c == og * R // NG // nt2 else 1)

    for g in range(P):
        gi, mt = divmod(g, G)
        used, k = 0, 0
        while True:
            e = (gi + 1) * R // NG
            u = gi * R // NG + used
            if u < e:
                c = u // nt2
                pe = min(e, (c + 1) * nt2)
                used += pe - u
                g0 = ((c * nt2 + 1) * NG - 1) // R
                g1 = ((c + 1) * nt2 * NG - 1) // R
                t = c * tiles_m + mt
                it = dict(g=g, t=t, u0=u - c * nt2, u1=pe - c * nt2, piece=g1 > g0)
                if it["piece"]:
                    g0_, own, np_ = piece_info(t, g)
                    it.update(own=own, np=np_, slab=slab_of(t, g0_, own),
                              slabs=[slab_of(t, g0_, jj) for jj in range(np_)])
                items.append(it)
                continue
            if k < full:
                items.append(dict(g=g, t=(rem + k * NG + gi) * tiles_m + mt, u0=0, u1=nt2, piece=False))
                k += 1
                continue
            break
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
        assert len(ps) == np_ and 2 <= np_ <= 8
        assert [p["own"] for p in ps] == list(range(np_)), "pieces not numbered in K order"
        for p in ps:
            assert 0 <= p["slab"] < 2 * P
            assert p["slab"] not in slabs, "two pieces share a slab"
            slabs.add(p["slab"])
            if "slabs" in p:      # every piece computes the same slab list for its tile
                assert p["slabs"] == [q["slab"] for q in ps]
    return pieces


@pytest.mark.parametrize("P", [256, 248, 64])
@pytest.mark.parametrize("cap", [4, 8])
def test_hybrid_split_decomposition(P, cap):
    for total, nt2 in itertools.product(range(1, 2 * P + 3, 3), (4, 5, 64)):
        full, rem = divmod(total, P)
        if rem and min(cap, P // rem) >= 2 and nt2 >= min(cap, P // rem):
            check(hybrid_items(P, total, nt2, cap), P, total, nt2)


@pytest.mark.parametrize("P", [256, 64])
def test_column_group_decomposition(P):
    """Launch shapes the host picks for column groups: the last partial wave more than half full
    (no whole-K split fits), tiles_m dividing the blocks of an XCD, fewer than 8 full waves."""
    n = 0
    for tiles_m in (1, 2, 4, 8, 16, 32):
        if (P // 8) % tiles_m:
            continue
        for tiles_n in range(1, 8 * P // tiles_m + 1, 1 if P <= 64 else 5):
            total = tiles_m * tiles_n
            full, rem = divmod(total, P)
            if not rem or min(4, P // rem) >= 2 or full >= 8:
                continue
            for nt2 in (4, 7, 64):
                pieces = check(group_items(P, tiles_m, tiles_n, nt2), P, total, nt2)
                assert all(len(ps) <= 3 for ps in pieces.values())
                n += 1
    assert n > 0


def test_decode_role_gate_up_shape():
    """70B gate_up at 512 rows: 2 x 224 tiles on 256 CUs, 1.75 waves -> every block gets 1.75
    tiles of K units (whole column round + 3/4 of a column)."""
    P, tiles_m, tiles_n, nt2 = 256, 2, 224, 64
    items = group_items(P, tiles_m, tiles_n, nt2)
    check(items, P, tiles_m * tiles_n, nt2)
    work = {}
    for it in items:
        work[it["g"]] = work.get(it["g"], 0) + it["u1"] - it["u0"]
    assert set(work.values()) == {112}      # 1.75 x 64 units on every block
