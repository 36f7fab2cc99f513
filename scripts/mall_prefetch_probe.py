#!/usr/bin/env python3
"""Does warming the MALL during batch-1 decode attention speed up the o-proj behind it?

Llama-3-8B geometry.  All times per iteration inside one captured hipGraph, weights rotated
through a set larger than the 256 MB MALL (cold unless prefetched):

* oproj_cold     : ops.decode_proj (the o-proj's persistent GEMV) on a cold weight;
* prefetch       : ops.mall_prefetch of that weight alone;
* oproj_warm     : prefetch, then the o-proj (serial) minus the prefetch alone;
* attn           : paged decode attention (batch 1, one split, 8 waves);
* attn+oproj     : attention, then the o-proj (what the decode layer does today);
* attn||pf+oproj : the prefetch forked onto a side stream beside the attention, joined
                   before the o-proj (the proposed layer);
* same with the first ``k`` pair tiles of every gate_up workgroup prefetched too (the rows the
  persistent SwiGLU GEMV streams first: 8 gate + 8 up rows per tile, 7 tiles per workgroup on
  256 CUs), and gate_up after the o-proj.
Prints one JSON line per context length."""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from dgi import ops

nh, nkv, hd, bs, H = 32, 8, 128, 16, 4096


def graph_us(fn, reps: int = 20, iters: int = 10) -> float:
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(3):
            fn(i)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(reps):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * iters)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, nargs="+", default=[256, 512, 1024])
    ap.add_argument("--blocks", type=int, nargs="+", default=[128, 256, 512])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ops.load_native(required=True)
    dev, bf = "cuda", torch.bfloat16
    nbuf = 12                                           # 12 x (33.5 + 235) MB >> MALL
    ow = [torch.randn(H, H, device=dev, dtype=bf) * 0.02 for _ in range(nbuf)]
    guw = [torch.randn(2 * 14336, H, device=dev, dtype=bf) * 0.02 for _ in range(nbuf)]
    x = torch.randn(1, H, device=dev, dtype=bf)
    side = torch.cuda.Stream()
    I, tpw = 14336, 7
    gu_rows = {}
    for k in (1, 2):
        g = [b * tpw * 8 + t * 8 + j for b in range(I // 8 // tpw) for t in range(k) for j in range(8)]
        gu_rows[k] = torch.tensor(g + [I + r for r in g], dtype=torch.int32, device=dev)
    rows = []
    base = {}
    base["oproj_cold"] = graph_us(lambda i: ops.decode_proj(x, ow[i % nbuf]))
    for blk in a.blocks:
        base[f"prefetch_b{blk}"] = graph_us(lambda i: ops.mall_prefetch(ow[i % nbuf], blocks=blk))
        both = graph_us(lambda i: (ops.mall_prefetch(ow[i % nbuf], blocks=blk), ops.decode_proj(x, ow[i % nbuf])))
        base[f"oproj_warm_b{blk}"] = both - base[f"prefetch_b{blk}"]
    print(json.dumps({k: round(v, 2) for k, v in base.items()}), flush=True)
    scale = 1 / math.sqrt(hd)
    for C in a.ctx:
        nb_seq = (C + bs - 1) // bs
        kcs = [torch.randn(nb_seq + 1, nkv, bs, hd, device=dev, dtype=bf) for _ in range(4)]
        vcs = [torch.randn_like(k) for k in kcs]
        bt = (torch.arange(nb_seq, device=dev, dtype=torch.int32) + 1).view(1, nb_seq)
        ctx = torch.full((1,), C, device=dev, dtype=torch.int32)
        q = torch.randn(1, (nh + 2 * nkv) * hd, device=dev, dtype=bf)
        out = torch.empty(1, nh * hd, device=dev, dtype=bf)
        act = torch.empty(1, 14336, device=dev, dtype=bf)

        def attn(i):
            ops.paged_decode(q, kcs[i % 4], vcs[i % 4], bt, ctx, nh, nkv, scale, max_splits=1,
                             part_size=1 << 20, out=out)

        def forked(i, blk, gu_rows):
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                ops.mall_prefetch(ow[i % nbuf], blocks=blk)
                if gu_rows is not None:
                    ops.mall_prefetch(guw[i % nbuf], gu_rows, blocks=blk)
            attn(i)
            main.wait_stream(side)

        row = {"ctx": C, "attn": graph_us(attn)}
        row["attn+oproj"] = graph_us(lambda i: (attn(i), ops.decode_proj(out, ow[i % nbuf])))
        gamma, res_out = torch.ones(H, device=dev, dtype=bf), torch.empty_like(x)
        gu_fn = lambda i: ops.fused_skinny(act, ops.decode_proj(out, ow[i % nbuf]), x, res_out,  # noqa: E731
                                           gamma, 1e-5, guw[i % nbuf], None, 2, 1)
        row["attn+oproj+gu"] = graph_us(lambda i: (attn(i), gu_fn(i)))
        for blk in a.blocks:
            row[f"fork_b{blk}+oproj"] = graph_us(lambda i: (forked(i, blk, None), ops.decode_proj(out, ow[i % nbuf])))
            for k, idx in gu_rows.items():
                row[f"fork_b{blk}_gu{k}t+oproj+gu"] = graph_us(lambda i: (forked(i, blk, idx), gu_fn(i)))
        row = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in row.items()}
        print(json.dumps(row), flush=True)
        rows.append(row)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"base": base, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
