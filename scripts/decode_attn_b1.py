#!/usr/bin/env python3
"""Small-batch decode attention latency (Llama-3-8B geometry: 32 q / 8 kv heads x 128).

Times ``--chain`` back-to-back ``ops.paged_decode`` launches captured in one hipGraph (what
the decode step replays), per launch, for the three plans the graph runner can capture:

* one split per (sequence, kv head), 8-wave workgroups (the short-context graph);
* split plan (device-side, parts of >= 128 tokens) + the reduce kernel;
* split plan with the in-kernel ticket reduce (workspace counters);

plus a trivial copy kernel chained the same way (the dependent-launch floor).  Prints one
JSON line per (batch, context)."""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from dgi import ops

nh, nkv, hd, bs = 32, 8, 128, 16


def graph_us(fn, chain: int, reps: int = 20) -> float:
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(chain):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / (reps * chain)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 4])
    ap.add_argument("--ctx", type=int, nargs="+", default=[128, 256, 384, 512, 1024, 2048])
    ap.add_argument("--chain", type=int, default=32)
    ap.add_argument("--heads", type=int, nargs=2, default=[nh, nkv])
    a = ap.parse_args()
    globals().update(nh=a.heads[0], nkv=a.heads[1])
    ops.load_native(required=True)
    dev = "cuda"
    scale = 1 / math.sqrt(hd)
    for B in a.batch:
        for C in a.ctx:
            nb_seq = (C + bs - 1) // bs
            nblk = B * nb_seq + 1
            kc = torch.randn(nblk, nkv, bs, hd, device=dev, dtype=torch.bfloat16)
            vc = torch.randn_like(kc)
            perm = torch.randperm(nblk - 1, device=dev).to(torch.int32) + 1
            bt = perm.view(B, nb_seq).contiguous()
            ctx = torch.full((B,), C, device=dev, dtype=torch.int32)
            q = torch.randn(B, (nh + 2 * nkv) * hd, device=dev, dtype=torch.bfloat16)
            out = torch.empty(B, nh * hd, device=dev, dtype=torch.bfloat16)
            ms = 2048 // 128
            ws = (torch.empty(B * nh * ms * hd, device=dev), torch.empty(B * nh * ms, device=dev))
            wsc = ws + (torch.zeros(B * nkv, dtype=torch.int32, device=dev),)
            want = max(1, -(-4 * 256 // (B * nkv)))
            splits = min(ms, want)
            ref = ops.paged_decode_ref(q, kc, vc, bt, ctx, nh, nkv, scale).float()
            row = {"batch": B, "ctx": C, "heads": [nh, nkv]}
            _variants(row, q, kc, vc, bt, ctx, out, ref, ws, wsc, splits, scale, a.chain)
            src = torch.randn(B, nh * hd, device=dev, dtype=torch.bfloat16)
            row["copy_floor_us"] = round(graph_us(lambda: out.copy_(src), a.chain), 2)
            print(json.dumps(row), flush=True)


def _variants(row, q, kc, vc, bt, ctx, out, ref, ws, wsc, splits, scale, chain):
    for name, kw in (("one_split", dict(max_splits=1, part_size=1 << 20)),
                     ("split_reduce", dict(max_splits=splits, part_size=-128, workspace=ws)),
                     ("split_fused", dict(max_splits=splits, part_size=-128, workspace=wsc))):
        fn = lambda kw=kw: ops.paged_decode(q, kc, vc, bt, ctx, nh, nkv, scale, out=out, **kw)  # noqa: E731
        row[name + "_us"] = round(graph_us(fn, chain), 2)
        row[name + "_err"] = round((out.float() - ref).abs().max().item(), 4)


if __name__ == "__main__":
    main()
