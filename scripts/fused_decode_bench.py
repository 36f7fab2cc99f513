#!/usr/bin/env python3
"""Microbenchmarks for the decode-step kernels, timed inside hipGraphs (as decode runs).

* fused_skinny (norm prologue + SwiGLU / RoPE epilogue) per launch config vs the
  unfused chain (rmsnorm + skinny/hipBLASLt GEMM + silu_mul / rope_cache);
* paged decode attention: fixed r1 split plan + reduce kernel vs the device-side
  plan (min part sizes) with the reduce kernel or the in-kernel ticket reduce.
Weights are bf16 random, streamed cold (a buffer set larger than the 256 MB MALL
is rotated through).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgi import ops  # noqa: E402


def graph_time(fn, reps=20, iters=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn(0)
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
    return e0.elapsed_time(e1) * 1000 / (iters * reps)


def bench_gemms(H, I, nh, nkv, Ms, cfgs):
    dev = "cuda"
    bf = torch.bfloat16
    nbuf = 6                       # 6 x (qkv + gate_up) > MALL: weights come from HBM
    qkv_w = [torch.randn((nh + 2 * nkv) * 128, H, device=dev, dtype=bf) * 0.02 for _ in range(nbuf)]
    gu_w = [torch.randn(2 * I, H, device=dev, dtype=bf) * 0.02 for _ in range(nbuf)]
    gamma = torch.ones(H, device=dev, dtype=bf)
    inv = 1.0 / (10000 ** (torch.arange(0, 64, device=dev).float() / 64))
    ang = torch.arange(4096, device=dev).float()[:, None] * inv[None]
    cs = torch.cat([ang.cos(), ang.sin()], 1).contiguous()
    kc = torch.zeros(512, nkv, 16, 128, device=dev, dtype=bf)
    vc = torch.zeros_like(kc)
    rows = []
    for M in Ms:
        x = torch.randn(M, H, device=dev, dtype=bf)
        res = torch.randn(M, H, device=dev, dtype=bf)
        ro = torch.empty_like(x)
        pos = torch.arange(100, 100 + M, device=dev, dtype=torch.int32)
        slots = torch.arange(M, device=dev, dtype=torch.int32)
        qkv = torch.empty(M, qkv_w[0].shape[0], device=dev, dtype=bf)
        act = torch.empty(M, I, device=dev, dtype=bf)
        row = {"M": M}
        ok = []
        for cfg in cfgs:                  # eager first: a fault names its variant
            try:
                for epi, (yy, ww) in ((2, (qkv, qkv_w[0])), (1, (act, gu_w[0]))):
                    print(f"eager M={M} cfg={cfg} epi={epi}", flush=True)
                    ops.fused_skinny(yy, x, res, ro, gamma, 1e-5, ww, None, 2, epi, pos, cs, slots, kc, vc, nh,
                                     nkv, cfg=cfg)
                    torch.cuda.synchronize()
                ok.append(cfg)
            except RuntimeError as e:     # launch config rejected for this M (LDS budget)
                print(f"skip cfg {cfg} at M={M}: {e}", flush=True)
        for cfg in ok:
            row[f"qkv_fused_c{cfg}"] = round(graph_time(lambda i: ops.fused_skinny(
                qkv, x, res, ro, gamma, 1e-5, qkv_w[i % nbuf], None, 2, 2, pos, cs, slots, kc, vc, nh, nkv,
                cfg=cfg)), 2)
            row[f"gu_fused_c{cfg}"] = round(graph_time(lambda i: ops.fused_skinny(
                act, x, res, ro, gamma, 1e-5, gu_w[i % nbuf], None, 2, 1, cfg=cfg)), 2)

        def unfused_qkv(i):
            xx = x.clone()
            rr = res.clone()
            ops.fused_add_rmsnorm(xx, rr, gamma, 1e-5)
            q = ops.linear(xx, qkv_w[i % nbuf])
            ops.rope_cache(q, pos, cs, nh, nkv, 128, slots, kc, vc, 0)

        def unfused_gu(i):
            xx = x.clone()
            rr = res.clone()
            ops.fused_add_rmsnorm(xx, rr, gamma, 1e-5)
            ops.silu_mul(ops.linear(xx, gu_w[i % nbuf]))
        row["qkv_unfused"] = round(graph_time(unfused_qkv), 2)
        row["gu_unfused"] = round(graph_time(unfused_gu), 2)
        row["clone_x2"] = round(graph_time(lambda i: (x.clone(), res.clone())), 2)
        print(json.dumps(row), flush=True)
        rows.append(row)
    return rows


def bench_plain(shapes, Ms):
    """skinny_gemm launch configs vs hipBLASLt (torch.matmul) on plain decode projections."""
    dev, bf = "cuda", torch.bfloat16
    rows = []
    for name, N, K in shapes:
        nbuf = max(2, int(2.5e9 // (N * K * 2)))      # rotate > MALL worth of weights
        ws = [torch.randn(N, K, device=dev, dtype=bf) * 0.02 for _ in range(nbuf)]
        for M in Ms:
            x = torch.randn(M, K, device=dev, dtype=bf)
            y = torch.empty(M, N, device=dev, dtype=bf)
            row = {"gemm": name, "M": M, "N": N, "K": K,
                   "hipblaslt": round(graph_time(lambda i: torch.matmul(x, ws[i % nbuf].t(), out=y)), 2)}
            for cfg in range(1, 12):
                try:
                    row[f"skinny_c{cfg}"] = round(graph_time(
                        lambda i: torch.ops.dgi.skinny_gemm(y, x, ws[i % nbuf], None, cfg)), 2)
                except Exception as e:          # shape not supported by this config
                    row[f"skinny_c{cfg}"] = None
            print(json.dumps(row), flush=True)
            rows.append(row)
    return rows


def bench_attn(nh, nkv, Bs, ctxs):
    dev = "cuda"
    bf = torch.bfloat16
    bs = 16
    rows = []
    for B in Bs:
        for ctx in ctxs:
            nblk = B * ((ctx + bs - 1) // bs) + 4
            kc = torch.randn(nblk, nkv, bs, 128, device=dev, dtype=bf)
            vc = torch.randn_like(kc)
            maxw = (ctx + bs - 1) // bs
            bt = torch.arange(B * maxw, device=dev, dtype=torch.int32).view(B, maxw)
            cl = torch.full((B,), ctx, device=dev, dtype=torch.int32)
            q = torch.randn(B, (nh + 2 * nkv) * 128, device=dev, dtype=bf)
            out = torch.empty(B, nh * 128, device=dev, dtype=bf)
            S = 16
            ws2 = (torch.empty(B * nh * S * 128, device=dev), torch.empty(B * nh * S, device=dev))
            ws3 = ws2 + (torch.zeros(B * nkv, device=dev, dtype=torch.int32),)
            sc = 1 / 128 ** 0.5
            row = {"B": B, "ctx": ctx}
            row["r1_fixed256"] = round(graph_time(lambda i: ops.paged_decode(
                q, kc, vc, bt, cl, nh, nkv, sc, 8, 256, out=out, workspace=ws2)), 2)
            want = max(1, -(-4 * 256 // (B * nkv)))
            for mp in (32, 64, 128, 256):
                row[f"dyn{mp}"] = round(graph_time(lambda i: ops.paged_decode(
                    q, kc, vc, bt, cl, nh, nkv, sc, min(S, want), -mp, out=out, workspace=ws2)), 2)
                row[f"dyn{mp}_ticket"] = round(graph_time(lambda i: ops.paged_decode(
                    q, kc, vc, bt, cl, nh, nkv, sc, min(S, want), -mp, out=out, workspace=ws3)), 2)
            print(json.dumps(row), flush=True)
            rows.append(row)
    return rows


def bench_plain_fused(shapes, Ms, cfgs):
    """Plain projections (no prologue / epilogue: o-proj, down) through fused_skinny's
    launch configs (incl. the split-K ones) vs ops.linear (skinny_gemm / hipBLASLt)."""
    dev, bf = "cuda", torch.bfloat16
    rows = []
    for name, N, K in shapes:
        nbuf = max(2, int(2.5e9 // (N * K * 2)))
        ws = [torch.randn(N, K, device=dev, dtype=bf) * 0.02 for _ in range(nbuf)]
        for M in Ms:
            x = torch.randn(M, K, device=dev, dtype=bf)
            y = torch.empty(M, N, device=dev, dtype=bf)
            row = {"proj": name, "M": M, "linear": round(graph_time(lambda i: ops.linear(x, ws[i % nbuf])), 2)}
            for cfg in cfgs:
                try:
                    ops.fused_skinny(y, x, None, None, None, 0.0, ws[0], None, 0, 0, cfg=cfg)
                    torch.cuda.synchronize()
                except RuntimeError as e:
                    print(f"skip {name} cfg {cfg} M={M}: {e}", flush=True)
                    continue
                row[f"c{cfg}"] = round(graph_time(lambda i: ops.fused_skinny(
                    y, x, None, None, None, 0.0, ws[i % nbuf], None, 0, 0, cfg=cfg)), 2)
            print(json.dumps(row), flush=True)
            rows.append(row)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--cfgs", type=int, nargs="+", default=[0, 2, 3, 4, 5])
    ap.add_argument("--skip-attn", action="store_true")
    ap.add_argument("--skip-gemms", action="store_true", help="skip the fused qkv / gate_up table")
    ap.add_argument("--plain-fused", action="store_true", help="also o-proj / down through fused_skinny configs")
    ap.add_argument("--plain", action="store_true", help="only the plain skinny-vs-hipBLASLt table")
    ap.add_argument("--plain-fused-ms", type=int, nargs="+", default=[1, 4, 8], help="row counts of --plain-fused")
    ap.add_argument("--gemm-ms", type=int, nargs="+", default=[1, 2, 4, 8, 16], help="row counts of the fused table")
    ap.add_argument("--plain-fused-qkv", action="store_true", help="--plain-fused also times the qkv shape")
    a = ap.parse_args()
    if a.plain:
        ops.load_native(required=True)
        res = {"plain_8b": bench_plain([("down", 4096, 14336), ("o", 4096, 4096), ("qkv", 6144, 4096),
                                        ("gate_up", 28672, 4096)], [1, 2, 4, 8, 16])}
        if a.out:
            with open(a.out, "w") as f:
                json.dump(res, f, indent=1)
        return
    res = {} if a.skip_gemms else {"gemm_8b": bench_gemms(4096, 14336, 32, 8, a.gemm_ms, a.cfgs)}
    if a.plain_fused:
        shapes = [("o", 4096, 4096), ("down", 4096, 14336)] + ([("qkv", 6144, 4096)] if a.plain_fused_qkv else [])
        res["plain_fused_8b"] = bench_plain_fused(shapes, a.plain_fused_ms, a.cfgs)
    if not a.skip_attn:
        res["attn_8b"] = bench_attn(32, 8, [1, 4, 16], [256, 384, 1024, 4096])
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
