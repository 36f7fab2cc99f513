#!/usr/bin/env python3
"""Short driver for rocprofv3 ``--pmc`` passes over the hot HIP kernels at serving shapes
(VERDICT r4 #4): each kernel runs ``--iters`` times on uniform random data.

* paged_decode, batch 1 at 2048 tokens (8B decode) and 768 rows at 576 tokens (70B decode
  stage), both with the graphs' device split plan;
* paged_prefill, 8 x 512 causal and 1 x 8192 causal (70B heads);
* mfma_gemm_pp (70B gate_up + SwiGLU and down at M = 768 and 2048);
* fused_skinny (8B qkv with RMSNorm + RoPE/KV epilogue, gate_up + SwiGLU at M = 1).

``--only`` picks a subset (comma list of: decode, prefill, gemm, skinny)."""
from __future__ import annotations

import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgi import ops  # noqa: E402

dev = "cuda"


def rnd(*shape, scale=1.0):
    return ((torch.rand(*shape, device=dev) * 2 - 1) * scale).to(torch.bfloat16)


def decode(B, C, nh, nkv, iters):
    hd, bs = 128, 16
    nbs = (C + bs - 1) // bs
    nblk = B * nbs + 1
    kc, vc = rnd(nblk, nkv, bs, hd), rnd(nblk, nkv, bs, hd)
    bt = torch.randperm(nblk - 1, device=dev).add(1).int()[: B * nbs].view(B, nbs).contiguous()
    ctx = torch.full((B,), C, device=dev, dtype=torch.int32)
    q = rnd(B, (nh + 2 * nkv) * hd)
    ws_splits = (2048 + 127) // 128 if C <= 2048 else (C + 127) // 128
    ws = (torch.empty(B * nh * ws_splits * hd, device=dev), torch.empty(B * nh * ws_splits, device=dev))
    want = max(1, -(-4 * 256 // max(1, B * nkv)))
    splits, part = min(ws_splits, want), -(128 if B < 8 else 64)
    out = torch.empty(B, nh * hd, device=dev, dtype=torch.bfloat16)
    for _ in range(iters):
        ops.paged_decode(q, kc, vc, bt, ctx, nh, nkv, 1 / math.sqrt(hd), splits, part, out=out, workspace=ws)


def prefill(B, L, iters):
    nh, nkv, hd, bs = 64, 8, 128, 16
    nblk = B * (L // bs) + 1
    kc, vc = rnd(nblk, nkv, bs, hd), rnd(nblk, nkv, bs, hd)
    bt = torch.arange(1, nblk, device=dev, dtype=torch.int32).view(B, L // bs)
    cu = torch.arange(0, (B + 1) * L, L, device=dev, dtype=torch.int32)
    ctx = torch.full((B,), L, device=dev, dtype=torch.int32)
    q = rnd(B * L, (nh + 2 * nkv) * hd)
    tiles = torch.tensor(ops.prefill_tiles(cu.tolist()), dtype=torch.int32, device=dev)
    out = torch.empty(B * L, nh * hd, device=dev, dtype=torch.bfloat16)
    for _ in range(iters):
        ops.paged_prefill(q, kc, vc, bt, cu, ctx, nh, nkv, 1 / math.sqrt(hd), tiles=tiles, out=out)


def gemm(M, iters):
    for N, K, epi in ((57344, 8192, 1), (8192, 28672, 0)):
        x, w = rnd(M, K), rnd(N, K, scale=0.02)
        for _ in range(iters):
            ops.mfma_gemm(x, w, epi)


def skinny(iters):
    K, nh, nkv, hd, bs, nb = 4096, 32, 8, 128, 16, 256
    x, res = rnd(1, K), rnd(1, K)
    gamma = (1 + 0.1 * torch.randn(K, device=dev)).bfloat16()
    wq, wg = rnd((nh + 2 * nkv) * hd, K, scale=0.02), rnd(2 * 14336, K, scale=0.02)
    pos = torch.tensor([700], device=dev, dtype=torch.int32)
    cos_sin = ops.rope_cos_sin(128, 4096, 500000.0, device=torch.device(dev))
    slots = torch.tensor([77], device=dev, dtype=torch.int32)
    kc = torch.zeros(nb, nkv, bs, hd, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    yq = torch.empty(1, wq.shape[0], device=dev, dtype=torch.bfloat16)
    yg = torch.empty(1, 14336, device=dev, dtype=torch.bfloat16)
    ro = torch.empty_like(x)
    for _ in range(iters):
        ops.fused_skinny(yq, x, res, ro, gamma, 1e-5, wq, None, 2, 2, pos, cos_sin, slots, kc, vc, nh, nkv)
        ops.fused_skinny(yg, x, res, ro, gamma, 1e-5, wg, None, 2, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="decode,prefill,gemm,skinny")
    a = ap.parse_args()
    ops.load_native(required=True)
    only = set(a.only.split(","))
    if "decode" in only:
        decode(1, 2048, 32, 8, a.iters)
        decode(768, 576, 64, 8, a.iters)
    if "prefill" in only:
        prefill(8, 512, a.iters)
        prefill(1, 8192, a.iters)
    if "gemm" in only:
        gemm(768, a.iters)
        gemm(2048, a.iters)
    if "skinny" in only:
        skinny(a.iters)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
