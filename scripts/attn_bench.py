"""Attention kernel microbenchmarks at Llama-3-70B head geometry (nh=64, nkv=8, hd=128).

* paged prefill (dgi HIP kernel): B prompts of L tokens, causal, KV in the paged pool;
  reference point: torch SDPA (ROCm flash/CK path) on the same dense problem;
* paged decode (dgi HIP kernel): B sequences at context C; effective KV bandwidth.
"""
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from dgi import ops

nh, nkv, hd, bs = 64, 8, 128, 16
dev = "cuda"


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def prefill(B, L):
    nblk = B * (L // bs) + 1
    kc = torch.randn(nblk, nkv, bs, hd, device=dev, dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.arange(1, nblk, device=dev, dtype=torch.int32).view(B, L // bs)
    cu = torch.arange(0, (B + 1) * L, L, device=dev, dtype=torch.int32)
    ctx = torch.full((B,), L, device=dev, dtype=torch.int32)
    q = torch.randn(B * L, (nh + 2 * nkv) * hd, device=dev, dtype=torch.bfloat16)
    tl = ops.prefill_tiles(cu.tolist())
    if os.environ.get("ATTN_TILE_ORDER", "1") == "0":      # A/B: (sequence, row) order
        tl = sorted(tl)
    tiles = torch.tensor(tl, dtype=torch.int32, device=dev)
    out = torch.empty(B * L, nh * hd, device=dev, dtype=torch.bfloat16)
    scale = 1 / math.sqrt(hd)
    us = timed(lambda: ops.paged_prefill(q, kc, vc, bt, cu, ctx, nh, nkv, scale, tiles=tiles, out=out))
    flops = 4 * nh * hd * B * L * L / 2
    qd = torch.randn(B, nh, L, hd, device=dev, dtype=torch.bfloat16)
    kd = torch.randn(B, nh, L, hd, device=dev, dtype=torch.bfloat16)
    vd = torch.randn_like(kd)
    us_sdpa = timed(lambda: F.scaled_dot_product_attention(qd, kd, vd, is_causal=True))
    return {"kernel": "prefill", "B": B, "L": L, "tile": ops.PREFILL_TILE, "db": ops.PREFILL_DB,
            "order": os.environ.get("ATTN_TILE_ORDER", "1"), "us": round(us, 1),
            "TFLOPs": round(flops / us / 1e6, 1),
            "sdpa_us": round(us_sdpa, 1), "sdpa_TFLOPs": round(flops / us_sdpa / 1e6, 1)}


def decode(B, C):
    nb_seq = (C + bs - 1) // bs
    nblk = B * nb_seq + 1
    kc = torch.randn(nblk, nkv, bs, hd, device=dev, dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.arange(1, nblk, device=dev, dtype=torch.int32).view(B, nb_seq)
    ctx = torch.full((B,), C, device=dev, dtype=torch.int32)
    q = torch.randn(B, (nh + 2 * nkv) * hd, device=dev, dtype=torch.bfloat16)
    splits, part = ops.decode_split_plan(B, C, nkv)
    out = torch.empty(B, nh * hd, device=dev, dtype=torch.bfloat16)
    ws = (torch.empty(B * nh * ((C + 127) // 128) * hd, device=dev), torch.empty(B * nh * ((C + 127) // 128), device=dev))
    scale = 1 / math.sqrt(hd)
    us = timed(lambda: ops.paged_decode(q, kc, vc, bt, ctx, nh, nkv, scale, splits, part, out=out, workspace=ws))
    byts = B * C * nkv * hd * 2 * 2
    return {"kernel": "decode", "B": B, "C": C, "splits": splits, "us": round(us, 1),
            "KV_TBs": round(byts / us / 1e6, 2)}


if __name__ == "__main__":
    for tile in [int(t) for t in os.environ.get("ATTN_TILES", "128").split(",")]:
        for db in [int(d) for d in os.environ.get("ATTN_DB", str(ops.PREFILL_DB)).split(",")]:
            ops.PREFILL_TILE, ops.PREFILL_DB = tile, db
            for B, L in [(1, 512), (3, 512), (8, 512), (4, 2048), (1, 8192)]:
                print(json.dumps(prefill(B, L)), flush=True)
    if os.environ.get("ATTN_PREFILL_ONLY"):
        sys.exit(0)
    for B, C in [(1, 1024), (64, 1024), (256, 640), (384, 640), (512, 2048), (32, 8192)]:
        print(json.dumps(decode(B, C)), flush=True)
