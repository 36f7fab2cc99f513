#!/usr/bin/env python3
"""Decode down-projection (8B: [M, 14336] x [4096, 14336]^T) on the fused_skinny
GEMV (no prologue, plain store) per launch config vs hipBLASLt, hipGraph-timed with
weights streamed cold (rotated over buffers larger than the MALL).  Prints one JSON
line per M with us per launch and the max error vs the fp32 reference.

    python scripts/down_gemv_bench.py [--ms 1 2 4 8 16] [--cfgs 6 7 8 10 11 12 13 14 15 16]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgi import ops  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from fused_decode_bench import graph_time  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", type=int, nargs="+", default=[1, 2, 4, 8, 16])
    ap.add_argument("--cfgs", type=int, nargs="+", default=[6, 7, 8, 10, 11, 12, 13, 14, 15, 16])
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--k", type=int, default=14336)
    a = ap.parse_args()
    ops.load_native(required=True)
    dev, bf = "cuda", torch.bfloat16
    N, K = a.n, a.k
    nbuf = max(2, int(600e6 // (N * K * 2)) + 1)
    ws = [torch.randn(N, K, device=dev, dtype=bf) * 0.02 for _ in range(nbuf)]
    for M in a.ms:
        x = torch.randn(M, K, device=dev, dtype=bf)
        y = torch.empty(M, N, device=dev, dtype=bf)
        ref = (x.float() @ ws[0].float().t())
        row = {"M": M, "N": N, "K": K,
               "hipblaslt_us": round(graph_time(lambda i: torch.nn.functional.linear(x, ws[i % nbuf])), 2)}
        for cfg in a.cfgs:
            try:
                print(f"eager M={M} cfg={cfg}", file=sys.stderr, flush=True)
                ops.fused_skinny(y, x, None, None, None, 0.0, ws[0], None, 0, 0, cfg=cfg)
                torch.cuda.synchronize()
            except RuntimeError as e:
                row[f"c{cfg}"] = f"skip: {str(e)[:60]}"
                continue
            err = (y.float() - ref).abs().max().item() / ref.abs().max().item()
            t = graph_time(lambda i: ops.fused_skinny(y, x, None, None, None, 0.0, ws[i % nbuf], None, 0, 0, cfg=cfg))
            row[f"c{cfg}"] = round(t, 2)
            row[f"c{cfg}_relerr"] = round(err, 5)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
