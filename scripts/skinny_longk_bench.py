#!/usr/bin/env python3
"""Decode projections with long K on the skinny weight-streaming kernel (skinny_gemm.hip, every
launch config) vs hipBLASLt, hipGraph-timed with weights streamed cold (rotated over buffers larger
than the MALL): the 8B down-proj [M, 14336] x [4096, 14336]^T and the 8B o-proj [M, 4096] x
[4096, 4096]^T.  One JSON line per (shape, M): us per launch and TB/s of weight stream."""
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
    ap.add_argument("--ms", type=int, nargs="+", default=[1, 4])
    ap.add_argument("--cfgs", type=int, nargs="+", default=list(range(1, 12)))
    a = ap.parse_args()
    ops.load_native(required=True)
    dev, bf = "cuda", torch.bfloat16
    for name, N, K in (("down", 4096, 14336), ("o", 4096, 4096)):
        nbuf = max(2, int(600e6 // (N * K * 2)) + 1)
        ws = [torch.randn(N, K, device=dev, dtype=bf) * 0.02 for _ in range(nbuf)]
        gb = N * K * 2 / 1e9
        for M in a.ms:
            x = torch.randn(M, K, device=dev, dtype=bf)
            y = torch.empty(M, N, device=dev, dtype=bf)
            ref = x.float() @ ws[0].float().t()
            t = graph_time(lambda i: torch.nn.functional.linear(x, ws[i % nbuf]))
            row = {"shape": name, "M": M, "N": N, "K": K, "hipblaslt_us": round(t, 2), "hipblaslt_TBs": round(gb / t * 1e6 / 1e3, 2)}
            best = None
            for cfg in a.cfgs:
                try:
                    torch.ops.dgi.skinny_gemm(y, x, ws[0], None, cfg)
                    torch.cuda.synchronize()
                except RuntimeError as e:
                    row[f"c{cfg}"] = f"skip: {str(e)[:50]}"
                    continue
                err = (y.float() - ref).abs().max().item() / ref.abs().max().item()
                t = graph_time(lambda i: torch.ops.dgi.skinny_gemm(y, x, ws[i % nbuf], None, cfg))
                row[f"c{cfg}"] = round(t, 2)
                if err > 0.02:
                    row[f"c{cfg}_bad"] = round(err, 4)
                elif best is None or t < best[1]:
                    best = (cfg, t)
            if best:
                row["best"] = {"cfg": best[0], "us": round(best[1], 2), "TBs": round(gb / best[1] * 1e6 / 1e3, 2)}
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
