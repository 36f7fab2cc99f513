#!/usr/bin/env python3
"""Two vs four MFMA phases per K tile for the fused-norm GEMMs (mfma_gemm.hip EPI 2-4) at the 70B
headline's mixed-step row counts.  The auto rule (2 phases up to M = 2560) was measured on the plain
and SwiGLU epilogues (round 3); this checks it for the fused-norm ones.  hipGraph-timed, 20 launches
per replay, weights rotated through a set larger than the MALL.  One JSON line per (proj, M)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgi import ops  # noqa: E402
from scripts.norm_gemm_bench import graph_us  # noqa: E402


def main():
    ops.load_native(required=True)
    dev, bf = "cuda", torch.bfloat16
    H = 8192
    Ms = [int(x) for x in os.environ.get("NP_M", "1536,1792,2048").split(",")]
    shapes = (("qkv", 10240, H, ops.NORM_PLAIN), ("gate_up", 57344, H, ops.NORM_SWIGLU),
              ("o", H, 8192, ops.NORM_RES), ("down", H, 28672, ops.NORM_RES))
    for name, N, K, kind in shapes:
        nbuf = max(2, int(1.2e9 // (N * K * 2)))
        ws = [torch.randn(N, K, device=dev, dtype=bf) * 0.02 for _ in range(nbuf)]
        for M in Ms:
            x = torch.randn(M, K, device=dev, dtype=bf)
            if kind == ops.NORM_RES:
                out = torch.randn(M, N, device=dev, dtype=bf)
                ss = torch.zeros(M, N // 256, device=dev)
            else:
                ss = torch.rand(M, 32, device=dev) * K * 0.1
                out = torch.empty(M, N // 2 if kind == ops.NORM_SWIGLU else N, device=dev, dtype=bf)
            row = {"proj": name, "M": M}
            for ph in (2, 4, 2, 4):          # alternating, twice: drift shows up as a spread
                us = graph_us(lambda i: ops.mfma_gemm_norm(x, ws[i % nbuf], kind, ss, 1e-5, out=out, phases=ph))
                row.setdefault(f"ph{ph}_us", []).append(round(us, 2))
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
