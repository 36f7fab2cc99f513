#!/usr/bin/env python3
"""Where the ping-pong MFMA GEMM loses time on the decode role's qkv / o (70B, M = 512-768).

At 512 rows qkv has 80 and o 64 output tiles of 256 x 256 on 256 CUs.  The kernel then splits the
tiles along K (hybrid split-K, ``mfma_gemm.hip`` "Work decomposition").  This probe times the
same GEMM with split-K off (whole tiles on 80 / 64 CUs: the per-tile rate) and with the grid
limited to fewer CUs (``ops.set_gemm_cus``: 2 instead of 3 pieces per tile).  From those numbers
the split overhead (fp32 slab round trip, pipeline refill per piece) can be read off against the
per-tile rate.  hipGraph-timed, 20 launches per replay, weights rotated through a set larger than
the MALL (decode weights arrive cold).  One JSON line per (projection, M, variant)."""
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
    Ms = [int(x) for x in os.environ.get("PP_M", "512,768").split(",")]
    shapes = (("qkv", 10240, 8192), ("o", 8192, 8192))
    variants = [("auto", 0, 0, 0), ("auto_ph2", 0, 0, 2), ("auto_ph4", 0, 0, 4), ("whole", 1, 0, 0),
                ("always", 2, 0, 0), ("cus160", 0, 160, 0), ("cus192", 0, 192, 0), ("cus128", 0, 128, 0)]
    for name, N, K in shapes:
        nbuf = max(2, int(1.2e9 // (N * K * 2)))
        ws = [torch.randn(N, K, device=dev, dtype=bf) * 0.02 for _ in range(nbuf)]
        for M in Ms:
            x = torch.randn(M, K, device=dev, dtype=bf)
            y = torch.empty(M, N, device=dev, dtype=bf)
            fl = 2 * M * N * K
            base = {"proj": name, "M": M, "tiles": ((M + 255) // 256) * (N // 256)}
            for vname, sk, cus, ph in variants:
                ops.set_gemm_cus(cus)
                try:
                    us = graph_us(lambda i: ops.mfma_gemm(x, ws[i % nbuf], 0, out=y, sched=3, streamk=sk, phases=ph))
                finally:
                    ops.set_gemm_cus(0)
                print(json.dumps({**base, "variant": vname, "us": round(us, 2), "pf": round(fl / us / 1e9, 3)}),
                      flush=True)
            us = graph_us(lambda i: ops.linear(x, ws[i % nbuf]))
            print(json.dumps({**base, "variant": "hipblaslt", "us": round(us, 2), "pf": round(fl / us / 1e9, 3)}),
                  flush=True)
            # warm weight (one buffer, MALL-resident): the compute-side rate alone
            us = graph_us(lambda i: ops.mfma_gemm(x, ws[0], 0, out=y, sched=3))
            print(json.dumps({**base, "variant": "auto_warm", "us": round(us, 2), "pf": round(fl / us / 1e9, 3)}),
                  flush=True)


if __name__ == "__main__":
    main()
