#!/usr/bin/env python3
"""70B qkv / o projections at decode-role row counts: hipBLASLt (ops.linear) vs the MFMA kernel's
ping-pong schedule (256 x 256 tiles + hybrid split-K) vs the 128 x 128 half tile (sched 4).
hipGraph-timed, 20 launches per replay, weights rotated through a set larger than the MALL.
One JSON line per (projection, M)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgi import ops  # noqa: E402


def graph_us(fn, reps=20, iters=5):
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
    ops.load_native(required=True)
    dev, bf = "cuda", torch.bfloat16
    for name, N, K in (("qkv", 10240, 8192), ("o", 8192, 8192)):
        nbuf = max(2, int(1.2e9 // (N * K * 2)))
        ws = [torch.randn(N, K, device=dev, dtype=bf) * 0.02 for _ in range(nbuf)]
        for M in (256, 512, 768, 1024):
            x = torch.randn(M, K, device=dev, dtype=bf)
            y = torch.empty(M, N, device=dev, dtype=bf)
            row = {"proj": name, "M": M}
            row["blas_us"] = graph_us(lambda i: ops.linear(x, ws[i % nbuf]))
            row["pp_us"] = graph_us(lambda i: ops.mfma_gemm(x, ws[i % nbuf], 0, out=y, sched=3))
            row["half_us"] = graph_us(lambda i: ops.mfma_gemm(x, ws[i % nbuf], 0, out=y, sched=4))
            ref = torch.nn.functional.linear(x, ws[0])
            got = ops.mfma_gemm(x, ws[0], 0, sched=4)
            row["half_err"] = round((got.float() - ref.float()).abs().max().item(), 4)
            fl = 2 * M * N * K
            for k in ("blas", "pp", "half"):
                row[k + "_pf"] = round(fl / row[k + "_us"] / 1e9, 3)
                row[k + "_us"] = round(row[k + "_us"], 2)
            print(json.dumps(row), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
