#!/usr/bin/env python3
"""hipBLASLt's default pick vs a TunableOp-tuned solution for the 70B projections at the decode
microbatch sizes (512 / 768 rows): is there a faster library kernel for qkv / o at M = 512?

Each GEMM is timed inside a captured hipGraph (20 launches, weights rotated through a set larger
than the MALL) first with TunableOp off, then tuned (rotating buffer, 30 ms budget per shape) and
timed again with the tuned solution.  One JSON line per (shape, M)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("qkv", 10240, 8192), ("o", 8192, 8192), ("gate_up", 57344, 8192), ("down", 8192, 28672)]


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
    import torch.cuda.tunable as tun
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tunableop_decode.csv"
    dev, bf = "cuda", torch.bfloat16
    rows = []
    for name, N, K in SHAPES:
        nbuf = max(2, int(1.2e9 // (N * K * 2)))
        ws = [torch.randn(N, K, device=dev, dtype=bf) * 0.02 for _ in range(nbuf)]
        for M in (512, 768):
            x = torch.randn(M, K, device=dev, dtype=bf)
            tun.enable(False)
            base = graph_us(lambda i: F.linear(x, ws[i % nbuf]))
            tun.enable(True)
            tun.tuning_enable(True)
            tun.set_filename(out)
            tun.set_max_tuning_duration(30)
            F.linear(x, ws[0])                 # tunes this (M, N, K) once
            torch.cuda.synchronize()
            tun.tuning_enable(False)
            tuned = graph_us(lambda i: F.linear(x, ws[i % nbuf]))
            tun.enable(False)
            r = {"proj": name, "M": M, "N": N, "K": K, "default_us": round(base, 2), "tuned_us": round(tuned, 2),
                 "default_pf": round(2 * M * N * K / base / 1e9, 3), "tuned_pf": round(2 * M * N * K / tuned / 1e9, 3)}
            print(json.dumps(r), flush=True)
            rows.append(r)
        del ws
        torch.cuda.empty_cache()
    # the tuned solutions are written to `out` by TunableOp itself at process exit


if __name__ == "__main__":
    main()
