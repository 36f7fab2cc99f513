#!/usr/bin/env python3
"""Re-time the routing table's qkv / o-proj columns (pq_blas / pq_mfma / po_blas / po_mfma) with
cold weights, as decoding sees them: 80 layers x 1.7 GB never fit the 256 MB MALL, while the
start-up table times one warm weight eagerly.  hipGraph-timed (20 launches per replay) with the
weights rotated through a set larger than the MALL, for every grid point up to --m-max rows.
Writes {grid point: {pq_blas, pq_mfma, po_blas, po_mfma}} (ms) as JSON."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgi import ops  # noqa: E402


def graph_ms(fn, reps=20, iters=3):
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
    return e0.elapsed_time(e1) / (reps * iters)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--table", default="dgi/tuned/gemm_table_8192x28672_2822d1108bbb.json")
    ap.add_argument("--m-max", type=int, default=1024)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    ops.load_native(required=True)
    with open(a.table) as f:
        grid = [m for m in json.load(f)["grid"] if m <= a.m_max]
    dev, bf = "cuda", torch.bfloat16
    H = 8192
    qkv = [torch.randn(10240, H, device=dev, dtype=bf) * 0.02 for _ in range(8)]
    o = [torch.randn(H, H, device=dev, dtype=bf) * 0.02 for _ in range(9)]
    x = torch.randn(a.m_max, H, device=dev, dtype=bf)
    ops.mfma_gemm(x[:256], qkv[0], 0)          # split-K workspace outside any capture
    res = {}
    for m in grid:
        xm = x[:m]
        r = {"pq_blas": graph_ms(lambda i: ops.linear(xm, qkv[i % 8])),
             "pq_mfma": graph_ms(lambda i: ops.mfma_gemm(xm, qkv[i % 8], 0)),
             "po_blas": graph_ms(lambda i: ops.linear(xm, o[i % 9])),
             "po_mfma": graph_ms(lambda i: ops.mfma_gemm(xm, o[i % 9], 0))}
        res[m] = {k: round(v, 5) for k, v in r.items()}
        print(json.dumps({"m": m, **res[m]}), flush=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
