#!/usr/bin/env python3
"""Do forked branches of a captured hipGraph run concurrently on this ROCm?

Two independent pieces of work — a compute-bound GEMM (the decode stage's
gate_up shape at 384 rows) and an HBM-bound stream (a large copy) — are timed
serially, eagerly on two streams, captured into one graph in stream order, and
captured with a fork/join across two streams (the two-batch-overlap structure).
Prints one JSON line per variant (median of ``--reps`` replays)."""
from __future__ import annotations

import argparse
import json
import statistics

import torch


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=384)
    ap.add_argument("--copy-mb", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    x = torch.randn(a.rows, 8192, device=dev, dtype=torch.bfloat16)
    w = torch.randn(57344, 8192, device=dev, dtype=torch.bfloat16) * 0.01
    y = torch.empty(a.rows, 57344, device=dev, dtype=torch.bfloat16)
    n = a.copy_mb * (1 << 20) // 2
    src = torch.randn(n, device=dev, dtype=torch.bfloat16)
    dst = torch.empty_like(src)
    side = torch.cuda.Stream(device=dev)
    main_s = torch.cuda.current_stream()

    def gemm():
        torch.matmul(x, w.t(), out=y)

    def copy():
        dst.copy_(src)

    def serial():
        gemm()
        copy()

    def forked():
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            copy()
        gemm()
        torch.cuda.current_stream().wait_stream(side)

    res = {"gemm_ms": timed(gemm, a.reps), "copy_ms": timed(copy, a.reps), "eager_serial_ms": timed(serial, a.reps),
           "eager_forked_ms": timed(forked, a.reps)}
    for name, body in (("graph_serial_ms", serial), ("graph_forked_ms", forked)):
        body()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            body()
        torch.cuda.synchronize()
        res[name] = timed(g.replay, a.reps)
    del main_s
    res = {k: round(v, 4) for k, v in res.items()}
    res["rows"], res["copy_mb"] = a.rows, a.copy_mb
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
