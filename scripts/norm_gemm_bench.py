#!/usr/bin/env python3
"""Fused-norm MFMA GEMMs (mfma_gemm.hip EPI 2-4) against their plain counterparts at the 70B
projection shapes: qkv / gate_up with the rstd epilogue vs plain (and hipBLASLt), o / down with the
residual + row-statistics epilogue vs plain, plus the RMSNorm kernels the fusion removes.
hipGraph-timed, 20 launches per replay, weights rotated through a set larger than the MALL (decode
weights arrive cold).  One JSON line per (projection, M).  (The r6s7 diagnosis runs that switched
parts of the fused epilogues off used a DGI_NORM_GEMM_DBG kernel knob since removed: commit 7b6799a has it.)"""
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
    H = 8192
    Ms = [int(x) for x in os.environ.get("NG_M", "512,1024,2048").split(",")]
    shapes = (("qkv", 10240, H, ops.NORM_PLAIN), ("gate_up", 57344, H, ops.NORM_SWIGLU),
              ("o", H, 8192, ops.NORM_RES), ("down", H, 28672, ops.NORM_RES))
    for name, N, K, kind in shapes:
        nbuf = max(2, int(1.2e9 // (N * K * 2)))
        ws = [torch.randn(N, K, device=dev, dtype=bf) * 0.02 for _ in range(nbuf)]
        for M in Ms:
            x = torch.randn(M, K, device=dev, dtype=bf)
            row = {"proj": name, "M": M}
            if kind == ops.NORM_RES:
                R = torch.randn(M, N, device=dev, dtype=bf)
                ss = torch.zeros(M, 32, device=dev)
                y = torch.empty(M, N, device=dev, dtype=bf)
                row["plain_us"] = graph_us(lambda i: ops.mfma_gemm(x, ws[i % nbuf], 0, out=y, sched=3))
                row["fused_us"] = graph_us(lambda i: ops.mfma_gemm_norm(x, ws[i % nbuf], kind, ss, 1e-5, out=R))
                row["blas_us"] = graph_us(lambda i: ops.linear(x, ws[i % nbuf]))
                # the norm kernel the fusion removes after this projection
                hh, rr, g = torch.randn(M, N, device=dev, dtype=bf), torch.randn(M, N, device=dev, dtype=bf), \
                    torch.ones(N, device=dev, dtype=bf)
                row["add_rmsnorm_us"] = graph_us(lambda i: ops.fused_add_rmsnorm(hh, rr, g, 1e-5))
            else:
                ss = torch.rand(M, 32, device=dev) * K * 0.1
                epi = 1 if kind == ops.NORM_SWIGLU else 0
                No = N // 2 if epi else N
                y = torch.empty(M, No, device=dev, dtype=bf)
                row["plain_us"] = graph_us(lambda i: ops.mfma_gemm(x, ws[i % nbuf], epi, out=y, sched=3))
                row["fused_us"] = graph_us(lambda i: ops.mfma_gemm_norm(x, ws[i % nbuf], kind, ss, 1e-5, out=y))
                if not epi:
                    row["blas_us"] = graph_us(lambda i: ops.linear(x, ws[i % nbuf]))
            fl = 2 * M * N * K
            for k in list(row):
                if k.endswith("_us") and k != "add_rmsnorm_us":
                    row[k.replace("_us", "_pf")] = round(fl / row[k] / 1e9, 3)
                if k.endswith("_us"):
                    row[k] = round(row[k], 2)
            print(json.dumps(row), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
