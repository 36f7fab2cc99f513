#!/usr/bin/env python3
"""Decode-sized GEMMs: hipBLASLt (F.linear) vs the weight-streaming skinny kernel.

Weights rotate over enough copies (> 1 GiB) that every call streams from HBM,
as in a real decode step where a layer's weights were last touched one full
model pass ago (the 256 MB MALL cannot hold them).  Prints one JSON line per
(shape, M, impl) with the time and the achieved weight bandwidth.
"""
import argparse
import json
import sys
import os

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgi import ops  # noqa: E402

SHAPES = {  # name: (N, K)
    "8b_qkv": (6144, 4096), "8b_o": (4096, 4096), "8b_gate_up": (28672, 4096), "8b_down": (4096, 14336),
    "lm_head": (128256, 4096),
    "70b_qkv": (10240, 8192), "70b_o": (8192, 8192), "70b_gate_up": (57344, 8192), "70b_down": (8192, 28672),
}


def timed(fn, iters):
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(iters):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", type=int, nargs="+", default=[1, 2, 4, 8, 16, 32])
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    ap.add_argument("--cfg", type=int, nargs="+", default=[0])
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ops.load_native(required=True)
    rows = []
    for name in a.shapes:
        N, K = SHAPES[name]
        copies = max(2, -(-(1 << 30) // (N * K * 2)))
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        for M in a.ms:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            impls = {"hipblaslt": lambda i: F.linear(x, ws[i % copies])}
            for c in a.cfg:
                impls[f"skinny_c{c}"] = (lambda c_: lambda i: torch.ops.dgi.skinny_gemm(
                    out, x, ws[i % copies], None, c_))(c)
            ref = F.linear(x.float(), ws[0].float())
            torch.ops.dgi.skinny_gemm(out, x, ws[0], None, 0)
            err = (out.float() - ref).abs().max().item()
            for impl, fn in impls.items():
                us = timed(fn, a.iters)
                rows.append({"shape": name, "M": M, "N": N, "K": K, "impl": impl, "us": round(us, 2),
                             "weight_TBs": round(N * K * 2 / us / 1e6, 2), "max_err": round(err, 4)})
                print(json.dumps(rows[-1]), flush=True)
        del ws
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
