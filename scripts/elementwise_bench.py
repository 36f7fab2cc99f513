"""Bandwidth of the memory-bound dgi kernels (silu_mul, fused_add_rmsnorm, rmsnorm) at serving shapes."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from dgi import ops


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


for T in (64, 384, 1920, 4096):
    I, H = 28672, 8192
    gu = torch.randn(T, 2 * I, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(T, I, device="cuda", dtype=torch.bfloat16)
    us = timed(lambda: ops.silu_mul(gu, out=out))
    print(json.dumps({"kernel": "silu_mul", "T": T, "I": I, "us": round(us, 2), "TBs": round(3 * T * I * 2 / us / 1e6, 2)}))
    x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
    r = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(H, device="cuda", dtype=torch.bfloat16)
    us = timed(lambda: ops.fused_add_rmsnorm(x, r, w, 1e-5))
    print(json.dumps({"kernel": "fused_add_rmsnorm", "T": T, "H": H, "us": round(us, 2), "TBs": round(4 * T * H * 2 / us / 1e6, 2)}))
    us = timed(lambda: ops.rmsnorm(x, w, 1e-5))
    print(json.dumps({"kernel": "rmsnorm", "T": T, "H": H, "us": round(us, 2), "TBs": round(2 * T * H * 2 / us / 1e6, 2)}), flush=True)
