#!/usr/bin/env python3
"""hipBLASLt (torch.nn.functional.linear) throughput for the Llama-3-70B/8B layer GEMMs at serving batch sizes."""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

SHAPES = {  # name: (N, K)
    "70b_qkv": (10240, 8192), "70b_o": (8192, 8192), "70b_gate_up": (57344, 8192), "70b_down": (8192, 28672),
    "8b_qkv": (6144, 4096), "8b_o": (4096, 4096), "8b_gate_up": (28672, 4096), "8b_down": (4096, 14336),
}
MS = [int(x) for x in os.environ.get("GEMM_MS", "64,256,512,1024,1280,2048,4096,8192").split(",")]


def bench(M, N, K, iters=20):
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    for _ in range(3):
        F.linear(x, w)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        F.linear(x, w)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    return dt * 1e6, 2 * M * N * K / dt / 1e12


def main():
    lib = os.environ.get("GEMM_LIB", "")
    if lib:   # "cublas" selects rocBLAS on ROCm, "cublaslt" hipBLASLt
        torch.backends.cuda.preferred_blas_library(lib)
    out = []
    for name, (N, K) in SHAPES.items():
        if len(sys.argv) > 1 and not name.startswith(sys.argv[1]):
            continue
        for M in MS:
            us, tf = bench(M, N, K)
            out.append({"gemm": name, "lib": lib or "default", "M": M, "N": N, "K": K, "us": round(us, 1),
                        "TFLOPs": round(tf, 1),
                        "weight_GBs": round(N * K * 2 / (us * 1e-6) / 1e9, 1)})
            print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
