#!/usr/bin/env python3
"""Hand-written MFMA GEMM (dgi/csrc/mfma_gemm.hip) vs hipBLASLt on the Llama-3
layer GEMMs at prefill / mixed-step row counts.

For gate_up the comparison is the whole MLP front half: hipBLASLt GEMM +
the separate silu_mul pass vs the kernel's fused SwiGLU epilogue (epi 1).
Variants are timed in interleaved rounds in one process on the same random
operands (uniform [-1, 1) activations, 0.02-scaled weights), median of the
rounds; one JSON line per (shape, M).

  python scripts/mfma_gemm_bench.py [shape-prefix]      GEMM_MS=1024,2048 ...
"""
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgi import ops  # noqa: E402

SHAPES = {  # name: (N, K)
    "70b_qkv": (10240, 8192), "70b_o": (8192, 8192), "70b_gate_up": (57344, 8192), "70b_down": (8192, 28672),
    "8b_qkv": (6144, 4096), "8b_o": (4096, 4096), "8b_gate_up": (28672, 4096), "8b_down": (4096, 14336),
}
MS = [int(x) for x in os.environ.get("GEMM_MS", "512,1024,1536,1792,2048,4096").split(",")]
ROUNDS = int(os.environ.get("GEMM_ROUNDS", "7"))
ITERS = int(os.environ.get("GEMM_ITERS", "10"))
# schedule ids; "3k" = schedule 3 with split-K off, "3p1" / "3p2" = schedule 3 with s_setprio variant 1 / 2,
# "3h" / "3f" = schedule 3 with two 32-MFMA / four 16-MFMA phases per K tile (default: by M),
# "3n" = schedule 3 without the cross-tile prologue / epilogue overlap
SCHEDS = os.environ.get("GEMM_SCHEDS", "1,0,2,3").split(",")


def timed(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(ITERS):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / ITERS


def main():
    ops.load_native(required=True)
    for name, (N, K) in SHAPES.items():
        if len(sys.argv) > 1 and not name.startswith(sys.argv[1]):
            continue
        w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16) * 0.02
        for M in MS:
            x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
            fused = name.endswith("gate_up")
            epi = 1 if fused else 0
            variants = {"hipblaslt+silu_mul": lambda: ops.silu_mul(F.linear(x, w))} if fused else \
                {"hipblaslt": lambda: F.linear(x, w)}
            for sc in SCHEDS:
                variants[("mfma_swiglu" if fused else "mfma") + ("" if sc == SCHEDS[0] else f"_s{sc}")] = \
                    (lambda sc=sc: ops.mfma_gemm(x, w, epi, sched=int(sc[0]), streamk=int("k" in sc),
                                                 prio=int(sc.split("p")[1][0]) if "p" in sc else 0,
                                                 phases=2 if "h" in sc else 4 if "f" in sc else 0,
                                                 overlap="n" not in sc))
            for f in variants.values():
                f()
            torch.cuda.synchronize()
            times = {k: [] for k in variants}
            for _ in range(ROUNDS):
                for k, f in variants.items():
                    times[k].append(timed(f))
            row = {"gemm": name, "M": M, "N": N, "K": K}
            flops = 2 * M * N * K
            for k, v in times.items():
                us = statistics.median(v)
                row[k + "_us"] = round(us, 1)
                row[k + "_TFLOPs"] = round(flops / (us * 1e-6) / 1e12, 1)
            base = "hipblaslt+silu_mul" if fused else "hipblaslt"
            mine = "mfma_swiglu" if fused else "mfma"
            row["speedup"] = round(row[base + "_us"] / row[mine + "_us"], 3)
            print(json.dumps(row), flush=True)
            del x
        del w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
