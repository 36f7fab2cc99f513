"""TunableOp sweep for the serving GEMM shapes that recur exactly every step.

Prefill ranks always run full ``max_num_batched_tokens`` chunks (M = 4096 or
8192) and decode microbatches run at bucketed M, so a per-shape tuned
solution is reused on every step.  Writes the TunableOp CSV (validated
against this PyTorch / HIP / hipBLASLt build) and prints default vs tuned
timings.

    PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 \
    PYTORCH_TUNABLEOP_FILENAME=profiles/tunableop_mi355x.csv python scripts/gemm_tune.py 70b 4096,8192
"""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

SHAPES = {
    "70b_qkv": (10240, 8192), "70b_o": (8192, 8192), "70b_gate_up": (57344, 8192), "70b_down": (8192, 28672),
    "8b_qkv": (6144, 4096), "8b_o": (4096, 4096), "8b_gate_up": (28672, 4096), "8b_down": (4096, 14336),
}


def timeit(x, w, iters=20):
    for _ in range(3):
        F.linear(x, w)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        F.linear(x, w)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    prefix = sys.argv[1] if len(sys.argv) > 1 else "70b"
    ms = [int(m) for m in (sys.argv[2] if len(sys.argv) > 2 else "4096,8192").split(",")]
    import torch.cuda.tunable as tun
    out = []
    for name, (N, K) in SHAPES.items():
        if not name.startswith(prefix):
            continue
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        for M in ms:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            tun.enable(False)
            base = timeit(x, w)
            tun.enable(True)
            tun.tuning_enable(True)
            F.linear(x, w)                      # tunes this shape once
            tun.tuning_enable(False)
            tuned = timeit(x, w)
            r = {"gemm": name, "M": M, "N": N, "K": K, "default_us": round(base, 1), "tuned_us": round(tuned, 1),
                 "gain": round(base / tuned, 3), "tuned_TFLOPs": round(2 * M * N * K / tuned / 1e6, 1)}
            out.append(r)
            print(json.dumps(r), flush=True)
    tun.write_file()
    print("wrote", tun.get_filename())


if __name__ == "__main__":
    main()
