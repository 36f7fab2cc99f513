#!/usr/bin/env python3
"""Short driver for rocprofv3 PMC passes: one 70B projection shape on the
hand-written MFMA kernel (schedule PMC_SCHED, default 3) and on hipBLASLt,
20 calls each.  PMC_SHAPE = gate_up (fused SwiGLU vs bare hipBLASLt GEMM) | o | qkv | down."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgi import ops  # noqa: E402

SHAPES = {"gate_up": (57344, 8192, 1), "o": (8192, 8192, 0), "qkv": (10240, 8192, 0), "down": (8192, 28672, 0)}
N, K, epi = SHAPES[os.environ.get("PMC_SHAPE", "gate_up")]
M = int(os.environ.get("PMC_M", "2048"))
sched = int(os.environ.get("PMC_SCHED", "3"))
ops.load_native(required=True)
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16) * 0.02
for _ in range(20):
    ops.mfma_gemm(x, w, epi, sched=sched)
for _ in range(20):
    F.linear(x, w)
torch.cuda.synchronize()
print("done")
