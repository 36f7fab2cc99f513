#!/usr/bin/env python3
"""Short driver for rocprofv3 PMC passes: the 70B gate_up shape at M = 2048 on
the fused MFMA SwiGLU kernel (schedule 1) and on hipBLASLt, 20 calls each."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgi import ops  # noqa: E402

M, N, K = int(os.environ.get("PMC_M", "2048")), 57344, 8192
ops.load_native(required=True)
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16) * 0.02
for _ in range(20):
    ops.mfma_gemm(x, w, 1, sched=1)
for _ in range(20):
    F.linear(x, w)
torch.cuda.synchronize()
print("done")
