#!/bin/bash
# Quarter-pair persistent decode GEMV: numerics + qkv/gate_up microbench; then the attention swizzle check.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "fused_skinny" > gpurun_out/r3_quarter_tests.log 2>&1 || { tail -30 gpurun_out/r3_quarter_tests.log; exit 1; }
tail -2 gpurun_out/r3_quarter_tests.log
timeout -k 10 300 python -u scripts/fused_decode_bench.py --cfgs 6 7 10 12 16 22 23 24 25 26 --skip-attn \
  --out gpurun_out/r3_quarter_bench.json > gpurun_out/r3_quarter_bench.log 2>&1 || { tail -30 gpurun_out/r3_quarter_bench.log; exit 1; }
grep '^{' gpurun_out/r3_quarter_bench.log
bash scripts/gpu_r3_attn_swz.sh
