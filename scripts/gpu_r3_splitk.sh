#!/bin/bash
# Split-K fused decode configs: numerics, qkv/gate_up microbench, then the full suite + smoke.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "fused_skinny" > gpurun_out/r3_splitk_tests.log 2>&1 || { tail -30 gpurun_out/r3_splitk_tests.log; exit 1; }
tail -2 gpurun_out/r3_splitk_tests.log
timeout -k 10 300 python -u scripts/fused_decode_bench.py --cfgs 6 7 10 17 18 19 20 21 --skip-attn --plain-fused \
  --out gpurun_out/r3_splitk_bench.json > gpurun_out/r3_splitk_bench.log 2>&1 || { tail -30 gpurun_out/r3_splitk_bench.log; exit 1; }
tail -30 gpurun_out/r3_splitk_bench.log
