#!/bin/bash
# Decode attention numerics + batch-1/4 TPOT + per-step kernel table.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "paged_decode or graph_decode or fused_decode" \
  > gpurun_out/r3_dec_tests.log 2>&1 || { tail -30 gpurun_out/r3_dec_tests.log; exit 1; }
tail -2 gpurun_out/r3_dec_tests.log
bash scripts/gpu_r3_decode_prof.sh
