#!/bin/bash
# Round 3: ping-pong MFMA GEMM (sched 3) numerics + timing vs sched 1 and hipBLASLt, 70B shapes.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mfma_gemm.py \
  > gpurun_out/r3_gemm_tests.log 2>&1 || { tail -30 gpurun_out/r3_gemm_tests.log; exit 1; }
tail -3 gpurun_out/r3_gemm_tests.log
GEMM_SCHEDS=${GEMM_SCHEDS:-3,3k,1} GEMM_MS=${GEMM_MS:-1024,1920,2048,4096} timeout -k 10 400 \
  python -u scripts/mfma_gemm_bench.py ${1:-70b} 2>&1 | tee gpurun_out/r3_gemm_bench.jsonl
