#!/bin/bash
# GEMM tests + A/B of schedule-3 variants (GEMM_SCHEDS) on the 70B shapes.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mfma_gemm.py \
  > gpurun_out/r3_gemm_tests.log 2>&1 || { tail -30 gpurun_out/r3_gemm_tests.log; exit 1; }
tail -2 gpurun_out/r3_gemm_tests.log
GEMM_SCHEDS=${GEMM_SCHEDS:-3,3h,3hp1,3hp2} GEMM_MS=${GEMM_MS:-1792,2048,4096} GEMM_ROUNDS=9 timeout -k 10 300 \
  python -u scripts/mfma_gemm_bench.py ${1:-70b} > gpurun_out/r3_gemm_ab.jsonl 2>&1 || { tail -20 gpurun_out/r3_gemm_ab.jsonl; exit 1; }
cut -c1-500 gpurun_out/r3_gemm_ab.jsonl
