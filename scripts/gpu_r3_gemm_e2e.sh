#!/bin/bash
# Round 3: GEMM tests + per-shape bench + 70B 1-GPU bench.py with the ping-pong / split-K kernel in the start-up table.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mfma_gemm.py \
  > gpurun_out/r3_gemm_tests.log 2>&1 || { tail -30 gpurun_out/r3_gemm_tests.log; exit 1; }
tail -2 gpurun_out/r3_gemm_tests.log
GEMM_SCHEDS=3,3k,1 GEMM_MS=1024,1792,1920,2048,2432,4096 timeout -k 10 400 \
  python -u scripts/mfma_gemm_bench.py 70b > gpurun_out/r3_gemm_bench.jsonl 2>&1 || exit 1
cut -c1-300 gpurun_out/r3_gemm_bench.jsonl
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench70b_s3.json 2> gpurun_out/r3_bench70b_s3.err || { tail -20 gpurun_out/r3_bench70b_s3.err; exit 1; }
cat gpurun_out/r3_bench70b_s3.json
