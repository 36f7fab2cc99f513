#!/bin/bash
# Prefill attention: numerics (both tile sizes, tree mask) + microbench at the 70B head geometry.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill or tree" \
  > gpurun_out/r3_pa_tests.log 2>&1 || { tail -30 gpurun_out/r3_pa_tests.log; exit 1; }
tail -1 gpurun_out/r3_pa_tests.log
DGI_PREFILL_TILE=256 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill or tree" \
  > gpurun_out/r3_pa_tests256.log 2>&1 || { tail -30 gpurun_out/r3_pa_tests256.log; exit 1; }
tail -1 gpurun_out/r3_pa_tests256.log
ATTN_TILES=${ATTN_TILES:-128} ATTN_PREFILL_ONLY=1 timeout -k 10 200 python -u scripts/attn_bench.py > gpurun_out/attn_prefill.jsonl 2>&1 || { tail gpurun_out/attn_prefill.jsonl; exit 1; }
grep -v amdgpu.ids gpurun_out/attn_prefill.jsonl
