#!/bin/bash
# Round 4, session 9: in-kernel split reduce of the paged decode attention (write-through partials,
# one acquire on the last arriver) — numerics, then 8B decode TPOT with it on / off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_s9_tests.log 2>&1 || { tail -30 gpurun_out/r4_s9_tests.log; exit 1; }
tail -3 gpurun_out/r4_s9_tests.log
timeout -k 10 300 python -u -m pytest tests/test_staged_gpu.py -m gpu -k "receive_batch or two_prefill" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_s9_rccl.log 2>&1 || { tail -30 gpurun_out/r4_s9_rccl.log; exit 1; }
tail -3 gpurun_out/r4_s9_rccl.log
timeout -k 10 300 python -u scripts/decode_latency.py --batch 1 4 16 64 --steps 128 --out gpurun_out/r4_declat_fused.json || exit 1
DGI_DECODE_FUSED_REDUCE=0 timeout -k 10 300 python -u scripts/decode_latency.py --batch 1 4 16 64 --steps 128 --out gpurun_out/r4_declat_kernel.json || exit 1
DGI_DECODE_SHORT_CTX=0 timeout -k 10 300 python -u scripts/decode_latency.py --batch 1 4 16 64 --steps 128 --out gpurun_out/r4_declat_fused_noshort.json || exit 1
timeout -k 10 300 python -u scripts/decode_latency.py --batch 1 4 16 64 --steps 128 --out gpurun_out/r4_declat_fused2.json || exit 1
echo ALLDONE
