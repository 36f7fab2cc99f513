#!/bin/bash
# Persistent one-ring fused decode GEMV (cfg 12-16): numerics, per-config timing, batch-1 TPOT.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "fused_skinny" \
  > gpurun_out/r3_persist_tests.log 2>&1 || { tail -30 gpurun_out/r3_persist_tests.log; exit 1; }
tail -1 gpurun_out/r3_persist_tests.log
timeout -k 10 400 python -u scripts/fused_decode_bench.py --cfgs 6 7 8 10 11 12 13 14 15 16 --skip-attn \
  --out gpurun_out/r3_persist_cfgs.json > gpurun_out/r3_persist_bench.log 2>&1 || { tail -20 gpurun_out/r3_persist_bench.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r3_persist_cfgs.json'))
for r in d['gemm_8b']: print(json.dumps(r))"
for c in 12 13 14 15 16; do
  DGI_FUSED_GU_CFG=$c timeout -k 10 200 python -u scripts/decode_latency.py --batch 1 4 --steps 96 2>/dev/null | sed "s/^/gu_cfg=$c /"
done
timeout -k 10 200 python -u scripts/decode_latency.py --batch 1 4 --steps 96 2>/dev/null | sed "s/^/default /"
