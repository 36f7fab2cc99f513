#!/bin/bash
# (1) decode: fused/graph GPU tests + TPOT at batch 1/4/8/16 with the persistent gate_up defaults;
# (2) 70B mixed steps: attention overlap A/B.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "fused or graph or model or engine" \
  > gpurun_out/r3_combo_tests.log 2>&1 || { tail -30 gpurun_out/r3_combo_tests.log; exit 1; }
tail -1 gpurun_out/r3_combo_tests.log
timeout -k 10 300 python -u scripts/decode_latency.py --batch 1 4 8 16 --steps 96 --out gpurun_out/r3_decode_tpot_persist.json 2>/dev/null || exit 1
for v in 1 0; do
  DGI_ATTN_OVERLAP=$v timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench70b_ov$v.json 2> gpurun_out/r3_bench70b_ov$v.err || { tail -20 gpurun_out/r3_bench70b_ov$v.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/r3_bench70b_ov$v.json'))
print('overlap=$v', d['value'], d['ttft_p50_ms'], d['tpot_p50_ms'])"
done
