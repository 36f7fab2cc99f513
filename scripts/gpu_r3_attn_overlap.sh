#!/bin/bash
# 70B 1-GPU bench with the decode / prefill attention overlap on (default) and off; engine GPU tests.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "model or engine or fused or graph" \
  > gpurun_out/r3_overlap_tests.log 2>&1 || { tail -30 gpurun_out/r3_overlap_tests.log; exit 1; }
tail -1 gpurun_out/r3_overlap_tests.log
for v in 1 0 1; do
  DGI_ATTN_OVERLAP=$v timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench70b_ov$v.json 2> gpurun_out/r3_bench70b_ov$v.err || { tail -20 gpurun_out/r3_bench70b_ov$v.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/r3_bench70b_ov$v.json'))
print('overlap=$v', d['value'], d['ttft_p50_ms'], d['tpot_p50_ms'])"
done
