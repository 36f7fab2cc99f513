#!/bin/bash
# 70B 1-GPU bench.py (driver defaults) N times back to back on the current tree.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in $(seq 1 ${RUNS:-2}); do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench70b_run$i.json 2> gpurun_out/r3_bench70b_run$i.err || { tail -20 gpurun_out/r3_bench70b_run$i.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/r3_bench70b_run$i.json'))
print('run $i', d['value'], d.get('ttft_p50_ms'), d.get('tpot_p50_ms'), d.get('mlp_table', '')[:300] if isinstance(d.get('mlp_table'), str) else d.get('mlp_table'))"
done
