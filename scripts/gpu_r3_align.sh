#!/bin/bash
# 70B 1-GPU bench with tile-aligned mixed steps (default) vs --token-align 0.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench70b_align.json 2> gpurun_out/r3_bench70b_align.err || { tail -20 gpurun_out/r3_bench70b_align.err; exit 1; }
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --token-align 0 > gpurun_out/r3_bench70b_noalign.json 2> gpurun_out/r3_bench70b_noalign.err || { tail -20 gpurun_out/r3_bench70b_noalign.err; exit 1; }
for f in align noalign; do python3 -c "
import json,sys;d=json.load(open('gpurun_out/r3_bench70b_$f.json'))
print('$f', d['value'], d['ttft_p50_ms'], d['ttft_p95_ms'], d['tpot_p50_ms'], d['extra']['engine'])"; done
