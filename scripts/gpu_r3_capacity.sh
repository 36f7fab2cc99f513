#!/bin/bash
# Per-role capacity (70B) on the round-3 tree (ping-pong GEMM + split-K, tile-aligned steps).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 700 python3 scripts/pd_capacity.py --model llama3-70b --mbt 2048 --decode 40:768,40:1024,80:576,27:768 \
  > gpurun_out/r3_pd_capacity_70b_gemm.jsonl 2> gpurun_out/r3_pd_capacity_70b_gemm.err || { tail -20 gpurun_out/r3_pd_capacity_70b_gemm.err; exit 1; }
cut -c1-300 gpurun_out/r3_pd_capacity_70b_gemm.jsonl
