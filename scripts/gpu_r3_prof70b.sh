#!/bin/bash
# Kernel-time table of the 70B 1-GPU bench (mixed steps) + the 8B 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof70b_r3 -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 > gpurun_out/prof70b_r3.log 2>&1 || { tail -20 gpurun_out/prof70b_r3.log; exit 1; }
f=$(ls gpurun_out/prof70b_r3/*/run_kernel_stats.csv gpurun_out/prof70b_r3/run_kernel_stats.csv 2>/dev/null | head -1)
python3 scripts/prof_summary.py "$f" "Llama-3-70B 1-GPU bench.py mixed steps, round 3 (ping-pong MFMA GEMM + split-K in the start-up table)" > gpurun_out/prof70b_r3.md
head -30 gpurun_out/prof70b_r3.md
timeout -k 10 300 python3 bench.py --model llama3-8b > gpurun_out/r3_bench8b_s3.json 2> gpurun_out/r3_bench8b_s3.err || exit 1
cut -c1-400 gpurun_out/r3_bench8b_s3.json
