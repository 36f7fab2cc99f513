#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof70b_r2s2 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --ramp-steps 16 > gpurun_out/prof70b_r2s2.log 2>&1 || exit 1
f=$(ls gpurun_out/prof70b_r2s2/*/run_kernel_stats.csv gpurun_out/prof70b_r2s2/run_kernel_stats.csv 2>/dev/null | head -1)
python3 scripts/prof_summary.py "$f" "Llama-3-70B 1-GPU bench.py mixed steps, round 2 session 2" > gpurun_out/prof70b_r2s2.md
timeout -k 10 300 python3 bench.py --model llama3-8b > gpurun_out/bench8b_r2s2.json 2> gpurun_out/bench8b_r2s2.err || exit 1
