#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/decode_latency.py --batch 1 4 16 64 > gpurun_out/declat_s2.json 2> gpurun_out/declat_s2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec1_s2 -o run --output-format csv -- python3 scripts/decode_latency.py --batch 1 --steps 128 > gpurun_out/prof_dec1_s2.log 2>&1 || exit 1
f=$(ls gpurun_out/prof_dec1_s2/run_kernel_stats.csv gpurun_out/prof_dec1_s2/*/run_kernel_stats.csv 2>/dev/null | head -1)
python3 scripts/prof_summary.py "$f" "Llama-3-8B decode, batch 1" > gpurun_out/prof_dec1_s2.md
