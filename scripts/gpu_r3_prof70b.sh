#!/bin/bash
# Kernel-time table of the 70B 1-GPU bench: whole process (incl. the start-up GEMM table) and
# the steady-state mixed steps only (last 8 sampler-delimited steps of the trace).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof70b_r3 -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 > gpurun_out/prof70b_r3.log 2>&1 || { tail -20 gpurun_out/prof70b_r3.log; exit 1; }
f=$(ls gpurun_out/prof70b_r3/*/run_kernel_stats.csv gpurun_out/prof70b_r3/run_kernel_stats.csv 2>/dev/null | head -1)
python3 scripts/prof_summary.py "$f" "Llama-3-70B 1-GPU bench.py, whole process (start-up GEMM table included)" > gpurun_out/prof70b_r3.md
t=$(ls gpurun_out/prof70b_r3/*/run_kernel_trace.csv gpurun_out/prof70b_r3/run_kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/decode_trace_layer.py "$t" --steps 8 > gpurun_out/prof70b_r3_steps.md
head -40 gpurun_out/prof70b_r3_steps.md
rm -f "$t"
