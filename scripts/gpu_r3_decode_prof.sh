#!/bin/bash
# Batch-1 Llama-3-8B decode: TPOT and per-kernel table (rocprofv3 kernel trace).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u scripts/decode_latency.py --batch 1 4 --steps 128 > gpurun_out/r3_decode_tpot.jsonl 2> gpurun_out/r3_decode_tpot.err || { tail -20 gpurun_out/r3_decode_tpot.err; exit 1; }
cat gpurun_out/r3_decode_tpot.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec8b -o run --output-format csv -- \
  python3 scripts/decode_latency.py --batch 1 --steps 256 > gpurun_out/prof_dec8b.log 2>&1 || { tail -20 gpurun_out/prof_dec8b.log; exit 1; }
python3 scripts/decode_trace_layer.py gpurun_out/prof_dec8b/run_kernel_trace.csv > gpurun_out/r3_decode_layer.md || true
cat gpurun_out/r3_decode_layer.md
