#!/bin/bash
# Round 4, session 11: GPU suite, then the batch-1 Llama-3-8B decode step table (rocprofv3 kernel
# trace) with the decode lookahead and the fused split reduce on.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_s11_tests.log 2>&1 || { tail -40 gpurun_out/r4_s11_tests.log; exit 1; }
tail -3 gpurun_out/r4_s11_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec8b_r4 -o run --output-format csv -- \
  python3 scripts/decode_latency.py --batch 1 --steps 256 > gpurun_out/prof_dec8b_r4.log 2>&1 || { tail -20 gpurun_out/prof_dec8b_r4.log; exit 1; }
python3 scripts/decode_trace_layer.py gpurun_out/prof_dec8b_r4/run_kernel_trace.csv > gpurun_out/r4_decode_layer.md || true
cat gpurun_out/r4_decode_layer.md
rm -f gpurun_out/prof_dec8b_r4/run_kernel_trace.csv.gz
echo ALLDONE
