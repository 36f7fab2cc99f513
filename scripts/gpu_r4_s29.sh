#!/bin/bash
# Round 4, session 29: EAGLE-3 speculative decoding on the final tree (Llama-3-8B, peaked random-init target,
# self-distilled draft; greedy, batch 1 / 4 / 16; oracle-acceptance controller points).
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u scripts/bench_spec.py --batch 1 4 16 --target peaked --train-steps 1500 --random-seqs 1024 \
  --oracle-accept 0.6 1.0 --out gpurun_out/r4_spec8b.json > gpurun_out/r4_spec8b.log 2>&1 || { tail -30 gpurun_out/r4_spec8b.log; exit 1; }
tail -30 gpurun_out/r4_spec8b.log
echo ALLDONE
