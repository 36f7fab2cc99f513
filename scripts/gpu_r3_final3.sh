#!/bin/bash
# End-of-session check: 8B decode TPOT + kernel table with the quarter-pair qkv default,
# full GPU suite + smoke.  Large traces are deleted after summarising (gpurun_out <= 64 MiB).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash scripts/gpu_r3_decode_prof.sh || exit 1
rm -rf gpurun_out/prof_dec8b
bash scripts/gpu_r3_suite.sh
