#!/bin/bash
# Round 4, session 25: o-proj / down (no prologue/epilogue) through the fused_skinny persistent and
# quarter-pair configs vs ops.linear (skinny kernel / hipBLASLt), hipGraph-timed, cold weights.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u scripts/fused_decode_bench.py --cfgs 10 12 16 22 24 26 --skip-attn --plain-fused --out gpurun_out/r4_plain_fused.json > gpurun_out/r4_plain_fused.log 2>&1 || { tail -30 gpurun_out/r4_plain_fused.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r4_plain_fused.json'))
for k in ('plain_fused_8b',):
    for row in d.get(k, []): print(row)
"
echo ALLDONE
