#!/bin/bash
# Round 6, session 25: plain projections at the spec verify / batch-16 decode row counts (8B o, down,
# qkv at M = 8-16) through the persistent fused GEMV configs vs ops.linear (skinny / hipBLASLt).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s25
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 400 python -u scripts/fused_decode_bench.py --skip-attn --skip-gemms --plain-fused --plain-fused-qkv --plain-fused-ms 8 12 16 --cfgs 6 12 13 15 16 22 23 24 --out $O/plain_fused_m16.json > $O/plain_fused.log 2>&1
rc=$?
echo "=== plain_fused rc=$rc"; tail -12 $O/plain_fused.log | cut -c1-400
exit $rc
