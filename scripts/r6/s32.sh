#!/bin/bash
# Round 6, session 32: fused qkv (RMSNorm prologue + RoPE/KV epilogue) at 9-16 rows (spec verify,
# batch-16 decode) against the unfused chain, across the fused GEMV launch configs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s32
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 400 python -u scripts/fused_decode_bench.py --skip-attn --gemm-ms 8 12 16 --cfgs 7 13 15 22 23 26 --out $O/fused_qkv_m16.json > $O/fused.log 2>&1
rc=$?
echo "=== fused rc=$rc"; grep '^{' $O/fused.log | cut -c1-600; grep -i "skip" $O/fused.log | head -5
exit $rc
