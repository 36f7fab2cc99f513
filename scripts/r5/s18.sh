#!/bin/bash
# Round 5, session 18: 8-wave decode attention with Q issued after the first tile's K/V loads:
# numerics, the small-batch latency table (compare profiles/r4_decode/attn_b1_plans.jsonl), 8B TPOT.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s18
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
step tests 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "paged_decode or decode or lookahead"
step attn_b1 300 python -u scripts/decode_attn_b1.py
step declat8b 600 python -u scripts/decode_latency.py --batch 1 4 16 --out $O/declat8b.json
step profdec 600 rocprofv3 --kernel-trace --stats -d $O/profdec -o run -- python3 -u scripts/decode_latency.py --batch 1 --steps 200
echo ALLDONE
