#!/bin/bash
# Round 5, session 19: fused_skinny launch configs (split-K, persistent, quarter) on the 8B down and o
# against hipBLASLt (ops.linear) at M = 1, 4, 8.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s19
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
step downcfg 600 python -u scripts/fused_decode_bench.py --skip-gemms --skip-attn --plain-fused --cfgs 0 3 6 11 12 13 14 15 16 17 18 19 20 21 22 23 24 25 26 --out $O/plain_fused_cfgs.json
echo ALLDONE
