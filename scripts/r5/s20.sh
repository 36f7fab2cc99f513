#!/bin/bash
# Round 5, session 20: warming the MALL beside batch-1 decode attention (scripts/mall_prefetch_probe.py)
# o-proj and gate_up after a forked prefetch vs cold.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s20
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
step probe 500 python -u scripts/mall_prefetch_probe.py --out $O/mall_prefetch_probe.json
echo ALLDONE
