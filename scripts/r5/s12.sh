#!/bin/bash
# Round 5, session 12: longest-first prefill tile order (A/B), full GPU suite on the current tree,
# headline bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s12
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-900
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
step attn_order 300 env ATTN_PREFILL_ONLY=1 ATTN_TILE_ORDER=0 python -u scripts/attn_bench.py
step attn_lpt 300 env ATTN_PREFILL_ONLY=1 ATTN_TILE_ORDER=1 python -u scripts/attn_bench.py
soft=1 step suite 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
step bench70b 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench70b.json
echo ALLDONE
