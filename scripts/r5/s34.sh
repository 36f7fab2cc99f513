#!/bin/bash
# Round 5, session 34: EAGLE-3 on the final tree (split sampler): batch 1 / 4, peaked target,
# self-distilled draft, tree width 3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s34
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
step spec_w3 900 python -u scripts/bench_spec.py --batch 1 4 --target peaked --train-steps 1500 --random-seqs 1024 \
  --oracle-accept --width 3 --out $O/spec_w3.json
echo ALLDONE
