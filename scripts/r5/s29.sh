#!/bin/bash
# Round 5, session 29: full-depth decode steps the planner now prices from the probe: a whole-model
# 70B decode GPU at 512 rows (80 layers) and a 2-stage replica's stage at 768 rows (40 layers),
# graph-replayed at 576 tokens of context.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s29
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
step dec80_512 500 python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512.json
step dec40_768 500 python -u scripts/decode_stage_prof.py --layers 40 --rows 768 --ctx 576 --steps 30 --out $O/dec40_768.json
echo ALLDONE
