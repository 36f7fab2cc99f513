#!/bin/bash
# Round 5, session 30: kernel trace of the whole-model 70B decode step at 512 rows (the decode role of
# the 8-GPU plan), 80 layers, 576 tokens of context, graph replay.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s30
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
step prof80_512 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 10
echo ALLDONE
