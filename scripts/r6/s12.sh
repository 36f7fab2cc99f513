#!/bin/bash
# Round 6, session 12: determinism probe of the mixed-step lookahead test (fold on / off), then the
# GPU suite, smoke, the headline and the 512-row decode step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s12
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step probe_fold 200 python -u scripts/r6/lookahead_check.py
step probe_nofold 200 env DGI_NORM_FOLD=0 python -u scripts/r6/lookahead_check.py
step gpu_suite 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
echo ALLDONE
