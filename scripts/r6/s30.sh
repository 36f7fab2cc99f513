#!/bin/bash
# Round 6, session 30: GPU suite + smoke after the SSE stream decoder.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s30
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step gpu_suite 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
echo ALLDONE
