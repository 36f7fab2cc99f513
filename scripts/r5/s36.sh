#!/bin/bash
# Round 5, session 36: the 1-GPU headline three times on one box, final tree (run-to-run spread).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s36
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
for r in 1 2 3; do
  step bench70b_$r 500 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench70b_$r.json
done
echo ALLDONE
