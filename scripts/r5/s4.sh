#!/bin/bash
# Round 5, session 4: shipped GEMM routing table (3 passes, median), start-up probe of the 70B roles
# (prefill at 2048 and 1024 tokens / step) and the 8-GPU plan under it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s4
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}

step probe70b 400 python -u -c "
import json, dataclasses
from dgi.parallel.probe import run_probe, capacity_from_probe, plan_from_probe
p = run_probe('llama3-70b', 'cuda:0')
c = capacity_from_probe(p)
print(json.dumps({'probe': p.to_dict(), 'capacity': dataclasses.asdict(c), 'plan8': plan_from_probe(8, c), 'plan4': plan_from_probe(4, c), 'plan2': plan_from_probe(2, c)}, default=str))
"
echo ALLDONE
