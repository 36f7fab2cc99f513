#!/bin/bash
# Round 6, session 23: the start-up probe once more on a fresh box with the final tree (second box for
# the P/D pick).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s23
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for r in 1; do
step probe70b_$r 400 python -u -c "
import dataclasses, json
from dgi.parallel.probe import run_probe, capacity_from_probe, plan_from_probe
p = run_probe('llama3-70b', 'cuda:0', decode_rows=(512, 768), prefill_more=(1024,))
c = capacity_from_probe(p)
print(json.dumps({'probe': p.to_dict(), 'capacity': dataclasses.asdict(c), 'plan8': plan_from_probe(8, c),
                  'plan4': plan_from_probe(4, c), 'plan2': plan_from_probe(2, c)}, default=str))
"
done
echo ALLDONE
