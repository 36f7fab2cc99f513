#!/bin/bash
# Round 4, session 5: steady-state (60-step windows) of the TPOT-SLO configurations at the
# concurrency each SLO's row budget sustains, and the start-up probe at 4 / 8 layers.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
for cs in "384 0" "200 120" "270 150" "190 110"; do
  set -- $cs
  step r4_ss70b_c$1_s$2 600 python bench.py --steps 60 --warmup 10 --concurrency $1 --tpot-slo-ms $2 --json-out gpurun_out/r4_ss70b_c$1_s$2.json
done
step r4_probe70b_48 400 python -u -c "
import json, dataclasses
from dgi.parallel.probe import run_probe, capacity_from_probe, plan_from_probe
p = run_probe('llama3-70b', 'cuda:0')
c = capacity_from_probe(p)
print(json.dumps({'probe': p.to_dict(), 'capacity': dataclasses.asdict(c), 'plan8': plan_from_probe(8, c)}, default=str))
"
echo ALLDONE
