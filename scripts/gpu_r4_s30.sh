#!/bin/bash
# Round 4, session 30 (final tree): start-up probe + 8-GPU plan for Llama-3-70B, then the TPOT-SLO frontier
# (60-step windows) at the default, 150 ms and 120 ms budgets.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step r4f_probe70b 400 python -u -c "
import json, dataclasses
from dgi.parallel.probe import run_probe, capacity_from_probe, plan_from_probe
p = run_probe('llama3-70b', 'cuda:0')
c = capacity_from_probe(p)
print(json.dumps({'probe': p.to_dict(), 'capacity': dataclasses.asdict(c), 'plan8': plan_from_probe(8, c), 'plan8_ratio1': plan_from_probe(8, c, min_ratio=1.0)}, default=str))
"
for cs in "384 0" "270 150" "200 120"; do
  set -- $cs
  step r4f_ss70b_c$1_s$2 600 python bench.py --steps 60 --warmup 10 --concurrency $1 --tpot-slo-ms $2 --json-out gpurun_out/r4f_ss70b_c$1_s$2.json
done
echo ALLDONE
