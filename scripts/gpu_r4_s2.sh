#!/bin/bash
# Round 4, session 2: new GPU tests, the start-up capacity probe on the real 70B shapes,
# and the 8-rank RCCL rehearsal of the P/D layouts after the head-of-line fix + timestamp window.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step r4_pytest_new 300 python -u -m pytest tests/test_host_tier.py tests/test_staged_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
step r4_probe70b 400 python -u -c "
import json, time, dataclasses
from dgi.parallel.probe import run_probe, capacity_from_probe, plan_from_probe
from dgi.parallel.plan import CAPACITY
p = run_probe('llama3-70b', 'cuda:0')
c = capacity_from_probe(p)
print(json.dumps({'probe': p.to_dict(), 'capacity': dataclasses.asdict(c), 'table': dataclasses.asdict(CAPACITY['llama3-70b']),
                  'plan8': plan_from_probe(8, c), 'plan8_table': plan_from_probe(8, CAPACITY['llama3-70b'])}, default=str))
"
cp gpurun_out/r4_probe70b.log gpurun_out/r4_probe70b.json
export DGI_HANG_DUMP_S=200
REHEARSE_MODEL=llama3-70b@L8 REHEARSE_CONC=256 REHEARSE_STEPS=20 REHEARSE_WARMUP=5 REHEARSE_TIMEOUT=280 REHEARSE_TAG=_r4 \
  bash scripts/rehearse_rccl_bench.sh pdpp8_5p_pp3 pdpp8_6p_pp2 > gpurun_out/r4_rehearse.log 2>&1
rc=$?; cat gpurun_out/r4_rehearse.log; exit $rc
