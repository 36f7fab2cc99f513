#!/bin/bash
# Round 5, session 35: final-tree re-runs of the TPOT-SLO row (70B, SLO 120 ms) and the 8B
# continuous-batching throughput row.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s35
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
step slo120 700 python -u bench.py --steps 60 --warmup 10 --tpot-slo-ms 120 --json-out $O/slo120.json
step bench8b 600 python -u bench.py --model llama3-8b --concurrency 384 --steps 40 --warmup 10 --json-out $O/bench8b.json
echo ALLDONE
