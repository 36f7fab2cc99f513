#!/bin/bash
# Round 4, session 4: TPOT-SLO frontier of the 1-GPU 70B bench at matched concurrency.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
for cs in "256 0" "224 120" "256 120" "192 100" "224 100" "288 150"; do
  set -- $cs
  step r4_f70b_c$1_s$2 600 python bench.py --steps 20 --warmup 5 --concurrency $1 --tpot-slo-ms $2 --json-out gpurun_out/r4_f70b_c$1_s$2.json
done
echo ALLDONE
