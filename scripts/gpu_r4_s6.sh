#!/bin/bash
# Round 4, session 6: 70B 1-GPU steps pinned to 2048 rows (max_batched_tokens 2048: every mixed
# step a whole number of 256-row tiles with gate_up at exactly 7 waves) at the concurrencies whose
# steady state fills them.
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
for cm in "400 2048" "416 2048" "384 2048" "448 2304"; do
  set -- $cm
  step r4_mbt70b_c$1_m$2 600 python bench.py --steps 60 --warmup 10 --concurrency $1 --max-batched-tokens $2 --json-out gpurun_out/r4_mbt70b_c$1_m$2.json
done
echo ALLDONE
