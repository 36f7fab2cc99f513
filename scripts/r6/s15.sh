#!/bin/bash
# Round 6, session 15: kernel table of the Llama-3-8B 1-GPU throughput config (concurrency 384),
# fused-norm layers on (default) and off.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s15
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step prof8b 400 rocprofv3 --kernel-trace --stats -d $O/prof8b -o run -- python3 bench.py --model llama3-8b --steps 10 --warmup 4 --json-out $O/prof8b_bench.json
step bench8b_fold 400 python -u bench.py --model llama3-8b --steps 20 --warmup 5 --json-out $O/bench8b_fold.json
step bench8b_nofold 400 env DGI_NORM_FOLD=0 python -u bench.py --model llama3-8b --steps 20 --warmup 5 --json-out $O/bench8b_nofold.json
echo ALLDONE
