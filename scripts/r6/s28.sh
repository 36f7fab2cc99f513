#!/bin/bash
# Round 6, session 28: the served path with long-poll + batch claims (next-jobs): GPU E2E test,
# then single_worker --backend all on Llama-3-8B at the worker's default 2 s poll interval.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s28
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step e2e_test 400 python -u -m pytest tests/test_worker_daemon.py -v -m gpu --timeout 300 --timeout-method thread
step e2e_8b 700 python -u benchmarks/single_worker.py --backend all --launch --model llama3-8b --num-requests 64 --concurrent 8 --max-tokens 128 --prompt-length 128 --steps 40 --warmup 5 --poll-interval 2.0 --output $O/e2e_8b_batchclaim.json
echo ALLDONE
