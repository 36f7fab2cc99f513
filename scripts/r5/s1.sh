#!/bin/bash
# Round 5, session 1: baseline on a fresh box — graph-branch concurrency probe, decode-stage step at 768 rows
# (plain and under a kernel trace), and the 1-GPU headline bench.
set -o pipefail
mkdir -p gpurun_out/r5s1
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r5s1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
step overlap384 120 python -u scripts/graph_overlap_probe.py --rows 384
step overlap768 120 python -u scripts/graph_overlap_probe.py --rows 768 --copy-mb 2048
step stage768 300 python -u scripts/decode_stage_prof.py --rows 768
step stage768_trace 300 rocprofv3 --kernel-trace --stats -d $O/prof_stage -o run -- python3 -u scripts/decode_stage_prof.py --rows 768 --steps 20
step bench70b 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench70b.json
echo ALLDONE
