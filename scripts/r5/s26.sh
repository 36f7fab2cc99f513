#!/bin/bash
# Round 5, session 26: kernel trace of the 8B batch-1 decode step with the split-row sampler
# (per-kernel time of sample_part_kernel + sample_final_kernel vs sample_kernel's 15.5 us).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s26
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
step profdec 600 rocprofv3 --kernel-trace --stats -d $O/profdec -o run -- python3 -u scripts/decode_latency.py --batch 1 --steps 200
echo ALLDONE
