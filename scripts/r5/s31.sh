#!/bin/bash
# Round 5, session 31: 128 x 128 half-tile MFMA GEMM (sched 4): numerics, then 70B qkv / o at
# 256-1024 rows against hipBLASLt and the ping-pong 256 x 256 schedule.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s31
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
step tests 300 python -u -m pytest tests/test_mfma_gemm.py -x -q --timeout 120 --timeout-method thread -k "half_tile or strided"
step bench 400 python -u scripts/half_tile_bench.py
echo ALLDONE
