#!/bin/bash
# Round 6, session 18: split-K pieces with the last arrival's partial kept in registers (mfma_gemm.hip
# drive()): GEMM numerics / determinism tests, the split probe again, the 512-row decode step, the
# 1-GPU headline.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s18
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-500
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step gemm_tests 400 python -u -m pytest tests/test_mfma_gemm.py -q -m gpu --timeout 120 --timeout-method thread
step pp_split 300 python -u scripts/pp_split_probe.py
cp $O/pp_split.log $O/pp_split.jsonl
step dec80_512 400 python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512.jsonl
step bench70b 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench70b.json
echo ALLDONE
