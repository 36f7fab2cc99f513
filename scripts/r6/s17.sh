#!/bin/bash
# Round 6, session 17: the whole-step spec graph after the vectorized metadata fill (GPU spec tests),
# the split-K probe of qkv / o at decode-role rows, EAGLE-3 with a draft vocabulary on a target
# whose outputs concentrate on 32k ids.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s17
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-500
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step spec_tests 400 python -u -m pytest tests/test_spec.py -v -m gpu --timeout 200 --timeout-method thread
step pp_split 300 python -u scripts/pp_split_probe.py
cp $O/pp_split.log $O/pp_split.jsonl
step spec_conc 900 python -u scripts/bench_spec.py --batch 1 4 --target concentrated --train-steps 1500 --random-seqs 1024 --oracle-accept --no-auto-off --out $O/spec_concentrated.json
echo ALLDONE
