#!/bin/bash
# Round 6, session 13: smoke, the 1-GPU headline (twice) and the 512-row decode-role step with its
# kernel table, on the tree with the fused-norm layers on by default.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s13
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench70b_1 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench70b_1.json
step bench70b_2 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench70b_2.json
step dec80_512 400 python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512.jsonl
step prof_dec 300 rocprofv3 --kernel-trace --stats -d $O/prof_dec -o run -- python3 scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 10
step bench8b 600 python -u bench.py --model llama3-8b --steps 20 --warmup 5 --json-out $O/bench8b.json
echo ALLDONE
