#!/bin/bash
# Round 6, session 4: EAGLE-3 whole-step graph: numerics, then Llama-3-8B batch 1 / 4
# on the peaked target with the whole-step graph vs the staged draft / verify graphs (same draft),
# and a rocprof kernel trace of the whole-step loop at batch 1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s4
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-1500
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step spec_tests 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_spec.py
S="python -u scripts/bench_spec.py --batch 1 4 --target peaked --train-steps 1500 --random-seqs 1024 --oracle-accept --no-auto-off"
step spec_whole 600 $S --save-draft /tmp/draft_r6s4.pt --out $O/spec_whole.json
step spec_staged 400 $S --load-draft /tmp/draft_r6s4.pt --staged --out $O/spec_staged.json
step prof_whole 300 rocprofv3 --kernel-trace --stats -d $O/prof_whole -o run -- python3 scripts/bench_spec.py --batch 1 --target peaked --load-draft /tmp/draft_r6s4.pt --oracle-accept --no-auto-off --repeats 1 --output-len 64
rm -f /tmp/draft_r6s4.pt
echo ALLDONE
