#!/bin/bash
# Round 5, session 13: HIP token-slot KV compaction, one D2H sync per verify, width-3 default (tests + spec bench + step
# trace), and the 1-GPU headline with mixed-step lookahead back off (TTFT).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s13
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-900
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
step tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_spec.py -x -q --timeout 120 --timeout-method thread -k "topk or sample or spec or verify or draft or slot"
step spec_w3 900 python -u scripts/bench_spec.py --batch 1 4 --target peaked --train-steps 1500 --random-seqs 1024 \
  --oracle-accept --width 3 --save-draft /tmp/draft8b.pt --out $O/spec_w3.json
step spec_trace 600 rocprofv3 --kernel-trace --stats -d $O/prof_spec -o run -- python3 -u scripts/bench_spec.py \
  --batch 1 --target peaked --oracle-accept --width 3 --repeats 1 --load-draft /tmp/draft8b.pt
echo ALLDONE
