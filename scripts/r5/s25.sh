#!/bin/bash
# Round 5, session 25: split-row sampler (small batches over 8192-logit workgroups): numerics
# against the one-workgroup-per-row kernel, 8B TPOT with and without it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s25
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
step tests 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "sample or topk or lookahead or spec"
step declat8b_split 600 python -u scripts/decode_latency.py --batch 1 4 16 --out $O/declat8b_split.json
DGI_SAMPLE_SPLIT=0 step declat8b_nosplit 600 python -u scripts/decode_latency.py --batch 1 4 16 --out $O/declat8b_nosplit.json
step declat8b_split2 600 python -u scripts/decode_latency.py --batch 1 4 16 --out $O/declat8b_split2.json
echo ALLDONE
