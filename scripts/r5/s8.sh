#!/bin/bash
# Round 5, session 8: prefill attention double-buffered LDS (tests + A/B at 70B heads), full GPU suite
# (fused layers now take <= 16-row prefill / tree-verify steps), SLO-120 with the running-set admission
# limit, EAGLE-3 tree width 3 (16 nodes: fused verify) vs 4 (21 nodes), and a kernel trace of the spec step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s8
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-900
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
step prefill_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "paged_prefill"
step attn_ab 300 env ATTN_PREFILL_ONLY=1 ATTN_TILES=128,256 ATTN_DB=0,1 python -u scripts/attn_bench.py
soft=1 step suite 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
step slo120 600 python -u bench.py --steps 60 --warmup 10 --tpot-slo-ms 120 --json-out $O/slo120.json
step spec_w3 900 python -u scripts/bench_spec.py --batch 1 4 --target peaked --train-steps 1500 --random-seqs 1024 \
  --oracle-accept --width 3 --save-draft /tmp/draft8b.pt --out $O/spec_w3.json
step spec_w4 600 python -u scripts/bench_spec.py --batch 1 4 --target peaked --oracle-accept --width 4 \
  --load-draft /tmp/draft8b.pt --out $O/spec_w4.json
step spec_w3_unfused 600 env DGI_FUSED_SMALL_PREFILL=0 python -u scripts/bench_spec.py --batch 1 --target peaked \
  --oracle-accept --width 3 --load-draft /tmp/draft8b.pt --out $O/spec_w3_unfused.json
step spec_trace 600 rocprofv3 --kernel-trace --stats -d $O/prof_spec -o run -- python3 -u scripts/bench_spec.py \
  --batch 1 --target peaked --oracle-accept --width 3 --repeats 1 --load-draft /tmp/draft8b.pt
echo ALLDONE
