#!/bin/bash
# Round 4, session 3: decode-stage step in isolation (+ kernel profile), the two-source
# batched-receive RCCL test, and the 1-GPU 70B bench at several concurrencies / TPOT SLOs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step r4_two_src 200 python -u -m pytest tests/test_staged_gpu.py -m gpu -k "two_prefill or rccl_pd_on" -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
for r in 576 768 1024; do
  step r4_stage27_r$r 300 python -u scripts/decode_stage_prof.py --layers 27 --rows $r --out gpurun_out/r4_stage27.jsonl
done
export TMPDIR=/tmp
step r4_stage27_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_stage_prof -o run --output-format csv -- python3 scripts/decode_stage_prof.py --layers 27 --rows 768 --steps 20
for c in 384 416 448; do
  step r4_bench70b_c$c 600 python bench.py --steps 20 --warmup 5 --concurrency $c --json-out gpurun_out/r4_bench70b_c$c.json
done
for slo in 150 120; do
  step r4_bench70b_slo$slo 600 python bench.py --steps 20 --warmup 5 --tpot-slo-ms $slo --json-out gpurun_out/r4_bench70b_slo$slo.json
done
echo ALLDONE
