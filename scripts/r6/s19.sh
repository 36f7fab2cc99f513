#!/bin/bash
# Round 6, session 19: column-group stream-K for GEMMs whose last wave is more than half full
# (70B gate_up at 512 rows: 1.75 waves).  GEMM numerics / determinism, A/B (DGI_GEMM_GROUP_SK=0)
# of the fused-norm projections, the 512-row decode step and the 8B throughput config.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s19
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
NG_M=512 step ng_group 300 python -u scripts/norm_gemm_bench.py
DGI_GEMM_GROUP_SK=0 NG_M=512 step ng_nogroup 300 python -u scripts/norm_gemm_bench.py
step dec_group 400 python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512_group.jsonl
DGI_GEMM_GROUP_SK=0 step dec_nogroup 400 python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512_nogroup.jsonl
step b8_group 600 python -u bench.py --model llama3-8b --steps 20 --warmup 5 --json-out $O/bench8b_group.json
DGI_GEMM_GROUP_SK=0 step b8_nogroup 600 python -u bench.py --model llama3-8b --steps 20 --warmup 5 --json-out $O/bench8b_nogroup.json
DGI_GEMM_MAX_SPLITS=8 step b8_split8 600 python -u bench.py --model llama3-8b --steps 20 --warmup 5 --json-out $O/bench8b_split8.json
echo ALLDONE
