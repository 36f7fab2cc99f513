#!/bin/bash
# Round 5, session 3: two-batch overlap (CU-masked streams) — correctness tests, 27-layer 70B stage step A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
soft=1 step tests 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "two_batch or decode_proj or lookahead"
step g1_768 300 python -u scripts/decode_stage_prof.py --rows 768 --graphs 1
step e0_768 300 env DGI_TBO=0 python -u scripts/decode_stage_prof.py --rows 768 --graphs 0
step t4_768 300 env DGI_TBO=1 DGI_TBO_SIDE=4 python -u scripts/decode_stage_prof.py --rows 768 --graphs 0
step t3_768 300 env DGI_TBO=1 DGI_TBO_SIDE=3 python -u scripts/decode_stage_prof.py --rows 768 --graphs 0
step t6_768 300 env DGI_TBO=1 DGI_TBO_SIDE=6 python -u scripts/decode_stage_prof.py --rows 768 --graphs 0
step t4_1024 300 env DGI_TBO=1 DGI_TBO_SIDE=4 python -u scripts/decode_stage_prof.py --rows 1024 --graphs 0
step e0_1024 300 env DGI_TBO=0 python -u scripts/decode_stage_prof.py --rows 1024 --graphs 0
step t4_768_trace 300 rocprofv3 --kernel-trace --stats -d $O/prof_t4 -o run -- python3 -u scripts/decode_stage_prof.py --rows 768 --graphs 0 --steps 20
step gemm_table 400 python -u scripts/gemm_table_build.py --passes 3 --out gpurun_out/r5s3/gemm_table_70b.json
echo ALLDONE
