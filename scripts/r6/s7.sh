#!/bin/bash
# Round 6, session 7: where the fused-norm epilogues' time goes at decode-role and headline row
# counts (cold weights, graph-timed), with parts of the epilogues switched off.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s7
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step ng_full 300 python -u scripts/norm_gemm_bench.py
step ng_norstd 300 env DGI_NORM_GEMM_DBG=1 NG_M=512,2048 python -u scripts/norm_gemm_bench.py
step ng_nostats 300 env DGI_NORM_GEMM_DBG=2 NG_M=512,2048 python -u scripts/norm_gemm_bench.py
step ng_noresread 300 env DGI_NORM_GEMM_DBG=6 NG_M=512,2048 python -u scripts/norm_gemm_bench.py
echo ALLDONE
