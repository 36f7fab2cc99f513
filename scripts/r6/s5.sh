#!/bin/bash
# Round 6, session 5: multi-rank rehearsals on one GPU (DGI_SHARED_GPU=1, real RCCL data plane over
# loopback) of what the driver's scaling run launches — --layout auto at 2 and 8 ranks — on the
# round-6 tree (fused-norm layers on the prefill / mixed steps, async host tier), 70B layer shapes
# truncated to 8 layers, 512-in / 128-out.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s5
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then exit $rc; fi
}
export REHEARSE_MODEL=llama3-70b@L8 REHEARSE_CONC=0 REHEARSE_STEPS=20 REHEARSE_WARMUP=3 REHEARSE_TIMEOUT=420 \
  DGI_HANG_DUMP_S=400 REHEARSE_TAG=_r6s5 REHEARSE_EXTRA="--prompt-len 512 --output-len 128"
step rehearse_auto2 460 bash scripts/rehearse_rccl_bench.sh auto2
step rehearse_auto8 460 bash scripts/rehearse_rccl_bench.sh auto8
cp gpurun_out/rehearse_auto2_r6s5.json gpurun_out/rehearse_auto2_r6s5.err gpurun_out/rehearse_auto8_r6s5.json gpurun_out/rehearse_auto8_r6s5.err $O/ 2>/dev/null
echo ALLDONE
