#!/bin/bash
# Round 5, session 24: 8-rank shared-GPU RCCL rehearsal of --layout auto (now 6 prefill + 2
# whole-model decode GPUs at 512-row microbatches) at the 512/128 headline load.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s24
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
export REHEARSE_MODEL=llama3-70b@L8 REHEARSE_CONC=0 REHEARSE_STEPS=20 REHEARSE_WARMUP=3 REHEARSE_TIMEOUT=600 \
  DGI_HANG_DUMP_S=560 REHEARSE_TAG=_r5s24 REHEARSE_EXTRA="--prompt-len 512 --output-len 128"
step rehearse_auto8 640 bash scripts/rehearse_rccl_bench.sh auto8
cp gpurun_out/rehearse_auto8_r5s24.json gpurun_out/rehearse_auto8_r5s24.err $O/ 2>/dev/null
echo ALLDONE
