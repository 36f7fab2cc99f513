#!/bin/bash
# Round 5, session 7: RCCL transport log check (2 shared-GPU ranks); TPOT-SLO rows with the load-shape prior;
# EAGLE-3 with a 32k draft vocabulary vs the full one (8B, peaked target, batch 1 / 4).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s7
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-900
  [ $rc -eq 0 ] || exit $rc
}
step rccl_log 120 env DGI_SHARED_GPU=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 DGI_WATCHDOG=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29655 scripts/rccl_log_probe.py
step slo120 600 python -u bench.py --steps 60 --warmup 10 --tpot-slo-ms 120 --json-out $O/slo120.json
step spec_v32k 900 python -u scripts/bench_spec.py --batch 1 4 --target peaked --train-steps 1500 --random-seqs 1024 --oracle-accept --draft-vocab 32768 --out $O/spec_v32k.json
step spec_full 900 python -u scripts/bench_spec.py --batch 1 4 --target peaked --train-steps 1500 --random-seqs 1024 --oracle-accept --out $O/spec_full.json
echo ALLDONE
