#!/bin/bash
# Round 5, session 6: long-K decode GEMV on the skinny kernel vs hipBLASLt (8B down / o-proj); the TPOT-SLO
# row with admission coupling (SLO 120 ms, closed loop); a kernel trace of the 1-GPU 70B headline step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s6
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-700
  [ $rc -eq 0 ] || exit $rc
}
step rccl_log 120 env DGI_SHARED_GPU=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 DGI_WATCHDOG=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29655 scripts/rccl_log_probe.py
ls -la /tmp/dgi_rccl_* > $O/rccl_files.txt 2>&1; head -c 20000 /tmp/dgi_rccl_29655_0.log > $O/rccl_rank0_log.txt 2>/dev/null
step skinny_longk 300 python -u scripts/skinny_longk_bench.py
step slo120 600 python -u bench.py --steps 60 --warmup 10 --tpot-slo-ms 120 --json-out $O/slo120.json
step slo150 600 python -u bench.py --steps 60 --warmup 10 --tpot-slo-ms 150 --json-out $O/slo150.json
step trace70b 600 rocprofv3 --kernel-trace --stats -d $O/prof70b -o run -- python3 -u bench.py --steps 12 --warmup 3
echo ALLDONE
