#!/bin/bash
# Debug session: RCCL batched receives from two sources on one shared GPU, three variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1 DGI_SHARED_GPU=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 DGI_WATCHDOG=0
for v in warm warmgroupsend; do
  echo "=== $v"
  VARIANT=$v NCCL_DEBUG=WARN timeout -k 5 60 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 \
    --master-port $((29700 + RANDOM % 100)) scripts/debug/rccl_batch_recv.py > gpurun_out/r4_dbg_$v.log 2>&1
  echo "rc=$?"; grep -E "rank|TIMEOUT|Error" gpurun_out/r4_dbg_$v.log | grep -v "^\[W" | head -12
done
echo ALLDONE
