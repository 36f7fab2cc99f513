#!/bin/bash
# Multi-rank bench.py on ONE GPU with a real RCCL data plane (DGI_SHARED_GPU=1:
# per-rank NCCL_HOSTID, RCCL network transport over loopback).  Exercises the
# 8-GPU code path's RCCL ordering (pair set-up, KV migration, stage hops) at
# small scale before the driver runs it on a whole node.  Llama-3-8B, short run.
set -o pipefail
mkdir -p gpurun_out
export DGI_SHARED_GPU=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 DGI_HANG_DUMP_S=360
run() {  # name, nproc, extra args
  local name=$1 n=$2; shift 2
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus "$n" --model llama3-8b --steps 8 --warmup 2 --ramp-steps 4 \
    --concurrency 64 --output-len 32 --prompt-len 256 "$@" > "gpurun_out/rehearse_${name}.json" 2> "gpurun_out/rehearse_${name}.err"
}
run pdpp4_1p_pp3 4 --layout pdpp --prefill-ranks 1 --decode-stages 3 || exit 1
run pd4_2p_2d 4 --layout pd --prefill-ranks 2 --decode-replicas 2 || exit 1
