#!/bin/bash
# Multi-rank bench.py on ONE GPU with a real RCCL data plane (DGI_SHARED_GPU=1:
# per-rank NCCL_HOSTID, RCCL network transport over loopback).  Exercises the
# 8-GPU code path's RCCL ordering (pair set-up, KV migration, stage hops) at
# small scale before the driver runs it on a whole node.  Llama-3-8B, short run.
# A rank still running after DGI_HANG_DUMP_S seconds dumps every thread's
# Python stack to the .err file and exits.
# usage: rehearse_rccl_bench.sh [case ...]   (default: all cases)
# env: REHEARSE_MODEL, REHEARSE_CONC, REHEARSE_STEPS / _WARMUP, REHEARSE_TIMEOUT, REHEARSE_TAG,
#      REHEARSE_EXTRA (appended bench.py flags, e.g. "--arrival-rate 280" for an open-loop run)
set -o pipefail
mkdir -p gpurun_out
export DGI_SHARED_GPU=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 DGI_HANG_DUMP_S=${DGI_HANG_DUMP_S:-100}
MODEL=${REHEARSE_MODEL:-llama3-8b}
CONC=${REHEARSE_CONC:-64}
run() {  # name, nproc, extra args
  local name=$1 n=$2; shift 2
  echo "== $name ($MODEL)" >&2
  timeout -k 10 ${REHEARSE_TIMEOUT:-200} python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus "$n" --model "$MODEL" --steps ${REHEARSE_STEPS:-8} --warmup ${REHEARSE_WARMUP:-2} --ramp-steps 4 \
    --concurrency "$CONC" --output-len 32 --prompt-len 256 "$@" $REHEARSE_EXTRA > "gpurun_out/rehearse_${name}${REHEARSE_TAG}.json" \
    2> "gpurun_out/rehearse_${name}${REHEARSE_TAG}.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  return $rc
}
cases=${*:-"pdpp4_1p_pp3 pdpp4_2p_pp2 pd4_2p_2d pd3_2p_1d pdpp8_5p_pp3"}
for c in $cases; do
  case $c in
    pdpp4_1p_pp3) run $c 4 --layout pdpp --prefill-ranks 1 --decode-stages 3 || exit 1 ;;
    pdpp4_2p_pp2) run $c 4 --layout pdpp --prefill-ranks 2 --decode-stages 2 || exit 1 ;;
    pd4_2p_2d) run $c 4 --layout pd --prefill-ranks 2 --decode-replicas 2 || exit 1 ;;
    pd3_2p_1d) run $c 3 --layout pd --prefill-ranks 2 --decode-replicas 1 || exit 1 ;;
    pdpp8_5p_pp3) run $c 8 --layout pdpp --prefill-ranks 5 --decode-stages 3 || exit 1 ;;
    pd8_5p_3d) run $c 8 --layout pd --prefill-ranks 5 --decode-replicas 3 || exit 1 ;;
    pd8_5p_3d_nooverflow) run $c 8 --layout pd --prefill-ranks 5 --decode-replicas 3 --prefill-local-cap 0 || exit 1 ;;
    pd8_2p_6d) run $c 8 --layout pd --prefill-ranks 2 --decode-replicas 6 || exit 1 ;;
    auto2) run $c 2 || exit 1 ;;         # what the driver's scaling run launches: the planner's layout
    dp2) run $c 2 --layout dp || exit 1 ;;
    dp4) run $c 4 --layout dp || exit 1 ;;
    auto4) run $c 4 || exit 1 ;;
    auto8) run $c 8 || exit 1 ;;
    pp8) run $c 8 --layout pp || exit 1 ;;
    pp4) run $c 4 --layout pp || exit 1 ;;
    pdpp8_6p_pp2) run $c 8 --layout pdpp --prefill-ranks 6 --decode-stages 2 || exit 1 ;;
    pdpp8_2p_2xpp3) run $c 8 --layout pdpp --prefill-ranks 2 --decode-stages 3 --decode-replicas 2 || exit 1 ;;
    pd4_3p_1d) run $c 4 --layout pd --prefill-ranks 3 --decode-replicas 1 || exit 1 ;;
    pd2_1p_1d_local) run $c 2 --layout pd --prefill-ranks 1 --decode-replicas 1 --decode-local-frac 0.46 || exit 1 ;;
    pdpp4_2p_pp2_local) run $c 4 --layout pdpp --prefill-ranks 2 --decode-stages 2 --decode-local-frac 0.5 || exit 1 ;;
    pdpp8_5p_pp3_local) run $c 8 --layout pdpp --prefill-ranks 5 --decode-stages 3 --decode-local-frac 0.2 || exit 1 ;;
  esac
done
