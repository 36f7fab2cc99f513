#!/bin/bash
# Staged rehearsals of the multi-rank layouts on ONE GPU (all ranks share it,
# gloo data plane: tensors bounce through host memory).  Exercises every GPU
# code path of the P/D + replica + pipeline runtime; the RCCL transport itself
# only runs on a real multi-GPU node.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DGI_STAGED_GPU=1
run() {  # name timeout nproc args...
  local name=$1 to=$2 n=$3; shift 3
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
      --master-port $((29700 + RANDOM % 200)) bench.py --gpus "$n" --model llama3-8b "$@" \
      --json-out "gpurun_out/$name.json" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
COMMON="--steps 60 --warmup 5 --ramp-steps 30 --concurrency 64 --max-batched-tokens 2048 --output-len 64"
for s in ${STEPS:-pd4rep pdpp8}; do
  case $s in
    pd4rep) run staged_pd4rep 600 4 --layout pd --prefill-ranks 2 $COMMON ;;
    pdpp4) run staged_pdpp4 600 4 --layout pdpp --prefill-ranks 2 --decode-stages 2 $COMMON ;;
    pdpp6rep) run staged_pdpp6rep 600 6 --layout pdpp --prefill-ranks 2 --decode-stages 2 $COMMON ;;
    pdpp8) run staged_pdpp8 900 8 $COMMON ;;
    pd8rep) run staged_pd8rep 900 8 --layout pd $COMMON ;;
  esac
done
echo ALLDONE
