#!/bin/bash
# Round 4, session 8: 8-rank RCCL rehearsals (one GPU, DGI_SHARED_GPU=1) of 5P+PP3 and 2P+6D with the
# batched per-source KV receives (default) vs one receive in flight (DGI_KV_RECV_BATCH=1), at the
# driver's --steps 20 --warmup 5 (node step sized from the prefill ranks' measured step time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DGI_HANG_DUMP_S=200
export REHEARSE_MODEL=llama3-70b@L8 REHEARSE_CONC=256 REHEARSE_STEPS=20 REHEARSE_WARMUP=5 REHEARSE_TIMEOUT=280
REHEARSE_TAG=_r4batch bash scripts/rehearse_rccl_bench.sh pdpp8_5p_pp3 pd8_2p_6d > gpurun_out/r4_reh_batch.log 2>&1 || { cat gpurun_out/r4_reh_batch.log; exit 1; }
DGI_KV_RECV_BATCH=1 REHEARSE_TAG=_r4serial bash scripts/rehearse_rccl_bench.sh pdpp8_5p_pp3 pd8_2p_6d > gpurun_out/r4_reh_serial.log 2>&1 || { cat gpurun_out/r4_reh_serial.log; exit 1; }
cat gpurun_out/r4_reh_batch.log gpurun_out/r4_reh_serial.log
echo ALLDONE
