#!/bin/bash
# Round 4, session 14: 8-rank RCCL rehearsals (shared GPU) with receive batches capped at 2
# sources, with and without batched sends (compare: session 12's r4b / r4s / r4bb).
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
export DGI_HANG_DUMP_S=200 REHEARSE_MODEL=llama3-70b@L8 REHEARSE_CONC=256 REHEARSE_STEPS=20 REHEARSE_WARMUP=5 REHEARSE_TIMEOUT=280
DGI_KV_RECV_BATCH=2 REHEARSE_TAG=_r4b2 bash scripts/rehearse_rccl_bench.sh pdpp8_5p_pp3 pd8_2p_6d > gpurun_out/r4_reh_b2.log 2>&1 || { cat gpurun_out/r4_reh_b2.log; exit 1; }
DGI_KV_RECV_BATCH=2 DGI_BATCH_P2P=1 REHEARSE_TAG=_r4b2bb bash scripts/rehearse_rccl_bench.sh pdpp8_5p_pp3 pd8_2p_6d > gpurun_out/r4_reh_b2bb.log 2>&1 || { cat gpurun_out/r4_reh_b2bb.log; exit 1; }
DGI_KV_RECV_BATCH=1 DGI_BATCH_P2P=1 REHEARSE_TAG=_r4sbb bash scripts/rehearse_rccl_bench.sh pdpp8_5p_pp3 > gpurun_out/r4_reh_sbb.log 2>&1 || { cat gpurun_out/r4_reh_sbb.log; exit 1; }
cat gpurun_out/r4_reh_b2.log gpurun_out/r4_reh_b2bb.log gpurun_out/r4_reh_sbb.log
echo ALLDONE
