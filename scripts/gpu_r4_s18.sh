#!/bin/bash
# Round 4, session 18: 5P + PP3 rehearsal (shared GPU, RCCL) at a load that keeps the prefill ranks busy
# (concurrency 768, 64 output tokens), to count prefill steps inside the 20-step window.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
export DGI_HANG_DUMP_S=250 REHEARSE_MODEL=llama3-70b@L8 REHEARSE_CONC=768 REHEARSE_STEPS=20 REHEARSE_WARMUP=5 REHEARSE_TIMEOUT=300
REHEARSE_TAG=_r4c768 bash scripts/rehearse_rccl_bench.sh pdpp8_5p_pp3 > gpurun_out/r4_reh_c768.log 2>&1 || { cat gpurun_out/r4_reh_c768.log; tail -30 gpurun_out/rehearse_pdpp8_5p_pp3_r4c768.err; exit 1; }
cat gpurun_out/r4_reh_c768.log
echo ALLDONE
