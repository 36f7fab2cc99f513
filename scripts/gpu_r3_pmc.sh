#!/bin/bash
# PMC passes: ping-pong MFMA GEMM vs hipBLASLt on one 70B shape (PMC_SHAPE / PMC_M).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc1 gpurun_out/pmc2
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS \
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc1 -o run --output-format csv \
  -- python3 scripts/mfma_gemm_pmc.py > gpurun_out/pmc1.log 2>&1 || { tail -20 gpurun_out/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc2 -o run --output-format csv \
  -- python3 scripts/mfma_gemm_pmc.py > gpurun_out/pmc2.log 2>&1 || { tail -20 gpurun_out/pmc2.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc1 | tee gpurun_out/pmc1_summary.md
python3 scripts/pmc_summary.py gpurun_out/pmc2 | tee gpurun_out/pmc2_summary.md
