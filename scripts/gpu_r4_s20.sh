#!/bin/bash
# Round 4, session 20: PMC passes on the small-batch decode attention (b = 1, ctx 2048: eight tiles per wave
# in the one-split kernel) — where the ~2.5 us per tile goes.
set -o pipefail
mkdir -p gpurun_out/pmc_attn1 gpurun_out/pmc_attn2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_attn1 -o run --output-format csv \
  -- python3 scripts/decode_attn_b1.py --batch 1 --ctx 2048 --chain 4 > gpurun_out/pmc_attn1.log 2>&1 || { tail -20 gpurun_out/pmc_attn1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES \
  SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_attn2 -o run --output-format csv \
  -- python3 scripts/decode_attn_b1.py --batch 1 --ctx 2048 --chain 4 > gpurun_out/pmc_attn2.log 2>&1 || { tail -20 gpurun_out/pmc_attn2.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_attn1 | tee gpurun_out/pmc_attn1_summary.md
python3 scripts/pmc_summary.py gpurun_out/pmc_attn2 | tee gpurun_out/pmc_attn2_summary.md
echo ALLDONE
