#!/bin/bash
# Round 4, session 22: PMC pass over the batch-1 Llama-3-8B decode step (which kernels wait on memory,
# which are issue-bound).
set -o pipefail
mkdir -p gpurun_out/pmc_dec8b
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc_dec8b -o run --output-format csv \
  -- python3 scripts/decode_latency.py --batch 1 --steps 48 > gpurun_out/pmc_dec8b.log 2>&1 || { tail -20 gpurun_out/pmc_dec8b.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_dec8b > gpurun_out/pmc_dec8b_summary.md
head -30 gpurun_out/pmc_dec8b_summary.md
grep -E "fused_skinny|skinny_gemm|paged_decode|Cijk" gpurun_out/pmc_dec8b_summary.md | grep "^- " | head -12
rm -f gpurun_out/pmc_dec8b/run_counter_collection.csv
echo ALLDONE
