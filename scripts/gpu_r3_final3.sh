#!/bin/bash
# End-of-session check: decode-attention LDS-conflict PMC pass, 8B decode TPOT + kernel table
# with the quarter-pair qkv default, full GPU suite + smoke, 70B 1-GPU bench.  Large traces
# are deleted after summarising (gpurun_out <= 64 MiB).
set -o pipefail
mkdir -p gpurun_out/pmc_dec
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE \
  -d gpurun_out/pmc_dec -o run --output-format csv -- python3 scripts/decode_latency.py --batch 1 4 --steps 32 \
  > gpurun_out/pmc_dec.log 2>&1 || { tail -20 gpurun_out/pmc_dec.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_dec > gpurun_out/pmc_dec_summary.md || true
grep -i "decode" gpurun_out/pmc_dec_summary.md | head -10
rm -rf gpurun_out/pmc_dec
bash scripts/gpu_r3_decode_prof.sh || exit 1
rm -rf gpurun_out/prof_dec8b
bash scripts/gpu_r3_suite.sh || exit 1
RUNS=1 bash scripts/gpu_r3_bench70b.sh
