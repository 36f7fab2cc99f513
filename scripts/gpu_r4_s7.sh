#!/bin/bash
# Round 4, session 7: Llama-3-8B batch-1/4 decode as it stands (TPOT, per-kernel step table,
# LDS bank-conflict PMC pass over the decode kernels).
set -o pipefail
mkdir -p gpurun_out/pmc_dec
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 python -u scripts/decode_latency.py --batch 1 4 --steps 128 > gpurun_out/r4_decode_tpot.jsonl 2> gpurun_out/r4_decode_tpot.err || { tail -20 gpurun_out/r4_decode_tpot.err; exit 1; }
cat gpurun_out/r4_decode_tpot.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec8b -o run --output-format csv -- \
  python3 scripts/decode_latency.py --batch 1 --steps 256 > gpurun_out/prof_dec8b.log 2>&1 || { tail -20 gpurun_out/prof_dec8b.log; exit 1; }
python3 scripts/decode_trace_layer.py gpurun_out/prof_dec8b/run_kernel_trace.csv > gpurun_out/r4_decode_layer.md || true
cat gpurun_out/r4_decode_layer.md
rm -rf gpurun_out/prof_dec8b
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE \
  -d gpurun_out/pmc_dec -o run --output-format csv -- python3 scripts/decode_latency.py --batch 1 4 --steps 32 \
  > gpurun_out/pmc_dec.log 2>&1 || { tail -20 gpurun_out/pmc_dec.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_dec > gpurun_out/r4_pmc_dec_summary.md || true
cat gpurun_out/r4_pmc_dec_summary.md | head -30
rm -rf gpurun_out/pmc_dec
echo ALLDONE
