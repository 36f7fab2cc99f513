#!/bin/bash
# Decode attention merge-buffer swizzle: numerics, LDS-conflict PMC pass, TPOT + kernel table.
set -o pipefail
mkdir -p gpurun_out/pmc_dec
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "paged_decode or graph_decode or fused_decode or decode" \
  > gpurun_out/r3_dec_tests.log 2>&1 || { tail -30 gpurun_out/r3_dec_tests.log; exit 1; }
tail -2 gpurun_out/r3_dec_tests.log
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE \
  -d gpurun_out/pmc_dec -o run --output-format csv -- python3 scripts/decode_latency.py --batch 1 4 --steps 32 \
  > gpurun_out/pmc_dec.log 2>&1 || { tail -20 gpurun_out/pmc_dec.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_dec > gpurun_out/pmc_dec_summary.md || true
grep -i "decode" gpurun_out/pmc_dec_summary.md | head -10
bash scripts/gpu_r3_decode_prof.sh
