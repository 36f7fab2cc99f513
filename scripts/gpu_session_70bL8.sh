#!/bin/bash
mkdir -p gpurun_out
REHEARSE_MODEL=llama3-70b@L8 REHEARSE_CONC=256 REHEARSE_TAG=_70bL8 bash scripts/rehearse_rccl_bench.sh pdpp4_2p_pp2 pdpp8_5p_pp3 pd3_2p_1d || exit 1
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_gemm -o run -- python3 scripts/mfma_gemm_pmc.py > gpurun_out/pmc_gemm.log 2>&1 || exit 1
python3 scripts/pmc_summary.py gpurun_out/pmc_gemm > gpurun_out/pmc_gemm.md 2>&1
