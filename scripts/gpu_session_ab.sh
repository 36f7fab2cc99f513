#!/bin/bash
# MFMA GEMM schedule A/B + 70B bench with and without the MFMA MLP kernels + RCCL bench rehearsal.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mfma_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mfma_test2.log 2>&1 || { tail -30 gpurun_out/mfma_test2.log; exit 1; }
GEMM_MS=1024,1792,2048,2560,3072,4096 timeout -k 10 300 python -u scripts/mfma_gemm_bench.py 70b > gpurun_out/mfma_bench2_70b.jsonl 2> gpurun_out/mfma_bench2.err || exit 1
DGI_MFMA_GEMM=0 timeout -k 10 240 python bench.py > gpurun_out/bench70b_blas.json 2> gpurun_out/bench70b_blas.err || exit 1
timeout -k 10 240 python bench.py > gpurun_out/bench70b_mfma.json 2> gpurun_out/bench70b_mfma.err || exit 1
bash scripts/rehearse_rccl_bench.sh
