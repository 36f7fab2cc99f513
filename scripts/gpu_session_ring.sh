#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mfma_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mfma_test3.log 2>&1 || { tail -30 gpurun_out/mfma_test3.log; exit 1; }
GEMM_MS=1792,2048,3072,4096 timeout -k 10 300 python -u scripts/mfma_gemm_bench.py 70b > gpurun_out/mfma_bench3_70b.jsonl 2> gpurun_out/mfma_bench3.err || exit 1
bash scripts/rehearse_rccl_bench.sh pd3_2p_1d pdpp4_2p_pp2 pd4_2p_2d
