mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mfma_gemm.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mfma_test.log 2>&1 || { echo MFMA_TEST_FAILED; tail -30 gpurun_out/mfma_test.log; exit 1; }
timeout -k 10 300 python -u scripts/mfma_gemm_bench.py 70b > gpurun_out/mfma_bench_70b.jsonl 2> gpurun_out/mfma_bench.err || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "not rccl and not mfma" > gpurun_out/gputest_r2s2.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r2s2.log 2>&1 || exit 1
timeout -k 10 240 python bench.py > gpurun_out/bench70b_r2s2.json 2> gpurun_out/bench70b_r2s2.err || exit 1
timeout -k 10 400 python -u -m pytest tests/test_staged_gpu.py -x -v --timeout 180 --timeout-method thread -k rccl > gpurun_out/rccl_shared_r2s2.log 2>&1
