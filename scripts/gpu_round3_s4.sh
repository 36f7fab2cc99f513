# Round-3 GPU session 4: GPU suite (incl. the RCCL tensor-parallel test), the 8-GPU auto layout's
# rehearsal with the capacity check, open-loop 70B 1-GPU latency at steady state.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gpu_suite_s4.log 2>&1 || { tail -30 gpurun_out/r3_gpu_suite_s4.log; exit 1; }
tail -2 gpurun_out/r3_gpu_suite_s4.log
REHEARSE_MODEL=llama3-70b@L8 REHEARSE_CONC=256 REHEARSE_TAG=_70bL8_r3s4 DGI_HANG_DUMP_S=170 \
  bash scripts/rehearse_rccl_bench.sh auto8 > gpurun_out/rehearse_auto_s4.log 2>&1 || { cat gpurun_out/rehearse_auto_s4.log; exit 1; }
for rate in 12.4 13.1; do
  timeout -k 10 500 python bench.py --steps 120 --warmup 250 --arrival-rate $rate > gpurun_out/bench70_open_${rate}_s4.json 2> gpurun_out/bench70_open_${rate}_s4.err || exit 1
done
