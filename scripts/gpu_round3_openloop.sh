# Round-3 GPU session: the auto layouts the driver's scaling run launches (70B shapes on one GPU,
# RCCL rehearsal) and open-loop 70B 1-GPU latency at 80 / 90 % of the closed-loop capacity.
set -o pipefail
REHEARSE_MODEL=llama3-70b@L8 REHEARSE_CONC=256 REHEARSE_TAG=_70bL8_r3 DGI_HANG_DUMP_S=170 \
  bash scripts/rehearse_rccl_bench.sh auto8 auto4 auto2 > gpurun_out/rehearse_auto.log 2>&1 || { cat gpurun_out/rehearse_auto.log; exit 1; }
cat gpurun_out/rehearse_auto.log
for rate in 12.4 11.0; do
  timeout -k 10 400 python bench.py --steps 60 --warmup 10 --arrival-rate $rate > gpurun_out/bench70_open_${rate}.json 2> gpurun_out/bench70_open_${rate}.err || exit 1
  tail -c 400 gpurun_out/bench70_open_${rate}.json
done
