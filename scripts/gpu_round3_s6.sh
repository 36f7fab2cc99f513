# Round-3 session 6: numerics of the new fused / skinny launch configs (one-tile
# workgroups, deeper load rings), their kernel timings, the MALL prefetch probe,
# then 8B batch-1/4 TPOT with the promising configs.
set -o pipefail
if [ -n "$RUN_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "fused_skinny or skinny_gemm" > gpurun_out/r3_s6_tests.log 2>&1 || { tail -30 gpurun_out/r3_s6_tests.log; exit 1; }
fi
tail -2 gpurun_out/r3_s6_tests.log
timeout -k 10 300 python -u scripts/fused_decode_bench.py --cfgs 0 2 3 4 5 6 7 8 9 10 11 --skip-attn \
  --out gpurun_out/fdb_s6.json > gpurun_out/fdb_s6.log 2>&1 || { tail -20 gpurun_out/fdb_s6.log; exit 1; }
timeout -k 10 300 python -u scripts/fused_decode_bench.py --plain --out gpurun_out/fdb_plain_s6.json \
  > gpurun_out/fdb_plain_s6.log 2>&1 || { tail -20 gpurun_out/fdb_plain_s6.log; exit 1; }
timeout -k 10 200 python -u scripts/mall_probe.py > gpurun_out/mall_probe_s6.log 2>&1 || { tail -20 gpurun_out/mall_probe_s6.log; exit 1; }
cat gpurun_out/mall_probe_s6.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python scripts/decode_latency.py --batch 1 4 --prompt-len 256 --steps 64 \
    --out gpurun_out/s6_${tag}.json > gpurun_out/s6_${tag}.log 2>&1 || return 1
  python -c "import json; d=json.load(open('gpurun_out/s6_${tag}.json')); print('${tag}', [(r['batch'], r['tpot_ms']) for r in d])"
}
run base DGI_X=0 || exit 1
for c in 3 6 10; do run q$c DGI_FUSED_QKV_CFG=$c || exit 1; done
for c in 6 11 8; do run g$c DGI_FUSED_GU_CFG=$c || exit 1; done
run q6g6 DGI_FUSED_QKV_CFG=6 DGI_FUSED_GU_CFG=6 || exit 1
run q3g6 DGI_FUSED_QKV_CFG=3 DGI_FUSED_GU_CFG=6 || exit 1
for c in 7 8 11; do run s$c DGI_SKINNY_CFG=$c || exit 1; done
DGI_GPU_SPAN=1 timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench70_s6_span.json 2> gpurun_out/bench70_s6_span.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/bench70_s6_span.json')); print(d['value'], d['ms_per_step'], d['extra']['phases'])"
# open-loop P/D rehearsal (70B layer shapes, the N=8 auto layout) at ~90 % of its closed-loop request rate
REHEARSE_MODEL=llama3-70b@L8 REHEARSE_TAG=_open280 REHEARSE_STEPS=40 REHEARSE_WARMUP=20 REHEARSE_TIMEOUT=300 \
  REHEARSE_EXTRA="--arrival-rate 280 --decode-local-frac 0" bash scripts/rehearse_rccl_bench.sh auto8 || exit 1
python scripts/summarize_rehearsal.py gpurun_out/rehearse_auto8_open280.json 2>&1 | tail -5 || true
