# 8B batch-1 decode TPOT across the fused (qkv / gate_up) and skinny (o-proj) launch configs.
set -o pipefail
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python scripts/decode_latency.py --batch 1 4 --prompt-len 256 --steps 64 \
    --out gpurun_out/sweep_${tag}.json > gpurun_out/sweep_${tag}.log 2>&1 || return 1
  python -c "import json; d=json.load(open('gpurun_out/sweep_${tag}.json')); print('${tag}', [(r['batch'], r['tpot_ms']) for r in d])"
}
run base DGI_X=0 || exit 1
for c in 0 2 3 5; do run fq$c DGI_FUSED_CFG=$c || exit 1; done
for c in 1 2 3 5 6; do run sk$c DGI_SKINNY_CFG=$c || exit 1; done
