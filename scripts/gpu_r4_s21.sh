#!/bin/bash
# Round 4, session 21: same-box A/B of the decode attention page16 load path (scalar page bases for full
# tiles) — 8B decode TPOT and 70B-head attention at batch 384 / 768, interleaved runs.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "paged_decode or model_decode or lookahead" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_s21_tests.log 2>&1 || { tail -30 gpurun_out/r4_s21_tests.log; exit 1; }
tail -2 gpurun_out/r4_s21_tests.log
D="scripts/decode_latency.py --batch 1 4 16 64 --steps 128"
for r in 1 2; do
  for p in 1 0; do
    DGI_DECODE_PAGE16=$p timeout -k 10 300 python -u $D --out gpurun_out/r4_declat_p16_${p}_$r.json > /dev/null || exit 1
  done
done
for p in 1 0; do
  DGI_DECODE_PAGE16=$p timeout -k 10 200 python -u scripts/decode_attn_b1.py --heads 64 8 --batch 384 768 --ctx 576 --chain 8 > gpurun_out/r4_attn70b_p16_$p.jsonl 2>> gpurun_out/r4_attn_p16.err || exit 1
  DGI_DECODE_PAGE16=$p timeout -k 10 200 python -u scripts/decode_attn_b1.py --batch 1 --ctx 384 512 1024 > gpurun_out/r4_attn8b_p16_$p.jsonl 2>> gpurun_out/r4_attn_p16.err || exit 1
done
python3 - <<'PY'
import json
for r in (1, 2):
    for p in (1, 0):
        rows = json.load(open(f"gpurun_out/r4_declat_p16_{p}_{r}.json"))
        print(f"page16={p} run{r}", " | ".join(f"b{x['batch']} {x['tpot_ms']:.3f}" for x in rows))
for p in (1, 0):
    for f in (f"gpurun_out/r4_attn70b_p16_{p}.jsonl", f"gpurun_out/r4_attn8b_p16_{p}.jsonl"):
        for l in open(f):
            d = json.loads(l)
            print(f"page16={p}", d["batch"], d["ctx"], d["one_split_us"], d["split_reduce_us"])
PY
echo ALLDONE
