#!/bin/bash
# Round 4, session 26: decode attention tile loop as load / consume lambdas (and, first run, the 8-wave prefetch form): numerics, plan
# timings (new vs previous commit, same box), 8B decode TPOT A/B.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "paged_decode or model_decode or lookahead" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_s26_tests.log 2>&1 || { tail -30 gpurun_out/r4_s26_tests.log; exit 1; }
tail -2 gpurun_out/r4_s26_tests.log
A="scripts/decode_attn_b1.py --batch 1 4 --ctx 256 384 512 768 1024 2048"
timeout -k 10 300 python -u $A > gpurun_out/r4_attn_pf8_new.jsonl 2>> gpurun_out/r4_attn_pf8.err || exit 1
(cd _oldtree && timeout -k 10 300 python -u $A > ../gpurun_out/r4_attn_pf8_old.jsonl 2>> ../gpurun_out/r4_attn_pf8.err) || exit 1
D="scripts/decode_latency.py --batch 1 4 16 64 --steps 128"
for r in 1 2; do
  timeout -k 10 300 python -u $D --out gpurun_out/r4_declat_pf8_new_$r.json > /dev/null || exit 1
  (cd _oldtree && timeout -k 10 300 python -u $D --out ../gpurun_out/r4_declat_pf8_old_$r.json > /dev/null) || exit 1
done
python3 - <<'PY'
import json
for t in ("new", "old"):
    for l in open(f"gpurun_out/r4_attn_pf8_{t}.jsonl"):
        d = json.loads(l)
        print(t, d["batch"], d["ctx"], "one_split", d["one_split_us"], "split", d["split_reduce_us"])
for r in (1, 2):
    for t in ("new", "old"):
        rows = json.load(open(f"gpurun_out/r4_declat_pf8_{t}_{r}.json"))
        print(t, r, " | ".join(f"b{x['batch']} {x['tpot_ms']:.3f}" for x in rows))
PY
echo ALLDONE
