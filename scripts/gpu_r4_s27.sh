#!/bin/bash
# Round 4, session 27: batch-1 decode o-proj through the persistent fused GEMV (cfg 16): numerics, then
# same-box 8B decode TPOT A/B (DGI_OPROJ_FUSED=1 vs 0), interleaved.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "fused or model_decode or lookahead or graph_decode" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_s27_tests.log 2>&1 || { tail -30 gpurun_out/r4_s27_tests.log; exit 1; }
tail -2 gpurun_out/r4_s27_tests.log
D="scripts/decode_latency.py --batch 1 2 4 --steps 128"
for r in 1 2 3; do
  for v in 1 0; do
    DGI_OPROJ_FUSED=$v timeout -k 10 300 python -u $D --out gpurun_out/r4_declat_oproj${v}_$r.json > /dev/null || exit 1
  done
done
python3 - <<'PY'
import json
for r in (1, 2, 3):
    for v in (1, 0):
        rows = json.load(open(f"gpurun_out/r4_declat_oproj{v}_{r}.json"))
        print(f"oproj_fused={v} run{r}", " | ".join(f"b{x['batch']} {x['tpot_ms']:.3f}" for x in rows))
PY
echo ALLDONE
