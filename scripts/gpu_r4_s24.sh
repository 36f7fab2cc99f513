#!/bin/bash
# Round 4, session 24: fused decode GEMV loops without per-group integer divisions (cursor walk): numerics,
# then same-box 8B decode TPOT A/B against the previous commit (_oldtree) and a kernel trace of the new step.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "fused or model_decode or lookahead" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_s24_tests.log 2>&1 || { tail -30 gpurun_out/r4_s24_tests.log; exit 1; }
tail -2 gpurun_out/r4_s24_tests.log
D="scripts/decode_latency.py --batch 1 4 16 64 --steps 128"
for r in 1 2; do
  timeout -k 10 300 python -u $D --out gpurun_out/r4_declat_cur_new_$r.json > /dev/null || exit 1
  (cd _oldtree && timeout -k 10 300 python -u $D --out ../gpurun_out/r4_declat_cur_old_$r.json > /dev/null) || exit 1
done
python3 - <<'PY'
import json
for r in (1, 2):
    for t in ("new", "old"):
        rows = json.load(open(f"gpurun_out/r4_declat_cur_{t}_{r}.json"))
        print(t, r, " | ".join(f"b{x['batch']} {x['tpot_ms']:.3f}" for x in rows))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec8b_cur -o run --output-format csv -- \
  python3 scripts/decode_latency.py --batch 1 --steps 256 > gpurun_out/prof_dec8b_cur.log 2>&1 || { tail -20 gpurun_out/prof_dec8b_cur.log; exit 1; }
python3 scripts/decode_trace_layer.py gpurun_out/prof_dec8b_cur/run_kernel_trace.csv > gpurun_out/r4_decode_layer_cur.md || true
cat gpurun_out/r4_decode_layer_cur.md
rm -f gpurun_out/prof_dec8b_cur/run_kernel_trace.csv
echo ALLDONE
