#!/bin/bash
# Round 4, session 13: decode attention latency form (block ids in registers + next tile in flight):
# numerics, graph-chained micro-bench per pipe mode, large-batch check, 8B TPOT per mode.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "paged_decode or decode_lookahead or model_decode" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_s13_tests.log 2>&1 || { tail -40 gpurun_out/r4_s13_tests.log; exit 1; }
tail -2 gpurun_out/r4_s13_tests.log
timeout -k 10 300 python -u scripts/decode_attn_b1.py --modes 0 1 2 > gpurun_out/r4_attn_pipe.jsonl 2> gpurun_out/r4_attn_pipe.err || { tail -20 gpurun_out/r4_attn_pipe.err; exit 1; }
cat gpurun_out/r4_attn_pipe.jsonl
timeout -k 10 200 python -u scripts/decode_attn_b1.py --heads 64 8 --batch 384 --ctx 576 --modes 0 3 --chain 8 > gpurun_out/r4_attn_pipe70b.jsonl 2>> gpurun_out/r4_attn_pipe.err || { tail -20 gpurun_out/r4_attn_pipe.err; exit 1; }
cat gpurun_out/r4_attn_pipe70b.jsonl
D="scripts/decode_latency.py --batch 1 4 16 64 --steps 128"
DGI_DECODE_PIPE=2 timeout -k 10 300 python -u $D --out gpurun_out/r4_declat_pipe2.json > /dev/null || exit 1
DGI_DECODE_PIPE=0 timeout -k 10 300 python -u $D --out gpurun_out/r4_declat_pipe0.json > /dev/null || exit 1
DGI_DECODE_PIPE=1 timeout -k 10 300 python -u $D --out gpurun_out/r4_declat_pipe1.json > /dev/null || exit 1
DGI_DECODE_PIPE=2 DGI_DECODE_SHORT_CTX=0 timeout -k 10 300 python -u $D --out gpurun_out/r4_declat_pipe2_noshort.json > /dev/null || exit 1
python3 - <<'PY'
import json
for f in ["pipe2", "pipe0", "pipe1", "pipe2_noshort"]:
    rows = json.load(open(f"gpurun_out/r4_declat_{f}.json"))
    print(f, " | ".join(f"b{r['batch']} {r['tpot_ms']:.3f}" for r in rows))
PY
echo ALLDONE
