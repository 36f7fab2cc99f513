#!/bin/bash
# Round 4, session 19: decode attention (scalar page bases for full 16-token-page tiles, hardware exp2): numerics, small-batch plan
# timings, 70B batch-384 check, 8B decode TPOT.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "paged_decode or model_decode or lookahead" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_s19_tests.log 2>&1 || { tail -30 gpurun_out/r4_s19_tests.log; exit 1; }
tail -2 gpurun_out/r4_s19_tests.log
timeout -k 10 300 python -u scripts/decode_attn_b1.py > gpurun_out/r4_attn_btahead.jsonl 2> gpurun_out/r4_attn_btahead.err || { tail -20 gpurun_out/r4_attn_btahead.err; exit 1; }
cat gpurun_out/r4_attn_btahead.jsonl
timeout -k 10 200 python -u scripts/decode_attn_b1.py --heads 64 8 --batch 384 768 --ctx 576 --chain 8 > gpurun_out/r4_attn_btahead70b.jsonl 2>> gpurun_out/r4_attn_btahead.err || { tail -20 gpurun_out/r4_attn_btahead.err; exit 1; }
cat gpurun_out/r4_attn_btahead70b.jsonl
timeout -k 10 300 python -u scripts/decode_latency.py --batch 1 4 16 64 --steps 128 --out gpurun_out/r4_declat_btahead.json > /dev/null || exit 1
python3 -c "
import json
rows = json.load(open('gpurun_out/r4_declat_btahead.json'))
print(' | '.join(f\"b{r['batch']} {r['tpot_ms']:.3f}\" for r in rows))"
echo ALLDONE
