#!/bin/bash
# Round 4, session 28 (final tree): GPU suite + smoke, then the 1-GPU headline bench twice and a
# decode-stage step at 768 rows (P/D decode role).
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_s28_tests.log 2>&1 || { tail -40 gpurun_out/r4_s28_tests.log; exit 1; }
tail -2 gpurun_out/r4_s28_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_s28_smoke.log 2>&1 || { tail -20 gpurun_out/r4_s28_smoke.log; exit 1; }
tail -1 gpurun_out/r4_s28_smoke.log
for r in 1 2; do
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_s28_bench$r.json 2> gpurun_out/r4_s28_bench$r.err || { tail -20 gpurun_out/r4_s28_bench$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r4_s28_bench$r.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ttft_p50_ms'], d['tpot_p50_ms'])"
done
timeout -k 10 300 python -u scripts/decode_stage_prof.py --rows 768 > gpurun_out/r4_s28_stage.log 2>&1 || { tail -20 gpurun_out/r4_s28_stage.log; exit 1; }
tail -5 gpurun_out/r4_s28_stage.log
echo ALLDONE
