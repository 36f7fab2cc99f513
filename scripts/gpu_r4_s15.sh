#!/bin/bash
# Round 4, session 15: GPU suite + smoke (batched RCCL sends on, fused reduce off), then the 1-GPU
# headline bench the driver runs.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_s15_tests.log 2>&1 || { tail -40 gpurun_out/r4_s15_tests.log; exit 1; }
tail -2 gpurun_out/r4_s15_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_s15_smoke.log 2>&1 || { tail -20 gpurun_out/r4_s15_smoke.log; exit 1; }
tail -1 gpurun_out/r4_s15_smoke.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_s15_bench.json 2> gpurun_out/r4_s15_bench.err || { tail -20 gpurun_out/r4_s15_bench.err; exit 1; }
cat gpurun_out/r4_s15_bench.json
echo ALLDONE
