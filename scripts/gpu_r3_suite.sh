#!/bin/bash
# Full GPU suite + smoke on the current tree.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_gpu_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r3_gpu_suite.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/r3_gpu_suite.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -20 gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
