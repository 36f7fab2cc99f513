#!/bin/bash
# Round 4, session 1: the GPU suite on the HOL / export changes, then smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/r4_pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/r4_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r4_smoke.log; exit $rc
