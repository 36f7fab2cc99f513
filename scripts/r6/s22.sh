#!/bin/bash
# Round 6, session 22: the split-K timeout error word (GEMM tests, a DGI_DEBUG_SYNC run that reads
# it after every GEMM), then the GPU suite and smoke on the final tree.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s22
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step gemm_tests 300 python -u -m pytest tests/test_mfma_gemm.py -q -m gpu --timeout 120 --timeout-method thread
DGI_DEBUG_SYNC=1 step debug_sync 120 python -u -c "
import torch
from dgi import ops
x = torch.randn(512, 8192, device='cuda', dtype=torch.bfloat16)
w = torch.randn(10240, 8192, device='cuda', dtype=torch.bfloat16) * 0.02
for _ in range(3):
    y = ops.mfma_gemm(x, w, 0, sched=3)
print('split timeouts', ops.gemm_split_timeouts(), 'ok')
"
step gpu_suite 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
echo ALLDONE
