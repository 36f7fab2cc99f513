#!/bin/bash
# Round 6, session 1: the round's new GPU paths first (async host tier, prefix hits under graphs,
# swap-in feeding captured decode, served-path E2E), then the whole GPU suite, smoke and the
# 1-GPU headline bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s1
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-1200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step new_tests 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_host_tier.py tests/test_worker_daemon.py tests/test_kernels_gpu.py tests/test_mfma_gemm.py -k "host_tier or prefix or swap or served or kv_gather or kv_scatter or slot or norm"
step gpu_suite 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench70b 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench70b.json
echo ALLDONE
