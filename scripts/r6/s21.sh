#!/bin/bash
# Round 6, session 21: split-K on CU-limited grids (GPU test), the final tree's 70B headline kernel
# table, EAGLE-3 whole-step numbers on the final tree.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s21
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step cu_tests 200 python -u -m pytest tests/test_mfma_gemm.py -v -m gpu -k "cu_limited or splitk" --timeout 120 --timeout-method thread
step prof70b 500 rocprofv3 --kernel-trace --stats -d $O/prof70b -o run -- python3 bench.py --steps 10 --warmup 4 --json-out $O/prof70b_bench.json
step prof70b_table 120 python3 scripts/rocpd_stats.py $O/prof70b/run_results.db --top 25
step spec 700 python -u scripts/bench_spec.py --batch 1 4 --target peaked --train-steps 1500 --random-seqs 1024 --oracle-accept --no-auto-off --out $O/spec_whole.json
echo ALLDONE
