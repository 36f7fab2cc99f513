#!/bin/bash
# Round 6, session 24: bench.py with no flags (the contract's default run) on the final tree.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s24
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
t0=$(date +%s); timeout -k 10 900 python -u bench.py > $O/bench_default.log 2> $O/bench_default.err
rc=$?; t1=$(date +%s)
echo "=== bench_default rc=$rc"; grep '^{"metric"' $O/bench_default.log | cut -c1-600; echo "wall_s=$((t1 - t0))"
exit $rc
