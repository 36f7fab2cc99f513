#!/bin/bash
# Round 6, session 31: the 8B throughput config on the end-of-round tree.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s31
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 600 python -u bench.py --model llama3-8b --steps 20 --warmup 5 --json-out $O/bench8b_final.json > $O/bench8b.log 2>&1
rc=$?
echo "=== bench8b rc=$rc"; grep '^{"metric"' $O/bench8b.log | cut -c1-400
exit $rc
