#!/bin/bash
# Round 6, session 27: 2 vs 4 MFMA phases for the fused-norm GEMMs at the headline's mixed-step rows.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s27
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 500 python -u scripts/norm_phase_probe.py > $O/norm_phase.jsonl 2> $O/norm_phase.err
rc=$?
echo "=== norm_phase rc=$rc"; cat $O/norm_phase.jsonl | cut -c1-300; tail -3 $O/norm_phase.err
exit $rc
