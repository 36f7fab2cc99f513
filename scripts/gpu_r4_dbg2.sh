#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u scripts/debug/lookahead_ids.py > gpurun_out/r4_dbg_la.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/r4_dbg_la.log | tail -60
