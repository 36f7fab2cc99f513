#!/bin/bash
# Round 6, session 20: effective clock of the MFMA GEMM with 80 vs 240-256 CUs busy (GRBM counters,
# own run), then the end-of-round validation of the tree: GPU suite, smoke, 70B headline, the
# 512-row decode step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s20
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step clock_pmc 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/pmc -- python3 scripts/clock_probe.py
step clock_sum 60 python3 scripts/clock_probe.py --summarize $O/pmc
step gpu_suite 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench70b 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench70b.json
step dec80_512 400 python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512.jsonl
echo ALLDONE
