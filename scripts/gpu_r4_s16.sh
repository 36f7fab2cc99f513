#!/bin/bash
# Round 4, session 16: what the driver's scaling run launches (bench.py --layout auto: start-up probe on
# every rank, median plan) on a real RCCL data plane, all ranks on one GPU, Llama-3-8B.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
export DGI_HANG_DUMP_S=250 REHEARSE_MODEL=llama3-8b REHEARSE_CONC=64 REHEARSE_STEPS=20 REHEARSE_WARMUP=5 REHEARSE_TIMEOUT=300
REHEARSE_TAG=_r4 bash scripts/rehearse_rccl_bench.sh auto2 auto4 auto8 > gpurun_out/r4_reh_auto.log 2>&1 || { cat gpurun_out/r4_reh_auto.log; tail -30 gpurun_out/rehearse_auto*_r4.err; exit 1; }
cat gpurun_out/r4_reh_auto.log
for n in 2 4 8; do grep '^{"metric"' gpurun_out/rehearse_auto${n}_r4.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['value'], d['metric_scope'], d['extra'].get('planner',{}).get('source'))"; done
echo ALLDONE
