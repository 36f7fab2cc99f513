#!/bin/bash
# Round 5, session 9: prefill attention v3 (Q-load wait before the K/V pipeline, page16 scalar-base
# K/V loads, block ids prefetched one tile ahead): numerics at every tile / stage variant, A/B at the
# 70B head geometry, MFMA PMC pass, and the 1-GPU headline bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s9
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-900
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
step prefill_tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_spec.py -x -q --timeout 120 --timeout-method thread -k "paged_prefill or tree or spec_gpu or verify_graph"
step attn_ab 300 env ATTN_PREFILL_ONLY=1 ATTN_TILES=128,256 ATTN_DB=0,1 python -u scripts/attn_bench.py
step pmc_mfma 120 timeout -s KILL 110 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_mfma -o run --output-format csv -- python3 scripts/pmc_kernels.py --only prefill
step pmc_wait 120 timeout -s KILL 110 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/pmc_wait -o run --output-format csv -- python3 scripts/pmc_kernels.py --only prefill
step bench70b 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench70b.json
step slo120 600 python -u bench.py --steps 60 --warmup 10 --tpot-slo-ms 120 --json-out $O/slo120.json
echo ALLDONE
