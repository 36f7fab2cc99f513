#!/bin/bash
# Round 5, session 2: CU-masked stream overlap probe; PMC passes (MFMA / LDS counters) over the hot kernels.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -4 "$O/$name.log" | cut -c1-700
  [ $rc -eq 0 ] || exit $rc
}
step cumask32 180 python -u scripts/cu_mask_probe.py --side 32
step cumask64 180 python -u scripts/cu_mask_probe.py --side 64
step pmc_mfma 120 timeout -s KILL 110 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_mfma -o run --output-format csv -- python3 scripts/pmc_kernels.py
step pmc_lds 120 timeout -s KILL 110 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/pmc_lds -o run --output-format csv -- python3 scripts/pmc_kernels.py
step pmc_wait 120 timeout -s KILL 110 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/pmc_wait -o run --output-format csv -- python3 scripts/pmc_kernels.py
step pmc_hbm 120 timeout -s KILL 110 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/pmc_hbm -o run --output-format csv -- python3 scripts/pmc_kernels.py --only decode,prefill
echo ALLDONE
