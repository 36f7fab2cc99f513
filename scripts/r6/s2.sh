#!/bin/bash
# Round 6, session 2: fused-norm MFMA layers (RMSNorm gains folded into qkv / gate_up, residual +
# row statistics in the o / down epilogues): numerics, the 80-layer 512-row decode-role step and
# the 1-GPU headline, each A/B against the unfused layers; rocprof kernel table of the fused step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-1200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step norm_tests 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_mfma_gemm.py tests/test_kernels_gpu.py -k "norm"
step dec80_512_fold 400 env DGI_NORM_FOLD=force python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512.jsonl
step dec80_512_base 400 env DGI_NORM_FOLD=0 python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512.jsonl
step prof_dec_fold 300 rocprofv3 --kernel-trace --stats -d $O/prof_dec_fold -o run -- python3 scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 10 --force-fold
step bench70b_fold 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench70b_default.json
step bench70b_nofold 600 env DGI_NORM_FOLD=0 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench70b_nofold.json
echo ALLDONE
