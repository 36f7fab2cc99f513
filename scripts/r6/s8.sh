#!/bin/bash
# Round 6, session 8: the RoPE + paged-KV epilogue of the fused-norm qkv GEMM (EPI 5): numerics,
# fused layers end to end, the 512-row decode-role step (fused vs unfused) and the 1-GPU headline.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s8
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_mfma_gemm.py tests/test_kernels_gpu.py -k "norm or rope or paged or fused"
step dec80_512_fold 400 env DGI_NORM_FOLD=force python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512.jsonl
step dec80_512_base 400 env DGI_NORM_FOLD=0 python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512.jsonl
step bench70b 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench70b.json
step bench70b_norope 600 env DGI_NORM_FOLD_ROPE=0 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench70b_norope.json
echo ALLDONE
