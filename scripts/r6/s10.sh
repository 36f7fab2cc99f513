#!/bin/bash
# Round 6, session 10: software-pipelined prefill attention (numerics + A/B at the 70B head
# geometry), then the headline / decode-role A/B of the fused-norm RoPE epilogue (repeated).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s10
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step prefill_tests 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "paged_prefill"
step attn_ab 400 env ATTN_PREFILL_ONLY=1 ATTN_TILES=128,256 ATTN_DB=1 ATTN_PIPE=0,1 python -u scripts/attn_bench.py
for r in 1 2; do
  step bench_rope_$r 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench_rope_$r.json
  step bench_norope_$r 600 env DGI_NORM_FOLD_ROPE=0 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench_norope_$r.json
done
step dec_fold_norope 400 env DGI_NORM_FOLD=force DGI_NORM_FOLD_ROPE=0 python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512.jsonl
step dec_fold_rope 400 env DGI_NORM_FOLD=force python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512.jsonl
step dec_base 400 env DGI_NORM_FOLD=0 python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512.jsonl
echo ALLDONE
