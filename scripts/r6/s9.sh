#!/bin/bash
# Round 6, session 9: repeat the headline A/B (RoPE epilogue on / off, alternating) and the 512-row
# decode step with the fused-norm layers with and without the RoPE epilogue.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s9
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for r in 1 2; do
  step bench_rope_$r 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench_rope_$r.json
  step bench_norope_$r 600 env DGI_NORM_FOLD_ROPE=0 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench_norope_$r.json
done
step dec_fold_norope 400 env DGI_NORM_FOLD=force DGI_NORM_FOLD_ROPE=0 python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512.jsonl
step dec_fold_rope 400 env DGI_NORM_FOLD=force python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512.jsonl
step dec_base 400 env DGI_NORM_FOLD=0 python -u scripts/decode_stage_prof.py --layers 80 --rows 512 --ctx 576 --steps 30 --out $O/dec80_512.jsonl
echo ALLDONE
