#!/bin/bash
# Round 6, session 3: RadixAttention prefix sharing and the pinned host KV tier measured on one
# MI355X, then the served path (SDK -> control plane -> worker daemon -> engine)
# with engine-side and HTTP TTFT side by side.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then exit $rc; fi
}
B="python -u bench.py --steps 20 --warmup 5"
step 8b_base 420 $B --model llama3-8b --json-out $O/8b_base.json
step 8b_prefix384 420 $B --model llama3-8b --shared-prefix-len 384 --json-out $O/8b_prefix384.json
step 8b_prefix384_g8 420 $B --model llama3-8b --shared-prefix-len 384 --prefix-groups 8 --json-out $O/8b_prefix384_g8.json
step 8b_kvpress_recompute 420 $B --model llama3-8b --kv-blocks 9000 --json-out $O/8b_kvpress_recompute.json
step 8b_kvpress_swap 420 $B --model llama3-8b --kv-blocks 9000 --host-kv-gb 24 --json-out $O/8b_kvpress_swap.json
step 70b_prefix384 420 $B --model llama3-70b --shared-prefix-len 384 --json-out $O/70b_prefix384.json
step e2e_8b 600 python -u benchmarks/single_worker.py --backend all --launch --model llama3-8b --num-requests 64 --concurrent 8 --max-tokens 128 --prompt-length 128 --steps 40 --warmup 5 --output $O/e2e_8b.json
echo ALLDONE
