#!/bin/bash
# Round 6: RadixAttention prefix sharing and the pinned host KV tier on one MI355X
# (VERDICT r5 #2).  Each run is its own process under its own time limit; the first
# failure ends the script.
set -e
O=gpurun_out/r6_prefix
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 5"
run() { local name=$1; shift; echo "== $name: $*"; timeout -k 10 400 $B "$@" --json-out $O/$name.json > $O/$name.log 2>&1; tail -c 400 $O/$name.json; echo; }
run 8b_base        --model llama3-8b
run 8b_prefix384   --model llama3-8b --shared-prefix-len 384
run 8b_prefix384_g8 --model llama3-8b --shared-prefix-len 384 --prefix-groups 8
run 8b_kvpress_recompute --model llama3-8b --kv-blocks 9000
run 8b_kvpress_swap      --model llama3-8b --kv-blocks 9000 --host-kv-gb 24
run 70b_base       --model llama3-70b
run 70b_prefix384  --model llama3-70b --shared-prefix-len 384
