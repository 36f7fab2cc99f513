#!/bin/bash
# Round 6, session 6: kernel table of the 70B 1-GPU headline on the round-6 tree (fused-norm layers
# on), EAGLE-3 acceptance with a draft trained on the plain random-init (non-peaked) target, and the
# served-path benchmark with the engine row sized to the request count.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s6
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-1200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step prof70b 500 rocprofv3 --kernel-trace --stats -d $O/prof70b -o run -- python3 bench.py --steps 8 --warmup 4 --json-out $O/prof70b_bench.json
step spec_random 500 python -u scripts/bench_spec.py --batch 1 4 --target random --train-steps 1500 --random-seqs 1024 --oracle-accept --out $O/spec_random.json
step e2e_8b 600 python -u benchmarks/single_worker.py --backend all --launch --model llama3-8b --num-requests 64 --concurrent 8 --max-tokens 128 --prompt-length 128 --steps 40 --warmup 5 --output $O/e2e_8b.json
echo ALLDONE
