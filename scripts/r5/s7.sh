#!/bin/bash
# Round 5, session 7: RCCL transport log check (2 shared-GPU ranks); TPOT-SLO rows with the load-shape prior;
# prefill attention double-buffered LDS A/B; EAGLE-3 with a 32k draft vocabulary vs the full one (8B, peaked target, batch 1 / 4).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s7
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-900
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
step prefill_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "paged_prefill"
step attn_ab 300 env ATTN_PREFILL_ONLY=1 ATTN_TILES=128,256 ATTN_DB=0,1 python -u scripts/attn_bench.py
soft=1 step tests 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "mixed_step_lookahead or lookahead or two_batch"
for r in 1 2; do
  step bench70b_$r 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench70b_$r.json
done
step rccl_log 120 env DGI_SHARED_GPU=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 DGI_WATCHDOG=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29655 scripts/rccl_log_probe.py
step slo120 600 python -u bench.py --steps 60 --warmup 10 --tpot-slo-ms 120 --json-out $O/slo120.json
step spec_v32k 900 python -u scripts/bench_spec.py --batch 1 4 --target peaked --train-steps 1500 --random-seqs 1024 --oracle-accept --draft-vocab 32768 --out $O/spec_v32k.json
step spec_full 900 python -u scripts/bench_spec.py --batch 1 4 --target peaked --train-steps 1500 --random-seqs 1024 --oracle-accept --out $O/spec_full.json
echo ALLDONE
