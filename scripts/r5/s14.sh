#!/bin/bash
# Round 5, session 14 (final tree): GPU suite + smoke, the 1-GPU headline twice, 8B decode TPOT and
# continuous-batching throughput, and the 8-rank shared-GPU RCCL rehearsal of --layout auto at the
# 512/128 headline load (extra.rccl transport table in the JSON).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s14
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then [ "${soft:-0}" = 1 ] && [ $rc -eq 1 ] || exit $rc; fi
}
soft=1 step suite 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
for r in 1 2; do
  step bench70b_$r 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench70b_$r.json
done
step declat8b 600 python -u scripts/decode_latency.py --batch 1 4 16 --out $O/declat8b.json
step bench8b 600 python -u bench.py --model llama3-8b --concurrency 256 --steps 40 --warmup 10 --json-out $O/bench8b.json
export REHEARSE_MODEL=llama3-70b@L8 REHEARSE_CONC=0 REHEARSE_STEPS=20 REHEARSE_WARMUP=3 REHEARSE_TIMEOUT=600 \
  DGI_HANG_DUMP_S=560 REHEARSE_TAG=_r5final REHEARSE_EXTRA="--prompt-len 512 --output-len 128"
step rehearse_auto8 640 bash scripts/rehearse_rccl_bench.sh auto8
cp gpurun_out/rehearse_auto8_r5final.json gpurun_out/rehearse_auto8_r5final.err $O/ 2>/dev/null
echo ALLDONE
