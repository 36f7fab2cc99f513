#!/bin/bash
# Round 4, session 10: 8B decode TPOT A/B (lookahead, fused split reduce, short-context graphs),
# batched RCCL receives after pair warm-up (3 ranks, one GPU), the 8-rank RCCL rehearsals with
# batched vs single KV receives, then the GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
D="scripts/decode_latency.py --batch 1 4 16 64 --steps 128"
timeout -k 10 300 python -u $D --out gpurun_out/r4_declat_default.json || exit 1
DGI_DECODE_LOOKAHEAD=0 timeout -k 10 300 python -u $D --out gpurun_out/r4_declat_nola.json || exit 1
DGI_DECODE_LOOKAHEAD=0 DGI_DECODE_FUSED_REDUCE=0 timeout -k 10 300 python -u $D --out gpurun_out/r4_declat_r3.json || exit 1
DGI_DECODE_SHORT_CTX=0 timeout -k 10 300 python -u $D --out gpurun_out/r4_declat_noshort.json || exit 1
timeout -k 10 300 python -u $D --out gpurun_out/r4_declat_default2.json || exit 1
for v in warm warmgroupsend; do
  DGI_SHARED_GPU=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 DGI_WATCHDOG=0 VARIANT=$v timeout -k 5 60 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 \
    --master-port $((29700 + RANDOM % 100)) scripts/debug/rccl_batch_recv.py > gpurun_out/r4_dbg_$v.log 2>&1
  rc=$?; echo "batch-recv $v rc=$rc"; grep -E "^rank" gpurun_out/r4_dbg_$v.log
  [ $rc -eq 0 ] || exit 1
done
export DGI_HANG_DUMP_S=200 REHEARSE_MODEL=llama3-70b@L8 REHEARSE_CONC=256 REHEARSE_STEPS=20 REHEARSE_WARMUP=5 REHEARSE_TIMEOUT=280
REHEARSE_TAG=_r4batch bash scripts/rehearse_rccl_bench.sh pdpp8_5p_pp3 pd8_2p_6d > gpurun_out/r4_reh_batch.log 2>&1 || { cat gpurun_out/r4_reh_batch.log; exit 1; }
DGI_KV_RECV_BATCH=1 REHEARSE_TAG=_r4serial bash scripts/rehearse_rccl_bench.sh pdpp8_5p_pp3 pd8_2p_6d > gpurun_out/r4_reh_serial.log 2>&1 || { cat gpurun_out/r4_reh_serial.log; exit 1; }
cat gpurun_out/r4_reh_batch.log gpurun_out/r4_reh_serial.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_s10_tests.log 2>&1 || { tail -40 gpurun_out/r4_s10_tests.log; exit 1; }
tail -3 gpurun_out/r4_s10_tests.log
echo ALLDONE
