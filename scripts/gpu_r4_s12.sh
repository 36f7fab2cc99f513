#!/bin/bash
# Round 4, session 12: small-batch decode attention latency (graph-chained launches + kernel trace),
# then 8-rank RCCL rehearsals (shared GPU): batched receives (default) vs serial vs batched sends too.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
timeout -k 10 240 python -u scripts/decode_attn_b1.py > gpurun_out/r4_attn_b1.jsonl 2> gpurun_out/r4_attn_b1.err || { tail -20 gpurun_out/r4_attn_b1.err; exit 1; }
cat gpurun_out/r4_attn_b1.jsonl
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_attn_b1 -o run --output-format csv -- \
  python3 scripts/decode_attn_b1.py --batch 1 --ctx 384 > gpurun_out/prof_attn_b1.log 2>&1 || { tail -20 gpurun_out/prof_attn_b1.log; exit 1; }
head -12 gpurun_out/prof_attn_b1/run_kernel_stats.csv
export DGI_HANG_DUMP_S=200 REHEARSE_MODEL=llama3-70b@L8 REHEARSE_CONC=256 REHEARSE_STEPS=20 REHEARSE_WARMUP=5 REHEARSE_TIMEOUT=280
REHEARSE_TAG=_r4b bash scripts/rehearse_rccl_bench.sh pdpp8_5p_pp3 pd8_2p_6d > gpurun_out/r4_reh_b.log 2>&1 || { cat gpurun_out/r4_reh_b.log; exit 1; }
DGI_KV_RECV_BATCH=1 REHEARSE_TAG=_r4s bash scripts/rehearse_rccl_bench.sh pdpp8_5p_pp3 pd8_2p_6d > gpurun_out/r4_reh_s.log 2>&1 || { cat gpurun_out/r4_reh_s.log; exit 1; }
DGI_BATCH_P2P=1 REHEARSE_TAG=_r4bb bash scripts/rehearse_rccl_bench.sh pdpp8_5p_pp3 pd8_2p_6d > gpurun_out/r4_reh_bb.log 2>&1 || { cat gpurun_out/r4_reh_bb.log; exit 1; }
cat gpurun_out/r4_reh_b.log gpurun_out/r4_reh_s.log gpurun_out/r4_reh_bb.log
echo ALLDONE
