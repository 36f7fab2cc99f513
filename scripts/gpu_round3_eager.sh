# Round-3: every 8-rank layout again with the EAGER RCCL world communicator bench.py now
# creates (the first round-3 rehearsals ran bench.py with a lazily initialised group).
set -o pipefail
export DGI_HANG_DUMP_S=170
REHEARSE_TAG=_eager bash scripts/rehearse_rccl_bench.sh pd8_5p_3d pd8_2p_6d pp8 pdpp8_5p_pp3 pd8_5p_3d_nooverflow > gpurun_out/rehearse_eager.log 2>&1 || { cat gpurun_out/rehearse_eager.log; exit 1; }
REHEARSE_MODEL=llama3-70b@L8 REHEARSE_CONC=256 REHEARSE_TAG=_70bL8_eager \
  bash scripts/rehearse_rccl_bench.sh auto8 pdpp8_5p_pp3_local pd8_5p_3d pp8 pd4_3p_1d pd2_1p_1d_local auto4 auto2 >> gpurun_out/rehearse_eager.log 2>&1 || { cat gpurun_out/rehearse_eager.log; exit 1; }
cat gpurun_out/rehearse_eager.log
grep -l "unbatched P2P" gpurun_out/rehearse_*_eager.err || echo "no lazy per-pair communicators"
