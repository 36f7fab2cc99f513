set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "paged_decode or model_decode or qwen or glm or fused_decode_model or graph" > gpurun_out/r3_kern.log 2>&1 || { tail -30 gpurun_out/r3_kern.log; exit 1; }
tail -2 gpurun_out/r3_kern.log
for sc in 1024 0; do DGI_DECODE_SHORT_CTX=$sc timeout -k 10 300 python scripts/decode_latency.py --batch 1 4 8 --prompt-len 256 --steps 64 --out gpurun_out/declat_sc${sc}.json > gpurun_out/declat_sc${sc}.log 2>&1 || exit 1; done
for sc in 1024 0; do DGI_DECODE_SHORT_CTX=$sc timeout -k 10 300 python scripts/decode_latency.py --batch 1 4 --prompt-len 900 --steps 64 --out gpurun_out/declat900_sc${sc}.json > gpurun_out/declat900_sc${sc}.log 2>&1 || exit 1; done
cat gpurun_out/declat_sc1024.json gpurun_out/declat_sc0.json gpurun_out/declat900_sc1024.json gpurun_out/declat900_sc0.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec1_r3 -o dec1 -- python3 scripts/decode_latency.py --batch 1 --prompt-len 256 --steps 128 > gpurun_out/prof_dec1_r3.log 2>&1 || exit 1
REHEARSE_MODEL=llama3-70b@L8 REHEARSE_CONC=256 REHEARSE_TAG=_70bL8_r3 DGI_HANG_DUMP_S=170 bash scripts/rehearse_rccl_bench.sh auto8 auto4 auto2 > gpurun_out/rehearse_auto.log 2>&1; cat gpurun_out/rehearse_auto.log
