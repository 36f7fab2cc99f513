#!/bin/bash
# One gpurun session: kernel tests, smoke, short benches, rocprof stats.
# Stops at the first GPU fault / abort / timeout (exit codes other than 0/1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name timeout cmd...
  local name=$1; local to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"pytest smoke bench8b bench70b"}
for s in $STEPS; do
  case $s in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench8b) run bench8b 900 python bench.py --model llama3-8b --steps 30 --warmup 5 --json-out gpurun_out/bench8b.json ;;
    bench70b) run bench70b 1200 python bench.py --steps 30 --warmup 5 --json-out gpurun_out/bench70b.json ;;
    prof8b) export TMPDIR=/tmp; run prof8b 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8b -o run --output-format csv -- python3 bench.py --model llama3-8b --steps 10 --warmup 2 --ramp-steps 16 ;;
    prof70b) export TMPDIR=/tmp; run prof70b 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof70b -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --ramp-steps 16 ;;
    staged_pd) run staged_pd 600 env DGI_STAGED_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 4 --model llama3-8b --layout pdpp --steps 40 --warmup 5 --ramp-steps 20 --concurrency 64 --max-batched-tokens 2048 ;;
    staged_pp) run staged_pp 600 env DGI_STAGED_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --model llama3-8b --layout pp --steps 40 --warmup 5 --ramp-steps 20 --concurrency 64 --max-batched-tokens 2048 ;;
    staged_pdpp8) run staged_pdpp8 900 env DGI_STAGED_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 8 --model llama3-8b --steps 200 --warmup 5 --ramp-steps 60 --concurrency 96 --max-batched-tokens 2048 --output-len 64 --json-out gpurun_out/staged_pdpp8.json ;;
    gemm) run gemm 600 python scripts/gemm_bench.py 70b ;;
    gemm_libs) run gemm_hipblaslt 600 env GEMM_MS=256,512,768,1024,1536,2048,3072,4096 GEMM_LIB=cublaslt python scripts/gemm_bench.py 70b && run gemm_rocblas 600 env GEMM_MS=256,512,768,1024,1536,2048,3072,4096 GEMM_LIB=cublas python scripts/gemm_bench.py 70b ;;
    staged_pd2) run staged_pd2 600 env DGI_STAGED_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 2 --model llama3-8b --steps 60 --warmup 5 --ramp-steps 30 --concurrency 64 --max-batched-tokens 2048 --output-len 64 --json-out gpurun_out/staged_pd2.json ;;
    staged_pd4) run staged_pd4 600 env DGI_STAGED_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29615 bench.py --gpus 4 --model llama3-8b --steps 60 --warmup 5 --ramp-steps 30 --concurrency 64 --max-batched-tokens 2048 --output-len 64 --json-out gpurun_out/staged_pd4.json ;;
    pmc_attn) export TMPDIR=/tmp; run pmc_attn 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_attn -o run -- python3 scripts/attn_bench.py ;;
    listpmc) export TMPDIR=/tmp; run listpmc 120 rocprofv3 -L ;;
    pdcap) run pdcap 1000 python scripts/pd_capacity.py --mbt 4096 --out gpurun_out/pdcap.jsonl ;;
    gemm_tuned) run gemm_tuned 900 env PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv GEMM_MS=256,1280,2048 python scripts/gemm_bench.py 70b ;;
    sweep70b) for c in 256 384 512; do run sweep70b_c$c 900 python bench.py --steps 40 --warmup 10 --concurrency $c --json-out gpurun_out/sweep70b_c$c.json; done ;;
    sweep70b_mbt) run sweep70b_c384_mbt8k 900 python bench.py --steps 40 --warmup 10 --concurrency 384 --max-batched-tokens 8192 --json-out gpurun_out/sweep70b_c384_mbt8k.json ;;
    spec8b) run spec8b 900 python scripts/bench_spec.py --out gpurun_out/spec8b.json ;;
    spec8b_peaked) run spec8b_peaked 900 python scripts/bench_spec.py --batch 1 4 16 --target peaked --train-steps 1500 --random-seqs 1024 --out gpurun_out/spec8b_peaked.json ;;
    pytest_spec) run pytest_spec 300 python -u -m pytest tests/test_spec.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    spec8b_peaked_eager) run spec8b_peaked_eager 900 python scripts/bench_spec.py --batch 1 4 16 --target peaked --train-steps 1500 --random-seqs 1024 --no-verify-graph --out gpurun_out/spec8b_peaked_eager.json ;;
    skinny_test) run skinny_test 300 python -u -m pytest tests/test_kernels_gpu.py -k skinny -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    skinny_bench) run skinny_bench 600 python scripts/skinny_bench.py --cfg 0 1 2 3 4 5 6 --out gpurun_out/skinny_bench.json ;;
    declat) run declat 600 python scripts/decode_latency.py --out gpurun_out/declat.json && DGI_SKINNY_MAX_M=0 run declat_blaslt 600 python scripts/decode_latency.py --out gpurun_out/declat_blaslt.json ;;
    profdec) export TMPDIR=/tmp; run profdec 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profdec -o run --output-format csv -- python3 scripts/decode_latency.py --batch 1 --steps 200 ;;
    spec8b_cfg3) run spec8b_cfg3 900 python scripts/bench_spec.py --batch 1 8 32 --target peaked --train-steps 1500 --random-seqs 1024 --out gpurun_out/spec8b_cfg3.json ;;
    padtable) run padtable 600 python scripts/mlp_pad_table.py --model llama3-70b --out gpurun_out/mlp_pad_70b.json ;;
    bench70b_nopad) DGI_MLP_PAD=0 run bench70b_nopad 1200 python bench.py --steps 30 --warmup 5 --json-out gpurun_out/bench70b_nopad.json ;;
    pdcap_mbt) run pdcap_mbt 1000 python scripts/pd_capacity.py --mbt 3072,3584,4096,4608,5120,6144 --decode "" --out gpurun_out/pdcap_mbt.jsonl ;;
    spec8b_ctl) run spec8b_ctl 900 python scripts/bench_spec.py --batch 1 4 16 --target peaked --train-steps 1500 --random-seqs 1024 --oracle-accept 0.6 1.0 --sampled --out gpurun_out/spec8b_ctl.json ;;
    fused_tests) run fused_tests 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_hf_parity.py -k "fused or paged_decode or decode_matches or hf_parity" -x -v -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    declat_fused) run declat_fused 600 python scripts/decode_latency.py --batch 1 2 4 16 64 --out gpurun_out/declat_fused.json && DGI_FUSED_DECODE=0 run declat_unfused 600 python scripts/decode_latency.py --batch 1 2 4 16 64 --out gpurun_out/declat_unfused.json && DGI_FUSED_DECODE=0 DGI_DECODE_DYNAMIC=0 run declat_r1 600 python scripts/decode_latency.py --batch 1 2 4 16 64 --out gpurun_out/declat_r1.json ;;
    profdec_fused) export TMPDIR=/tmp; run profdec_fused 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profdec_fused -o run --output-format csv -- python3 scripts/decode_latency.py --batch 1 --steps 200 ;;
    fdbench) run fdbench 600 python scripts/fused_decode_bench.py --out gpurun_out/fdbench.json ;;
    bench70b_long) run bench70b_long 1200 python bench.py --steps 200 --warmup 20 --json-out gpurun_out/bench70b_long.json ;;
  esac
done
echo ALLDONE
