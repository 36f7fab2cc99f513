#!/bin/bash
# Round-end style check of the current tree: GPU suite, smoke, 1-GPU bench; then the 8B decode tables.
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_final.log 2>&1 || { tail -40 gpurun_out/gputest_final.log; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit 1
timeout -k 10 240 python bench.py > gpurun_out/bench70b_final.json 2> gpurun_out/bench70b_final.err || exit 1
bash scripts/gpu_session_decode.sh
