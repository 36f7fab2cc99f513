#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_trim.log 2>&1 || { tail -40 gpurun_out/gputest_trim.log; exit 1; }
timeout -k 10 240 python bench.py > gpurun_out/bench70b_trim.json 2> gpurun_out/bench70b_trim.err || exit 1
DGI_TRIM_LAST_LAYER=0 timeout -k 10 240 python bench.py > gpurun_out/bench70b_notrim.json 2> gpurun_out/bench70b_notrim.err || exit 1
timeout -k 10 240 python bench.py > gpurun_out/bench70b_trim2.json 2> gpurun_out/bench70b_trim2.err || exit 1
