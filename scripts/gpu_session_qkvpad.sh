#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_qkvpad.log 2>&1 || { tail -40 gpurun_out/gputest_qkvpad.log; exit 1; }
timeout -k 10 240 python bench.py > gpurun_out/bench70b_qkvpad.json 2> gpurun_out/bench70b_qkvpad.err || exit 1
DGI_QKV_PAD=0 timeout -k 10 240 python bench.py > gpurun_out/bench70b_noqkvpad.json 2> gpurun_out/bench70b_noqkvpad.err || exit 1
timeout -k 10 240 python bench.py > gpurun_out/bench70b_qkvpad2.json 2> gpurun_out/bench70b_qkvpad2.err || exit 1
DGI_QKV_PAD=0 timeout -k 10 240 python bench.py > gpurun_out/bench70b_noqkvpad2.json 2> gpurun_out/bench70b_noqkvpad2.err || exit 1
