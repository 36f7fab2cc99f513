#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 500 python3 scripts/pd_capacity.py --model llama3-8b --mbt 4096 --decode 32:256,32:512,32:1024,16:1024,16:1536,11:768,11:1536 > gpurun_out/pd_capacity_8b_v2.jsonl 2> gpurun_out/pd_capacity_8b_v2.err || exit 1
timeout -k 10 600 python3 scripts/pd_capacity.py --model llama3-70b --mbt 4096 --decode 80:512,40:1024,27:768,27:1536 > gpurun_out/pd_capacity_70b_v2.jsonl 2> gpurun_out/pd_capacity_70b_v2.err || exit 1
