# Round-3 session 5: GPU tests after the host-path vectorisation, 8B / 70B 1-GPU benches,
# 8B decode launch-config sweep.
set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_staged_gpu.py tests/test_spec.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3_s5_tests.log 2>&1 || { tail -30 gpurun_out/r3_s5_tests.log; exit 1; }
tail -1 gpurun_out/r3_s5_tests.log
timeout -k 10 400 python bench.py --model llama3-8b --steps 30 --warmup 5 > gpurun_out/bench8b_s5.json 2> gpurun_out/bench8b_s5.err || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench70_s5.json 2> gpurun_out/bench70_s5.err || exit 1
python -c "
import json
for f in ('gpurun_out/bench8b_s5.json','gpurun_out/bench70_s5.json'):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ttft_p50_ms'], d['tpot_p50_ms'], d['extra']['phases'])"
bash scripts/gpu_round3_decode_sweep.sh
