"""Layer-pipeline benchmark (reference benchmarks/distributed.py; its default mode was an
``asyncio.sleep`` simulator — here every mode is measured).

``--workers`` GPUs each hold a contiguous layer range (``plan_layer_split``)
of ``--model`` and pass activations over RCCL; ``--pd`` puts the pipeline
behind prefill engines (the north-star P/D + PP layout).  ``--mode real``
additionally drives the HTTP control plane at ``--server-url``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _common import run_bench, save  # noqa: E402

MODELS = {"meta-llama/Llama-2-70b-chat-hf": "llama3-70b", "meta-llama/Meta-Llama-3-70B": "llama3-70b"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="simulate", choices=["simulate", "real"],
                    help="'simulate' is kept for CLI compatibility and runs the measured in-node pipeline")
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--layers-per-worker", type=int, default=0, help="ignored: split is balanced automatically")
    ap.add_argument("--num-requests", type=int, default=50)
    ap.add_argument("--concurrent", type=int, default=0)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--prompt-length", type=int, default=512)
    ap.add_argument("--pd", action="store_true", help="P/D + pipeline layout (pdpp)")
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--server-url", default="http://localhost:8000")
    ap.add_argument("--api-key", default="")
    ap.add_argument("--output", default="distributed_benchmark_results.json")
    a = ap.parse_args()
    args = ["--model", MODELS.get(a.model, a.model), "--layout", "pdpp" if a.pd else "pp", "--prompt-len",
            str(a.prompt_length), "--output-len", str(a.max_tokens), "--steps", str(a.steps), "--warmup",
            str(a.warmup)]
    if a.concurrent:
        args += ["--concurrency", str(a.concurrent)]
    from results import from_bench_pipeline
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dgi.models.config import get_config
    raw = run_bench(a.workers, args)
    res = {"pipeline": from_bench_pipeline(raw, a.workers, get_config(MODELS.get(a.model, a.model)).num_layers)
           .to_dict(), "raw": {k: raw[k] for k in ("value", "ms_per_step", "config", "latency_ms") if k in raw}}
    if a.mode == "real":
        from single_worker import bench_http
        ns = argparse.Namespace(server_url=a.server_url, api_key=a.api_key, num_requests=a.num_requests,
                                concurrent=max(1, a.concurrent or 4), max_tokens=a.max_tokens,
                                prompt_length=a.prompt_length)
        res["http"] = bench_http(ns)
    print(json.dumps(res))
    save(a.output, res)


if __name__ == "__main__":
    main()
