"""Single-worker serving benchmark (reference benchmarks/single_worker.py, measured instead of never run).

Closed-loop load against one engine: at most ``--concurrent`` requests in
flight, ``--max-tokens`` output each; results are the reference's
``BenchmarkResult`` records (benchmarks/results.py).  Backends:

* ``mi355x`` / ``native`` — the dgi engine in-process (HIP kernels, hipGraph decode);
* ``http`` — through the control plane + worker daemon at ``--server-url``
  (end-to-end TTFT including HTTP, queueing and the worker's pull loop).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * (len(xs) - 1) + 0.5))]


def bench_engine(a) -> dict:
    """The dgi engine under ``bench.py`` (closed loop at ``--concurrent``), as a
    reference ``BenchmarkResult``."""
    from _common import run_bench
    from results import from_bench_single, gpu_stats
    args = ["--model", a.model, "--layout", "single", "--concurrency", str(a.concurrent), "--prompt-len",
            str(a.prompt_length), "--output-len", str(a.max_tokens), "--max-batched-tokens",
            str(a.max_batched_tokens), "--steps", str(a.steps), "--warmup", str(a.warmup)]
    res = run_bench(1, args)
    out = from_bench_single(res, backend="mi355x", gpu=gpu_stats()).to_dict()
    out["tpot_p50_ms"] = res.get("tpot_p50_ms")
    return out


def bench_http(a) -> dict:
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sdk", "python"))
    from inference_client import InferenceClient
    lat, errs = [], 0
    lock = threading.Lock()
    todo = list(range(a.num_requests))
    toks = [0]

    def worker():
        nonlocal errs
        c = InferenceClient(a.server_url, api_key=a.api_key or None, timeout=600)
        while True:
            with lock:
                if not todo:
                    return
                i = todo.pop()
            t = time.perf_counter()
            try:
                r = c.chat([{"role": "user", "content": f"request {i}: " + "x" * a.prompt_length}],
                           max_tokens=a.max_tokens, temperature=0.0, sync=True, timeout=600)
                with lock:
                    lat.append((time.perf_counter() - t) * 1000)
                    toks[0] += ((r.get("result") or {}).get("usage") or {}).get("completion_tokens", 0)
            except Exception:
                with lock:
                    errs += 1
    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker) for _ in range(a.concurrent)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    el = time.perf_counter() - t0
    from results import BenchmarkResult
    p = lambda q: float(_pct(lat, q) or 0.0)  # noqa: E731
    mean = statistics.mean(lat) if lat else 0.0
    # sync jobs return whole completions: TTFT through the pull path equals E2E here
    return BenchmarkResult(backend="http", model_id=a.model, total_tokens=int(toks[0]), total_time_s=round(el, 3),
                           tokens_per_second=round(toks[0] / el, 1) if el > 0 else 0.0, avg_ttft_ms=mean,
                           p50_ttft_ms=p(0.5), p95_ttft_ms=p(0.95), p99_ttft_ms=p(0.99), avg_e2e_ms=mean,
                           p50_e2e_ms=p(0.5), p95_e2e_ms=p(0.95), p99_e2e_ms=p(0.99), gpu_memory_used_gb=0.0,
                           gpu_memory_total_gb=0.0, gpu_utilization_pct=0.0, avg_batch_size=float(a.concurrent),
                           total_requests=len(lat)).to_dict() | {"errors": errs, "server": a.server_url}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="mi355x", choices=["mi355x", "native", "http", "all"])
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--num-requests", type=int, default=100)
    ap.add_argument("--concurrent", type=int, default=8)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--prompt-length", type=int, default=128)
    ap.add_argument("--max-batched-tokens", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--server-url", default="http://localhost:8000")
    ap.add_argument("--api-key", default="")
    ap.add_argument("--output", default="benchmark_results.json")
    a = ap.parse_args()
    res = []
    if a.backend in ("mi355x", "native", "all"):
        res.append(bench_engine(a))
    if a.backend in ("http", "all"):
        res.append(bench_http(a))
    for r in res:
        print(json.dumps(r))
    with open(a.output, "w") as f:
        json.dump(res, f, indent=2)


if __name__ == "__main__":
    main()
