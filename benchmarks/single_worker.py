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
    # enough steps for ~--num-requests completions at this concurrency, so the engine row's
    # latency percentiles come from as many requests as the HTTP rows'
    steps = max(a.steps, -(-a.num_requests // max(1, a.concurrent)) * (a.max_tokens + 1))
    args = ["--model", a.model, "--layout", "single", "--concurrency", str(a.concurrent), "--prompt-len",
            str(a.prompt_length), "--output-len", str(a.max_tokens), "--max-batched-tokens",
            str(a.max_batched_tokens), "--steps", str(steps), "--warmup", str(a.warmup)]
    res = run_bench(1, args)
    out = from_bench_single(res, backend="mi355x", gpu=gpu_stats()).to_dict()
    out["tpot_p50_ms"] = res.get("tpot_p50_ms")
    return out


def _prompt_text(i: int, n: int) -> str:
    """~``n`` prompt tokens for the byte-level tokenizer of the random-init presets (one token per
    ASCII character), distinct per request so the prefix cache only shares the chat template."""
    import random
    rng = random.Random(i)
    head = f"request {i}: "
    return head + "".join(rng.choice("abcdefghijklmnopqrstuvwxyz ") for _ in range(max(0, n - len(head))))


def _result(backend, a, lat, ttft, toks, el, errs, extra=None) -> dict:
    from results import BenchmarkResult
    p = lambda xs, q: float(_pct(xs, q) or 0.0)  # noqa: E731
    r = BenchmarkResult(backend=backend, model_id=a.model, total_tokens=int(toks), total_time_s=round(el, 3),
                        tokens_per_second=round(toks / el, 1) if el > 0 else 0.0,
                        avg_ttft_ms=statistics.mean(ttft) if ttft else 0.0, p50_ttft_ms=p(ttft, 0.5),
                        p95_ttft_ms=p(ttft, 0.95), p99_ttft_ms=p(ttft, 0.99),
                        avg_e2e_ms=statistics.mean(lat) if lat else 0.0, p50_e2e_ms=p(lat, 0.5),
                        p95_e2e_ms=p(lat, 0.95), p99_e2e_ms=p(lat, 0.99), gpu_memory_used_gb=0.0,
                        gpu_memory_total_gb=0.0, gpu_utilization_pct=0.0, avg_batch_size=float(a.concurrent),
                        total_requests=len(lat)).to_dict()
    return r | {"errors": errs} | (extra or {})


def _closed_loop(a, one) -> tuple:
    """``a.num_requests`` calls of ``one(i) -> (e2e_ms, ttft_ms, tokens)`` from ``a.concurrent`` threads."""
    lat, ttft, errs = [], [], [0]
    lock = threading.Lock()
    todo = list(range(a.num_requests))
    toks = [0]

    def worker():
        while True:
            with lock:
                if not todo:
                    return
                i = todo.pop()
            try:
                e2e, t1, n = one(i)
                with lock:
                    lat.append(e2e)
                    ttft.append(t1)
                    toks[0] += n
            except Exception as e:   # noqa: BLE001 - counted and reported
                with lock:
                    errs[0] += 1
                    if errs[0] <= 3:
                        print(f"request {i} failed: {type(e).__name__}: {e}", file=sys.stderr)
    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker) for _ in range(a.concurrent)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    return lat, ttft, toks[0], time.perf_counter() - t0, errs[0]


def bench_http(a, server_url: str = "") -> dict:
    """Sync jobs through the control plane (SDK -> server job queue -> worker pull loop -> engine ->
    result post-back).  A sync job returns the whole completion, so its TTFT is its E2E time."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sdk", "python"))
    from inference_client import InferenceClient
    url = server_url or a.server_url
    local = threading.local()

    def one(i):
        c = getattr(local, "c", None) or InferenceClient(url, api_key=a.api_key or None, timeout=600)
        local.c = c
        t = time.perf_counter()
        r = c.chat([{"role": "user", "content": _prompt_text(i, a.prompt_length)}], max_tokens=a.max_tokens,
                   temperature=0.0, sync=True, timeout=600)
        if r.get("status") != "completed":
            raise RuntimeError(f"job {r.get('status')}: {r.get('error')}")
        ms = (time.perf_counter() - t) * 1000
        return ms, ms, ((r.get("result") or {}).get("usage") or {}).get("completion_tokens", 0)
    lat, ttft, toks, el, errs = _closed_loop(a, one)
    return _result("http", a, lat, ttft, toks, el, errs,
                   {"server": url, "path": "SDK -> control plane sync job -> worker pull -> engine",
                    "ttft_note": "sync jobs return the whole completion: TTFT = E2E"})


def bench_stream(a, direct_url: str) -> dict:
    """SSE from the worker's direct endpoint (SDK ``stream_chat`` path): HTTP TTFT = time to the
    first streamed chunk, E2E = time to the end of the stream."""
    import httpx
    local = threading.local()

    def one(i):
        c = getattr(local, "c", None) or httpx.Client(timeout=600)
        local.c = c
        body = {"type": "llm", "params": {"messages": [{"role": "user", "content": _prompt_text(i, a.prompt_length)}],
                                          "max_tokens": a.max_tokens, "temperature": 0.0}}
        t = time.perf_counter()
        first, n = None, 0
        with c.stream("POST", direct_url.rstrip("/") + "/inference/stream", json=body) as r:
            r.raise_for_status()
            for line in r.iter_lines():
                if not line.startswith("data:"):
                    continue
                ev = json.loads(line[5:].strip())
                if ev.get("error"):
                    raise RuntimeError(ev["error"])
                if ev.get("done"):
                    break
                if first is None:
                    first = time.perf_counter()
                n += 1
        end = time.perf_counter()
        return (end - t) * 1000, ((first or end) - t) * 1000, n
    lat, ttft, chunks, el, errs = _closed_loop(a, one)
    return _result("http-sse", a, lat, ttft, chunks, el, errs,
                   {"server": direct_url, "path": "SDK stream_chat -> worker direct SSE -> engine",
                    "ttft_note": "HTTP TTFT = first SSE chunk; total_tokens counts SSE chunks (>= 1 token each)"})


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
    ap.add_argument("--launch", action="store_true",
                    help="http/all: start the control plane + a worker daemon (llm_native on this GPU) as "
                         "separate processes (benchmarks/serve_stack.py) instead of using --server-url")
    ap.add_argument("--poll-interval", type=float, default=0.05, help="--launch: the worker's job poll interval (s)")
    ap.add_argument("--output", default="benchmark_results.json")
    a = ap.parse_args()
    res = []
    if a.backend in ("mi355x", "native", "all"):
        res.append(bench_engine(a))          # first: the launched stack below holds the GPU
    if a.backend in ("http", "all"):
        if a.launch:
            from serve_stack import ServeStack
            out_dir = os.path.join(os.path.dirname(os.path.abspath(a.output)) or ".", "stack_logs")
            eng = {"max_num_seqs": max(64, 2 * a.concurrent), "max_model_len": max(1024, 2 * (a.prompt_length +
                                                                                       a.max_tokens + 64))}
            with ServeStack(a.model, out_dir, poll_interval=a.poll_interval, engine=eng) as st:
                res.append(bench_http(a, st.server_url) | {"poll_interval_s": a.poll_interval})
                res.append(bench_stream(a, st.direct_url) | {"poll_interval_s": a.poll_interval})
        else:
            res.append(bench_http(a))
    if len(res) > 1:
        side = {"engine_ttft_p50_ms": res[0].get("p50_ttft_ms") if res[0]["backend"] == "mi355x" else None}
        for r in res:
            side[f"{r['backend']}_ttft_p50_ms"] = r["p50_ttft_ms"]
            side[f"{r['backend']}_e2e_p50_ms"] = r["p50_e2e_ms"]
        res.append({"side_by_side": side})
    for r in res:
        print(json.dumps(r))
    with open(a.output, "w") as f:
        json.dump(res, f, indent=2)


if __name__ == "__main__":
    main()
