"""Single-worker serving benchmark (reference benchmarks/single_worker.py, measured instead of never run).

Closed-loop load against one engine: ``--num-requests`` requests, at most
``--concurrent`` in flight, ``--max-tokens`` output each.  Reports output
tok/s, TTFT p50/p95 and TPOT p50.  Backends:

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


def _pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * (len(xs) - 1) + 0.5))]


def bench_engine(a) -> dict:
    import torch
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.sched.request import SamplingParams
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    eng = LLMEngine(EngineConfig(model=a.model, device=dev, max_num_seqs=max(a.concurrent, 1),
                                 max_num_batched_tokens=a.max_batched_tokens, max_model_len=4096))
    eng.warmup()
    g = torch.Generator().manual_seed(0)
    V = eng.model_cfg.vocab_size
    prompts = [torch.randint(min(1000, V // 4), V, (a.prompt_length,), generator=g).tolist()
               for _ in range(a.num_requests)]
    sp = SamplingParams(max_tokens=a.max_tokens, temperature=0.0, ignore_eos=True)
    pending = list(prompts)
    live, done = [], []
    t0 = time.perf_counter()
    while pending or live:
        while pending and len(live) < a.concurrent:
            live.append(eng.add_request(pending.pop(), sp))
        eng.step()
        still = []
        for r in live:
            (done if r.finish_reason else still).append(r)
        live = still
    el = time.perf_counter() - t0
    ttft = [r.ttft * 1000 for r in done]
    tpot = [(r.token_times[-1] - r.token_times[0]) / max(1, len(r.token_times) - 1) * 1000 for r in done]
    toks = sum(len(r.output) for r in done)
    return {"backend": "mi355x", "model": a.model, "device": dev, "requests": len(done), "concurrent": a.concurrent,
            "output_tok_s": round(toks / el, 1), "ttft_p50_ms": round(_pct(ttft, 0.5), 2),
            "ttft_p95_ms": round(_pct(ttft, 0.95), 2), "tpot_p50_ms": round(_pct(tpot, 0.5), 2),
            "seconds": round(el, 2)}


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
    return {"backend": "http", "server": a.server_url, "requests": len(lat), "errors": errs,
            "output_tok_s": round(toks[0] / el, 1), "latency_p50_ms": _pct(lat, 0.5),
            "latency_p95_ms": _pct(lat, 0.95), "mean_latency_ms": statistics.mean(lat) if lat else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="mi355x", choices=["mi355x", "native", "http", "all"])
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--num-requests", type=int, default=100)
    ap.add_argument("--concurrent", type=int, default=8)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--prompt-length", type=int, default=128)
    ap.add_argument("--max-batched-tokens", type=int, default=8192)
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
