"""Prefill/decode disaggregation benchmark (reference benchmarks/pd_separation.py, measured).

``--mode separated``: ``--prefill-workers`` prefill GPUs + ``--decode-workers``
decode GPUs (a layer pipeline when > 1) on one node, KV over RCCL.
``--mode hybrid``: the same GPUs as independent replicas (no P/D).
``--compare`` runs both.  Each run is ``bench.py`` under torch.distributed.run.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _common import run_bench, save  # noqa: E402

MODELS = {"Qwen/Qwen2.5-7B-Instruct": "llama3-8b"}


def run(a, mode: str) -> dict:
    n = a.prefill_workers + a.decode_workers
    common = ["--model", MODELS.get(a.model, a.model), "--prompt-len", str(a.prompt_length), "--output-len",
              str(a.max_tokens), "--steps", str(a.steps), "--warmup", str(a.warmup)]
    if a.concurrent:
        common += ["--concurrency", str(a.concurrent)]
    if mode == "separated":
        layout = "pdpp" if a.decode_workers > 1 else "pd"
        args = common + ["--layout", layout, "--prefill-ranks", str(a.prefill_workers)]
        return run_bench(n, args)
    return run_bench(n, common + ["--layout", "dp"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="separated", choices=["hybrid", "separated"])
    ap.add_argument("--compare", action="store_true")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--prefill-workers", type=int, default=2)
    ap.add_argument("--decode-workers", type=int, default=6)
    ap.add_argument("--num-requests", type=int, default=100, help="kept for CLI compatibility; load is step-bounded")
    ap.add_argument("--concurrent", type=int, default=0)
    ap.add_argument("--prompt-length", type=int, default=512)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--stress", action="store_true", help="saturating load (concurrency 512 per decode engine)")
    ap.add_argument("--output", default="pd_separation_results.json")
    a = ap.parse_args()
    if a.stress:
        a.concurrent = 512
    from results import from_bench_pd
    modes = ["separated", "hybrid"] if a.compare else [a.mode]
    out = {}
    for m in modes:
        raw = run(a, m)
        pre, dec = (a.prefill_workers, a.decode_workers) if m == "separated" else \
            (0, a.prefill_workers + a.decode_workers)
        out[m] = from_bench_pd(raw, m, pre, dec).to_dict()
    for m, r in out.items():
        print(m, json.dumps(r))
    save(a.output, out)


if __name__ == "__main__":
    main()
