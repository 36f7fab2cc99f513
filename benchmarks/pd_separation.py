"""Prefill/decode disaggregation benchmark (reference benchmarks/pd_separation.py, measured).

``--mode separated``: ``--prefill-workers`` prefill GPUs + ``--decode-workers``
decode GPUs on one node, KV over RCCL.  Every decode GPU is its own whole-model
decode replica (the reference's worker model, pd_scheduler.py:274-323: 2P+6D =
2 prefill + 6 decode workers); ``--decode-stages k`` groups them into
``decode_workers / k`` decode layer pipelines of k stages instead.
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
        k = max(1, a.decode_stages)
        if a.decode_workers % k:
            raise SystemExit(f"--decode-workers {a.decode_workers} is not a multiple of --decode-stages {k}")
        args = common + ["--layout", "pdpp" if k > 1 else "pd", "--prefill-ranks", str(a.prefill_workers),
                         "--decode-stages", str(k), "--decode-replicas", str(a.decode_workers // k)]
        return run_bench(n, args)
    return run_bench(n, common + ["--layout", "dp"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="separated", choices=["hybrid", "separated"])
    ap.add_argument("--compare", action="store_true")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--prefill-workers", type=int, default=2)
    ap.add_argument("--decode-workers", type=int, default=6)
    ap.add_argument("--decode-stages", type=int, default=1,
                    help="stages per decode replica (1: every decode GPU is a whole-model replica)")
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
