"""Speculative decoding benchmark (reference benchmarks/speculative.py, measured).

Wraps ``scripts/bench_spec.py``: self-distils the EAGLE-3 draft head of the
random-init target, then compares plain greedy decoding with tree
speculation (lossless check included).  ``--sweep-depth`` repeats for
depths 1..tree-depth.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODELS = {"Qwen/Qwen2.5-7B-Instruct": "llama3-8b"}


def run(model, depth, width, max_tokens, train_steps) -> dict:
    out = os.path.join(ROOT, f".spec_d{depth}.json")
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "bench_spec.py"), "--model", model, "--depth", str(depth),
           "--width", str(width), "--topk", str(max(width, 4)), "--output-len", str(max_tokens), "--train-steps",
           str(train_steps), "--out", out]
    subprocess.run(cmd, check=True)
    with open(out) as f:
        res = json.load(f)
    os.remove(out)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--enabled", default="true", choices=["true", "false"])
    ap.add_argument("--compare", action="store_true", help="always on: plain vs speculative is reported")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tree-depth", type=int, default=5)
    ap.add_argument("--tree-width", type=int, default=3)
    ap.add_argument("--num-requests", type=int, default=50)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--train-steps", type=int, default=300)
    ap.add_argument("--sweep-depth", action="store_true")
    ap.add_argument("--output", default="speculative_results.json")
    a = ap.parse_args()
    model = MODELS.get(a.model, a.model)
    depths = range(1, a.tree_depth + 1) if a.sweep_depth else [a.tree_depth]
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from results import from_spec_row
    res = {}
    for d in depths:
        raw = run(model, d, a.tree_width, a.max_tokens, a.train_steps)
        res[d] = [{"batch": row["batch"],
                   "enabled": from_spec_row(row, model, d, a.tree_width, True, a.max_tokens).to_dict(),
                   "disabled": from_spec_row(row, model, d, a.tree_width, False, a.max_tokens).to_dict()}
                  for row in raw["rows"]]
    print(json.dumps(res, indent=2))
    with open(a.output, "w") as f:
        json.dump(res, f, indent=2)


if __name__ == "__main__":
    main()
