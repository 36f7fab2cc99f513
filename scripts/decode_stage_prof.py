#!/usr/bin/env python3
"""One decode-pipeline stage step in isolation: ``--layers`` layers of the model
(Llama-3-70B shapes by default: a 27-layer stage of the 3-stage 70B decode
replica) over ``--rows`` pure-decode rows at ``--ctx`` tokens of context, replayed
as the serving engines do (hipGraph of the decode step).  Prints ms per step;
run under ``rocprofv3 --kernel-trace --stats`` for the per-kernel split.

KV pages are installed directly (dgi.parallel.probe._adopt), so the run is all
decode steps: no prefill kernels in the profile."""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import random
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dgi.models.config import get_config  # noqa: E402
from dgi.parallel.probe import _adopt, _engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--layers", type=int, default=27)
    ap.add_argument("--rows", type=int, default=768)
    ap.add_argument("--ctx", type=int, default=576)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--graphs", type=int, default=1)
    ap.add_argument("--out", default="")
    ap.add_argument("--force-fold", action="store_true", help="fused-norm layers on every step (DGI_NORM_FOLD=force)")
    a = ap.parse_args()
    if a.force_fold:
        from dgi.models import llama
        llama.NORM_FOLD = "force"
    mc = dataclasses.replace(get_config(a.model), num_layers=a.layers)
    bs = 16
    nb = a.rows * (a.ctx // bs + 4 + a.steps // bs + 4) + 8
    eng = _engine(a.model, mc, "cuda", a.rows, max(4096, a.rows), nb, graphs=bool(a.graphs), buckets=(a.rows,))
    _adopt(eng, a.rows, a.ctx, random.Random(0))
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    from dgi.models import llama
    res = {"model": a.model, "layers": a.layers, "rows": a.rows, "ctx": a.ctx, "graphs": a.graphs,
           "norm_fold": llama.NORM_FOLD,
           "ms_per_step": round(ms, 3), "tok_s": round(a.rows / ms * 1e3, 1)}
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
