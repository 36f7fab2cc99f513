#!/usr/bin/env python3
"""Per-role capacity of the P/D layouts, measured on ONE MI355X.

The node layouts (dgi/parallel/plan.py) split work into prefill GPUs and a
decode GPU / decode pipeline.  Their balance is decided by two numbers this
script measures on a single GPU with the real engine:

* prefill: prompts/s of a prefill-only engine (512-token prompts,
  max_tokens=1, ``--mbt`` tokens per step) — what one prefill rank feeds;
* decode: ms per pure-decode step of the full model at M rows with ~576
  tokens of context (512 prompt + 64 generated, the 512/128 mean) — a
  2-stage decode pipeline runs each half of it per microbatch.

Prints one JSON line per measurement plus a layout estimate for 8 GPUs
(6 prefill + 2-stage decode) and for N-1 prefill + 1 decode.
"""
from __future__ import annotations

import argparse
import dataclasses
import gc
import json
import os
import random
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dgi.engine import EngineConfig, LLMEngine  # noqa: E402
from dgi.models.config import get_config  # noqa: E402
from dgi.sched.request import SamplingParams  # noqa: E402


def _prompt(rng, n, vocab):
    return [rng.randrange(1000, vocab - 1000) for _ in range(n)]


def prefill_rate(model, mbt, steps, prompt_len):
    eng = LLMEngine(EngineConfig(model=model, device="cuda", max_num_seqs=256, max_num_batched_tokens=mbt,
                                 max_model_len=2048, use_graphs=False, enable_prefix_caching=False,
                                 kv_fraction=0.5))
    rng = random.Random(0)
    sp = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
    per_step = max(1, mbt // prompt_len)

    def top():
        while len(eng.scheduler.waiting) < 2 * per_step:
            eng.add_request(_prompt(rng, prompt_len, eng.model_cfg.vocab_size), sp)
    for _ in range(3):
        top()
        eng.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done = 0
    for _ in range(steps):
        top()
        done += sum(1 for o in eng.step() if o.finished)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    del eng
    _release()
    return {"kind": "prefill", "model": model, "mbt": mbt, "prompts_per_s": round(done / dt, 2),
            "ms_per_step": round(dt / steps * 1000, 2), "prefill_tok_per_s": round(done * prompt_len / dt, 1)}


def _release():
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def decode_step_ms(model, rows, steps, prompt_len, gen_before, layers=None):
    """Pure-decode step time; ``layers`` < the model's depth measures a pipeline
    stage of that many layers (same dims, own embedding + head)."""
    mc = get_config(model)
    if layers:
        mc = dataclasses.replace(mc, num_layers=layers)
    eng = LLMEngine(EngineConfig(model=model, device="cuda", max_num_seqs=rows, max_num_batched_tokens=8192,
                                 max_model_len=2048, use_graphs=True, enable_prefix_caching=False,
                                 graph_buckets=(rows,)), model_cfg=mc)
    eng.warmup()
    rng = random.Random(1)
    # nothing may finish inside the timed steps: the early admissions have already decoded
    # while the later prompts were prefilling, so size max_tokens to the context budget
    sp = SamplingParams(max_tokens=2048 - prompt_len - 8, temperature=0.0, ignore_eos=True)
    for _ in range(rows):
        eng.add_request(_prompt(rng, prompt_len, eng.model_cfg.vocab_size), sp)
    # prefill everything, then decode until the mean context reaches prompt_len + gen_before
    while eng.scheduler.waiting or any(r.in_prefill for r in eng.scheduler.running):
        eng.step()
    for _ in range(gen_before):
        eng.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    for _ in range(steps):
        n += len(eng.step())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert n == rows * steps, f"{n} decode outputs in {steps} steps of {rows} rows (sequences finished or were preempted)"
    del eng
    _release()
    return {"kind": "decode", "model": model, "layers": mc.num_layers, "rows": rows, "ctx": prompt_len + gen_before,
            "ms_per_step": round(dt / steps * 1000, 2), "tok_per_s": round(n / dt, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--decode", default="80:256,80:512,40:512,40:1024,40:1536",
                    help="layers:rows pairs (40 layers = one stage of a 2-stage 70B decode pipeline)")
    ap.add_argument("--mbt", default="4096,8192")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    res = []
    for mbt in [int(x) for x in a.mbt.split(",") if x]:
        res.append(prefill_rate(a.model, mbt, a.steps, a.prompt_len))
        print(json.dumps(res[-1]), flush=True)
    for item in [x for x in a.decode.split(",") if x]:
        layers, rows = (int(v) for v in item.split(":"))
        try:
            res.append(decode_step_ms(a.model, rows, a.steps, a.prompt_len, 64, layers))
        except torch.OutOfMemoryError as e:
            res.append({"kind": "decode", "layers": layers, "rows": rows, "error": "OOM"})
            _release()
        print(json.dumps(res[-1]), flush=True)
    pre = max((r for r in res if r["kind"] == "prefill"), key=lambda r: r["prompts_per_s"], default=None)
    dec = [r for r in res if r["kind"] == "decode" and "ms_per_step" in r]
    if pre and dec:
        out_per_prompt = 128
        demand = pre["prompts_per_s"] * out_per_prompt
        # S-stage pipeline, S microbatches of R rows: each stage step = t(L/S layers, R rows);
        # the pipeline emits S*R tokens per S stage steps -> R / t tokens/s
        L = get_config(a.model).num_layers
        stage = {r["rows"]: r["rows"] / (r["ms_per_step"] / 1000) for r in dec if r["layers"] * 2 == L}
        single = {r["rows"]: r["rows"] / (r["ms_per_step"] / 1000) for r in dec if r["layers"] == L}
        est = {"kind": "estimate", "prefill_gpu_output_demand_tok_s": round(demand, 1),
               "decode_gpu_tok_s": {k: round(v, 1) for k, v in single.items()},
               "decode_2stage_pipeline_tok_s": {k: round(v, 1) for k, v in stage.items()}}
        if stage:
            est["pdpp8_6p2d_tok_s"] = round(min(6 * demand, max(stage.values())), 1)
        res.append(est)
        print(json.dumps(est), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            for r in res:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
