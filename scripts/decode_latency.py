#!/usr/bin/env python3
"""Steady-state decode latency (TPOT) of one engine at small batch sizes.

Prefills B prompts, then times ``--steps`` pure decode steps (hipGraph
replays).  Run twice with DGI_SKINNY_MAX_M=0 / unset to A/B the skinny GEMM.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgi.engine import EngineConfig, LLMEngine  # noqa: E402
from dgi.sched.request import SamplingParams  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 4, 16, 32, 64])
    ap.add_argument("--prompt-len", type=int, default=256)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cfg = EngineConfig(model=a.model, device="cuda", max_num_seqs=max(a.batch), max_num_batched_tokens=8192,
                       max_model_len=2048, kv_fraction=0.5)
    eng = LLMEngine(cfg)
    eng.warmup()
    g = torch.Generator().manual_seed(0)
    V = eng.model_cfg.vocab_size
    rows = []
    for B in a.batch:
        sp = SamplingParams(max_tokens=a.steps + 8, temperature=0.0, ignore_eos=True)
        for _ in range(B):
            eng.add_request(torch.randint(1000, V - 1000, (a.prompt_len,), generator=g).tolist(), sp)
        while any(len(r.output) == 0 for r in eng.requests.values()):
            eng.step()
        for _ in range(4):
            eng.step()
        torch.cuda.synchronize()
        from dgi.utils.trace import phase_summary
        phase_summary(reset=True)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            eng.step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.steps * 1000
        ph = {k: v["ms_avg"] for k, v in phase_summary().items()}
        while eng.has_unfinished():
            eng.step()
        rows.append({"model": a.model, "batch": B, "tpot_ms": round(ms, 3), "tok_s": round(B / ms * 1000, 1),
                     "skinny_max_m": int(os.environ.get("DGI_SKINNY_MAX_M", "32")), "host_phases_ms": ph})
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
