#!/usr/bin/env python3
"""Debug: decode lookahead with the sampler writing the next ids in place (tiny model, 4 rows)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from dgi.engine import EngineConfig, LLMEngine
from dgi.models.config import get_config
from dgi.models.llama import LlamaModel
from dgi.sched.request import SamplingParams

mc = get_config("llama-tiny-hd128")
src = LlamaModel(mc, "cuda", seed=7)
prompts = [[1] + list(range(3, 3 + n)) for n in (5, 40, 130, 7)]
MT = lambda i: 9 + 4 * i   # noqa: E731  (the GPU test's lengths: rows leave the chain one by one)
for la, inst in ((False, False), (True, False), (True, True)):
    cfg = EngineConfig(model="llama-tiny-hd128", device="cuda", num_blocks=256, max_num_seqs=8, max_model_len=512,
                       max_num_batched_tokens=512, use_graphs=True, decode_lookahead=la)
    e = LLMEngine(cfg, model_cfg=mc, model=src)
    g = e.runner.graphs
    orig_launch = g.launch

    def launch(dec, ahead=0, _o=orig_launch, _g=g):
        torch.cuda.synchronize()
        print(f"  launch n={len(dec)} ahead={ahead} ids_before={_g.dev_in[:8].tolist()}", flush=True)
        h = _o(dec, ahead)
        torch.cuda.synchronize()
        print(f"    after: ids={_g.dev_in[:8].tolist()} out={_g.out[:8].tolist()}", flush=True)
        return h
    if inst:
        g.launch = launch
    reqs = [e.add_request(p, SamplingParams(max_tokens=MT(i), temperature=0.0, ignore_eos=True, seed=100 + i))
            for i, p in enumerate(prompts)]
    while e.has_unfinished():
        e.step()
    print("lookahead" if la else "plain", "instrumented" if inst else "", [r.output for r in reqs], flush=True)
