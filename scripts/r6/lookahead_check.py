"""Determinism probe for test_mixed_step_lookahead_matches_plain_steps (sampled): plain vs plain,
lookahead vs lookahead, plain vs lookahead, with the engine's eager norm fold on and off."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dgi.engine import EngineConfig, LLMEngine  # noqa: E402
from dgi.models.config import get_config  # noqa: E402
from dgi.models.llama import LlamaModel  # noqa: E402
from dgi.sched.request import SamplingParams  # noqa: E402

mc = get_config("llama-tiny-hd128")
src = LlamaModel(mc, "cuda", seed=13)
g = torch.Generator().manual_seed(2)
prompts = [torch.randint(5, 900, (n,), generator=g).tolist() for n in (40, 75, 9, 130, 22, 61)]


def run(mixed):
    cfg = EngineConfig(model="llama-tiny-hd128", device="cuda", num_blocks=256, max_num_seqs=8, max_model_len=512,
                       max_num_batched_tokens=64, use_graphs=True, enable_prefix_caching=False)
    e = LLMEngine(cfg, model_cfg=get_config("llama-tiny-hd128"), model=src)
    e.mixed_lookahead = mixed
    reqs = []
    for i, p in enumerate(prompts):
        reqs.append(e.add_request(p, SamplingParams(max_tokens=7 + 3 * i, temperature=0.8, top_k=20, seed=50 + i,
                                                    ignore_eos=True)))
        e.step()
    while e.has_unfinished():
        e.step()
    return [r.output for r in reqs]


a, b, c, d = run(False), run(False), run(True), run(True)
print("fold", os.environ.get("DGI_NORM_FOLD", "1"), "folded", src.norms_folded,
      "plain==plain", a == b, "la==la", c == d, "plain==la", a == c, flush=True)
