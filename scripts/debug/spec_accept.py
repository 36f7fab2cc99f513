"""Acceptance of the self-distilled EAGLE-3 draft on a peaked synthetic target, per model shape.

    python scripts/debug/spec_accept.py llama-tiny-hd128 cuda
    python scripts/debug/spec_accept.py llama3-8b cuda 2        # 8B dims, 2 layers
"""
import dataclasses
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from dgi.engine import EngineConfig  # noqa: E402
from dgi.models.config import get_config  # noqa: E402
from dgi.sched.request import SamplingParams  # noqa: E402
from dgi.spec.eagle3 import SpecConfig, SpecEngine, train_draft  # noqa: E402

model = sys.argv[1]
dev = sys.argv[2] if len(sys.argv) > 2 else "cuda"
layers = int(sys.argv[3]) if len(sys.argv) > 3 else 0
vocab = int(sys.argv[4]) if len(sys.argv) > 4 else 0
mc = get_config(model)
if layers:
    mc = dataclasses.replace(mc, num_layers=layers)
if vocab:
    mc = dataclasses.replace(mc, vocab_size=vocab)
cfg = EngineConfig(model=model, device=dev, max_num_seqs=8, max_num_batched_tokens=1024, max_model_len=1024,
                   use_graphs=False, kv_fraction=0.3)
se = SpecEngine(cfg, SpecConfig(depth=4, width=3, topk=4), model_cfg=mc)
m = se.model
perm = torch.randperm(m.embed.shape[0], generator=torch.Generator().manual_seed(7)).to(m.embed.device)
m.lm_head.copy_(m.embed.index_select(0, perm) / m.cfg.hidden_size ** 0.5)
t = time.time()
info = train_draft(se, steps=150, batch=8, prompt_len=16, gen_len=64, num_seqs=16, random_seqs=32)
print(model, layers, "train", info, round(time.time() - t, 1), flush=True)
g = torch.Generator().manual_seed(3)
prompts = [torch.randint(1000 if mc.vocab_size > 4000 else 5, mc.vocab_size, (20,), generator=g).tolist()
           for _ in range(2)]
sp = SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True)
se.spec_stats.update(spec_steps=0, spec_rows=0, accepted=0, spec_tokens=0)
outs = se.generate(prompts, sp)
a = se.acceptance()
inv = torch.argsort(perm).cpu()
p, o = prompts[0], outs[0].output
ok = o[:8] == [int(inv[t]) for t in ([p[-1]] + o[:7])]
print(model, layers, "acceptance", round(a["mean_accepted"], 3), "tokens/step", round(a["tokens_per_step"], 3),
      "target-is-permutation", ok, flush=True)
