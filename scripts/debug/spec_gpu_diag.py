"""Diagnose GPU spec-vs-plain mismatches: swap individual native ops for their torch refs."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from dgi import ops
from dgi.engine import EngineConfig, LLMEngine
from dgi.sched.request import SamplingParams
from dgi.spec.eagle3 import SpecConfig, SpecEngine, train_draft

model = sys.argv[1] if len(sys.argv) > 1 else "llama-tiny-hd128"
cfg = EngineConfig(model=model, device="cuda", max_num_seqs=8, max_num_batched_tokens=1024, max_model_len=1024,
                   use_graphs=False, kv_fraction=0.3)
base = LLMEngine(cfg)
se = SpecEngine(cfg, SpecConfig(depth=4, width=3, topk=4), model=base.model)
g = torch.Generator().manual_seed(0)
V = base.model_cfg.vocab_size
prompts = [torch.randint(5, V, (L,), generator=g).tolist() for L in (7, 20, 33, 12)]
sp = SamplingParams(max_tokens=32, temperature=0.0, ignore_eos=True)
ref = [r.output for r in base.generate(prompts, sp)]
print("train", train_draft(se, steps=80, batch=8, prompt_len=32, gen_len=96, num_seqs=32))

orig = {k: getattr(ops, k) for k in ("paged_prefill", "tree_verify", "tree_mask", "topk", "rope_cache")}
refs = {"paged_prefill": lambda q, kc, vc, bt, cu, ctx, nh, nkv, scale, tiles=None, tree_mask=None, tree_n=0, out=None:
        ops.paged_prefill_ref(q, kc, vc, bt, cu, ctx, nh, nkv, scale, tree_mask, tree_n),
        "tree_verify": ops.tree_verify_ref, "tree_mask": ops.tree_mask_ref,
        "topk": lambda x, k: x.float().topk(k, dim=-1), "rope_cache": ops.rope_cache_ref}


def run(tag):
    se.spec_stats.update(spec_steps=0, spec_rows=0, accepted=0, spec_tokens=0)
    out = [r.output for r in se.generate(prompts, sp)]
    same = [o == r for o, r in zip(out, ref)]
    first = [next((i for i, (a, b) in enumerate(zip(o, r)) if a != b), None) for o, r in zip(out, ref)]
    print(json.dumps({"variant": tag, "same": same, "first_diff": first,
                      "acc": round(se.acceptance()["mean_accepted"], 3)}), flush=True)


run("native")
for k in refs:
    setattr(ops, k, refs[k])
    run("ref_" + k)
    setattr(ops, k, orig[k])
for k in refs:
    setattr(ops, k, refs[k])
run("all_ref")
# plain engine with prefill-kernel single-token steps: compare base decode vs prefill-only decode
for k in refs:
    setattr(ops, k, orig[k])
