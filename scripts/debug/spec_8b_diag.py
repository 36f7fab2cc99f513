"""8B draft diagnosis: training-path vs inference-path draft outputs and depth-1 accuracy."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import torch.nn.functional as F
from dgi.engine import EngineConfig
from dgi.spec.eagle3 import SpecConfig, SpecEngine, train_draft, collect_features, _varlen_meta

model = sys.argv[1] if len(sys.argv) > 1 else "llama3-8b"
cfg = EngineConfig(model=model, device="cuda", max_num_seqs=16, max_num_batched_tokens=4096, max_model_len=1024,
                   kv_fraction=0.3)
se = SpecEngine(cfg, SpecConfig(depth=5, width=4, topk=4))
info = train_draft(se, steps=int(sys.argv[2]) if len(sys.argv) > 2 else 200, batch=16, prompt_len=64, gen_len=192,
                   num_seqs=32, random_seqs=96)
print("train", info, flush=True)
V = se.model_cfg.vocab_size
g = torch.Generator().manual_seed(5)
seqs = torch.randint(1000, V, (4, 128), generator=g)
raw, tg = collect_features(se, seqs)
dr = se.draft
P = {k: v for k, v in dr.parameters().items()}
with torch.no_grad():
    f = F.linear(raw, P["fc"])
    hid = torch.cat([torch.zeros_like(f[:, :1]), f[:, :-1]], 1)
    ids = seqs.cuda()
    pos = torch.arange(128, device="cuda")[None].expand(4, -1)
    gt = dr.train_forward(P, ids, hid, pos)
    acc_train = (dr.train_logits(P, gt).argmax(-1) == tg).float().mean().item()
    # inference path over the same rows (paged draft cache)
    pool, bs = se.pool, se.pool.block_size
    outs = []
    for b in range(4):
        blocks = pool.allocate(8)
        ps = np.arange(128)
        blk = np.asarray(blocks)
        meta = _varlen_meta(se.runner, ps.tolist(), (blk[ps // bs] * bs + ps % bs).tolist(), [blocks], [0, 128], [128],
                            se.device)
        gi = dr.forward(ids[b], hid[b], meta)
        outs.append(gi)
        pool.free(blocks)
    gi = torch.stack(outs)
    acc_inf = (dr.logprobs(gi.view(-1, gi.shape[-1])).argmax(-1).view(4, 128) == tg).float().mean().item()
    diff = (gi.float() - gt.float()).abs().max().item()
print(json.dumps({"acc_train_path": acc_train, "acc_infer_path": acc_inf, "max_abs_diff": diff,
                  "g_norm": gt.float().norm(dim=-1).mean().item()}), flush=True)
# live spec generation on fresh prompts
from dgi.sched.request import SamplingParams
prompts = [torch.randint(1000, V, (128,), generator=g).tolist() for _ in range(4)]
se.spec_stats.update(spec_steps=0, spec_rows=0, accepted=0, spec_tokens=0)
reqs = se.generate(prompts, SamplingParams(max_tokens=48, temperature=0.0, ignore_eos=True))
print(json.dumps(se.acceptance()), flush=True)
print("sample output", reqs[0].output[:48])
