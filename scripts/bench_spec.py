"""EAGLE-3 speculative decoding benchmark (BASELINE config #3: Llama-3-8B + EAGLE-3, 1 GPU).

Random-init target (no checkpoints offline), so the draft head is first
self-distilled on the target's own greedy continuations (``train_draft``);
then plain greedy decoding (hipGraph decode) and tree speculation decode the
same prompts and the script reports tokens/s, mean accepted drafts per step
and checks the outputs are identical (speculation is lossless).

    python scripts/bench_spec.py --model llama3-8b --batch 1 --output-len 128
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dgi.engine import EngineConfig, LLMEngine  # noqa: E402
from dgi.sched.request import SamplingParams  # noqa: E402
from dgi.spec.eagle3 import SpecConfig, SpecEngine, greedy_gap, train_draft  # noqa: E402


def timed_generate(eng, prompts, sp):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reqs = eng.generate(prompts, sp)
    torch.cuda.synchronize()
    return [r.output for r in reqs], time.perf_counter() - t0


def median_run(fn, n):
    """(result of the last run, median seconds) over n runs of fn() -> (result, seconds)."""
    res, ts = None, []
    for _ in range(max(1, n)):
        res, t = fn()
        ts.append(t)
    ts.sort()
    return res, ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 4, 16])
    ap.add_argument("--prompt-len", type=int, default=256)
    ap.add_argument("--output-len", type=int, default=128)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--width", type=int, default=3)
    ap.add_argument("--topk", type=int, default=4)
    ap.add_argument("--train-steps", type=int, default=300)
    ap.add_argument("--train-seqs", type=int, default=64)
    ap.add_argument("--random-seqs", type=int, default=192)
    ap.add_argument("--repeats", type=int, default=3, help="timed runs per measurement (median)")
    ap.add_argument("--oracle-accept", type=float, nargs="*", default=[0.6, 0.8, 1.0])
    ap.add_argument("--target", default="random", choices=["random", "peaked", "concentrated"],
                    help="random: plain random init (near-flat logits: greedy choices sit on bf16 near-ties, so "
                         "kernel-order noise flips them and acceptance collapses); peaked: the LM head is a "
                         "permuted copy of the embedding / sqrt(H), so the next token is a confident function "
                         "of the current one, like a trained model's top-1 margins (same FLOPs and shapes); "
                         "concentrated: as peaked, but every next token is one of --hot-size ids (a random "
                         "map of the vocabulary into that set, a permutation on it), as natural text "
                         "concentrates on its frequent tokens: what an EAGLE-3 draft vocabulary relies on")
    ap.add_argument("--hot-size", type=int, default=32768, help="ids the concentrated target emits")
    ap.add_argument("--no-verify-graph", action="store_true", help="eager verify pass (A/B for the hipGraph)")
    ap.add_argument("--staged", action="store_true",
                    help="separate draft / verify graphs with host-side compaction (A/B for the whole-step graph)")
    ap.add_argument("--no-auto-off", action="store_true", help="always speculate (no plain-decode fallback)")
    ap.add_argument("--no-adaptive", action="store_true", help="fixed tree depth")
    ap.add_argument("--sampled", action="store_true",
                    help="also run seeded temperature 0.8 / top-k 50 / top-p 0.9 requests (coupled verification)")
    ap.add_argument("--draft-vocab", type=int, default=-1,
                    help="EAGLE-3 draft vocabulary: the N token ids the target chose most often in the draft's "
                         "training corpus (0 = the whole vocabulary; -1 = the smallest of 8k/16k/32k/64k covering "
                         "99 %% of the corpus, else the whole vocabulary)")
    ap.add_argument("--save-draft", default=None, help="write the trained draft (torch.save, tensors only)")
    ap.add_argument("--load-draft", default=None, help="skip training: load a draft --save-draft wrote for this target")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cfg = EngineConfig(model=a.model, device="cuda", max_num_seqs=64, max_num_batched_tokens=8192,
                       max_model_len=2048, kv_fraction=0.5)
    spec = SpecEngine(cfg, SpecConfig(depth=a.depth, width=a.width, topk=a.topk, graphs=not a.no_verify_graph,
                                      auto_off=not a.no_auto_off, adaptive_depth=not a.no_adaptive))
    spec.whole_step = not a.staged
    if a.target == "peaked":
        m = spec.model
        perm = torch.randperm(m.embed.shape[0], generator=torch.Generator().manual_seed(7)).to(m.embed.device)
        m.lm_head.copy_(m.embed.index_select(0, perm) / m.cfg.hidden_size ** 0.5)
    elif a.target == "concentrated":
        # next(cur) = f(cur), f: V -> S (|S| = hot_size), a permutation on S: head row j is the sum of the
        # embeddings of j's preimages (~V / |S| of them), rows outside S are zero
        m = spec.model
        V = m.embed.shape[0]
        gen = torch.Generator().manual_seed(7)
        hot = torch.randperm(V, generator=gen)[:a.hot_size]
        f = hot[torch.randint(0, a.hot_size, (V,), generator=gen)]
        f[hot] = hot[torch.randperm(a.hot_size, generator=gen)]
        head = torch.zeros(m.lm_head.shape, dtype=torch.float32, device=m.lm_head.device)
        head.index_add_(0, f.to(head.device), m.embed.float())
        m.lm_head.copy_(head / m.cfg.hidden_size ** 0.5)
        del head
    t0 = time.perf_counter()
    if a.load_draft:
        blob = torch.load(a.load_draft, map_location=spec.device, weights_only=True)
        spec.draft.load(blob["params"])
        spec.draft.set_hot_vocab(blob.get("hot"))
        info = dict(blob["info"], loaded_from=a.load_draft)
    else:
        info = train_draft(spec, steps=a.train_steps, batch=16, prompt_len=64, gen_len=192, num_seqs=a.train_seqs,
                           random_seqs=a.random_seqs, log=lambda m: print(m, flush=True), draft_vocab=a.draft_vocab)
    info["train_seconds"] = round(time.perf_counter() - t0, 1)
    if a.save_draft:
        torch.save({"params": {k: v.detach() for k, v in spec.draft.parameters().items()},
                    "hot": spec.draft.hot, "info": info}, a.save_draft)
    print("draft training", info, flush=True)
    base = LLMEngine(cfg, model=spec.model)
    base.warmup()
    g = torch.Generator().manual_seed(123)
    V = spec.model_cfg.vocab_size
    rows = []
    for B in a.batch:
        prompts = [torch.randint(1000, V, (a.prompt_len,), generator=g).tolist() for _ in range(B)]
        sp = SamplingParams(max_tokens=a.output_len, temperature=0.0, ignore_eos=True)
        timed_generate(base, prompts, SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True))
        timed_generate(spec, prompts, SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True))
        spec.warmup_spec([B])            # every depth the controller can reach, outside the timed runs
        # every timed quantity is the median of --repeats runs (run-to-run spread of the
        # plain engine alone is a few %, the size of the effects measured here)
        ref, t_base = median_run(lambda: timed_generate(base, prompts, sp), a.repeats)

        def spec_run():
            spec.reset_controller()
            spec.spec_stats.update(spec_steps=0, spec_rows=0, accepted=0, spec_tokens=0, draft_s=0.0, verify_s=0.0,
                                   plain_steps=0, switches_off=0, depth_changes=0, whole_steps=0)
            return timed_generate(spec, prompts, sp)
        out, t_spec = median_run(spec_run, a.repeats)
        acc = spec.acceptance()
        toks = B * a.output_len
        gap = max(greedy_gap(spec, p, o) for p, o in zip(prompts, out))
        row = {"batch": B, "plain_tok_s": round(toks / t_base, 1), "spec_tok_s": round(toks / t_spec, 1),
               "speedup": round(t_base / t_spec, 3), "mean_accepted": round(acc["mean_accepted"], 3),
               "tokens_per_step": round(acc["tokens_per_step"], 3), "identical": out == ref,
               "max_greedy_gap": round(gap, 4),
               "draft_s": round(acc["draft_s"], 3), "verify_s": round(acc["verify_s"], 3),
               "whole_step_graph": spec.whole_step, "whole_steps": acc.get("whole_steps", 0),
               "spec_steps": acc["spec_steps"]}
        row["controller"] = {k: acc[k] for k in ("current_depth", "spec_on", "plain_steps", "switches_off",
                                                  "depth_changes")}
        if a.sampled:
            def spm(i):
                return SamplingParams(max_tokens=a.output_len, temperature=0.8, top_k=50, top_p=0.9,
                                      ignore_eos=True, seed=1000 + i)

            def run(eng):
                rs = [eng.add_request(pr, spm(i)) for i, pr in enumerate(prompts)]
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                while eng.has_unfinished():
                    eng.step()
                torch.cuda.synchronize()
                return [r.output for r in rs], time.perf_counter() - t1
            sref, ts_base = run(base)
            spec.reset_controller()
            spec.spec_stats.update(spec_steps=0, spec_rows=0, accepted=0, spec_tokens=0)
            sout, ts_spec = run(spec)
            sa = spec.acceptance()
            row["sampled"] = {"plain_tok_s": round(toks / ts_base, 1), "spec_tok_s": round(toks / ts_spec, 1),
                              "speedup": round(ts_base / ts_spec, 3), "mean_accepted": round(sa["mean_accepted"], 3),
                              "token_agreement": round(sum(int(x == y) for o, q in zip(sout, sref)
                                                           for x, y in zip(o, q)) / max(1, toks), 4)}
        # the feature-tapped plain path alone (what auto-off falls back to)
        spec.force_plain = True
        _, t_tap = median_run(lambda: timed_generate(spec, prompts, sp), a.repeats)
        spec.force_plain = False
        row["tapped_plain"] = {"tok_s": round(toks / t_tap, 1), "vs_plain": round(t_base / t_tap, 3)}
        # acceptance-controlled runs: the first tree chain is replaced by the known greedy
        # continuation, each token kept with probability p (ceiling / sensitivity of the machinery)
        for p in a.oracle_accept:
            def oracle_run():
                reqs_rid = {}
                spec.oracle = reqs_rid
                spec.oracle_accept = p
                rs = [spec.add_request(pr, sp) for pr in prompts]
                for r, o in zip(rs, ref):
                    reqs_rid[r.rid] = o
                spec.reset_controller(keep_plain_costs=True)     # plain cost per bucket is learned once per engine
                spec.step_times = {k: [0.0, 0] for k in spec.step_times}
                spec.spec_stats.update(spec_steps=0, spec_rows=0, accepted=0, spec_tokens=0, draft_s=0.0,
                                       verify_s=0.0, plain_steps=0, switches_off=0, depth_changes=0)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                while spec.has_unfinished():
                    spec.step()
                torch.cuda.synchronize()
                return [r.output for r in rs], time.perf_counter() - t1
            o_out, t_o = median_run(oracle_run, a.repeats)
            spec.oracle = None
            ao = spec.acceptance()
            row[f"oracle_p{p}"] = {"tok_s": round(toks / t_o, 1), "speedup": round(t_base / t_o, 3),
                                   "mean_accepted": round(ao["mean_accepted"], 3),
                                   "identical": o_out == ref,
                                   "spec_steps": ao["spec_steps"], "plain_steps": ao["plain_steps"],
                                   "depth": ao["current_depth"], "costs": ao["cost_ms_per_token"],
                                   "plain_ms_per_token": round(1000 * t_base / toks, 4),
                                   "step_ms": {k: round(1000 * v[0] / max(1, v[1]), 3) for k, v in spec.step_times.items()},
                                   "step_n": {k: v[1] for k, v in spec.step_times.items()}}
        print(json.dumps(row), flush=True)
        rows.append(row)
    res = {"model": a.model, "tree": {"depth": a.depth, "width": a.width, "topk": a.topk}, "target": a.target,
           "verify_graph": not a.no_verify_graph,
           "prompt_len": a.prompt_len, "output_len": a.output_len, "draft_training": info, "rows": rows,
           "data": "synthetic prompts, random-init target, self-distilled draft"}
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=2)


if __name__ == "__main__":
    main()
