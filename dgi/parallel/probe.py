"""Start-up per-role capacity probe (what ``bench.py --layout auto`` plans with).

Round 3 chose the 8-GPU layout from a table measured once on one box
(``plan.CAPACITY``); the P/D-vs-DP call sat within that box-to-box spread
(VERDICT r3 weak #9).  Here every rank of the node measures its own GPU for a
few seconds before the layout is fixed, with the real engine on shortened
copies of the model (same hidden size, heads, vocabulary and page size):

* prefill step  — ``prefill_mbt`` prompt tokens per step, max_tokens = 1;
* decode step   — ``rows`` pure-decode rows at the load's mean context
  (prompt + output/2 tokens), KV pages installed directly (no prefill);
* mixed step    — ``rows`` decode rows + prompt/output x rows prefill tokens,
  the steady state of a data-parallel GPU under the 512/128 load.

Each is timed at two layer counts, ``t(n) = fixed + n * per_layer``, and
extrapolated to the model's depth (the fixed part is the embedding, LM head,
sampler and host work of one step).  ``capacity_from_probe`` turns the fits
into a ``plan.RoleCapacity``; ranks gather their probes and plan with the
median, so every rank picks the same layout.
"""
from __future__ import annotations

import dataclasses
import os
import random
import time
from typing import Optional

import torch

from dgi.models.config import ModelConfig, get_config


@dataclasses.dataclass
class ProbeResult:
    model: str
    prefill: tuple          # (fixed_ms, per_layer_ms) at prefill_mbt tokens
    decode: dict            # rows -> (fixed_ms, per_layer_ms)
    mixed: tuple            # (fixed_ms, per_layer_ms) at mixed_rows decode rows
    prefill_mbt: int
    mixed_rows: int
    prompt_len: int
    output_len: int
    layers: tuple
    seconds: float
    prefill_more: dict = dataclasses.field(default_factory=dict)   # other step sizes: mbt -> fit

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)


def _time_steps(eng, steps: int, before=None) -> float:
    """Median ms of one ``eng.step()`` over ``steps`` (after 2 untimed; each step ends on its
    sampled tokens, so its wall time is its device time plus the host work of the step).  The
    median keeps one slow step (a late allocation, a clock transition) out of the fit."""
    import statistics
    sync = (lambda: torch.cuda.synchronize()) if eng.device.type == "cuda" else (lambda: None)
    for _ in range(2):
        if before:
            before()
        eng.step()
    ts = []
    for _ in range(steps):
        if before:
            before()
        sync()
        t0 = time.perf_counter()
        eng.step()
        sync()
        ts.append((time.perf_counter() - t0) * 1e3)
    return statistics.median(ts)


def _engine(model: str, mc: ModelConfig, device: str, max_seqs: int, mbt: int, num_blocks: int,
            graphs: bool, buckets=None):
    from dgi.engine import EngineConfig, LLMEngine
    cfg = EngineConfig(model=model, device=device, max_num_seqs=max_seqs, max_num_batched_tokens=mbt,
                       max_model_len=2048, use_graphs=graphs, enable_prefix_caching=False, num_blocks=num_blocks,
                       graph_buckets=buckets)
    eng = LLMEngine(cfg, model_cfg=mc)
    if graphs:
        eng.warmup()
    return eng


def _adopt(eng, n: int, ctx: int, rng) -> None:
    """``n`` running sequences with ``ctx`` tokens of (uninitialised) KV each."""
    from dgi.sched.request import Request, SamplingParams
    bs = eng.pool.block_size
    sp = SamplingParams(max_tokens=1 << 20, temperature=0.0, ignore_eos=True)
    V = eng.model_cfg.vocab_size
    for _ in range(n):
        r = Request([rng.randrange(1, V) for _ in range(ctx - 1)], sp)
        r.output = [rng.randrange(1, V)]
        eng.scheduler.add_prefilled(r, eng.pool.allocate((ctx + bs - 1) // bs))
        eng.requests[r.rid] = r


def _release(device: str) -> None:
    """Give the probe engines' memory (weights, KV, graph pools) back before the
    serving engine sizes its KV pool from free HBM."""
    import gc
    gc.collect()
    if device != "cpu":
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


def _fit(ts: dict) -> tuple:
    (n0, t0), (n1, t1) = sorted(ts.items())
    per = max(0.0, (t1 - t0) / (n1 - n0))
    return (round(max(0.0, t0 - n0 * per), 4), round(per, 4))


def run_probe(model: str, device: str, prompt_len: int = 512, output_len: int = 128, prefill_mbt: int = 2048,
              decode_rows=(576, 768), mixed_rows: int = 384, layers=(4, 8), steps: int = 8,
              seed: int = 0, prefill_more=(1024,)) -> ProbeResult:
    """Also times prefill steps of each size in ``prefill_more`` (the planner picks the step
    size for TTFT).  Decode rows that take two-batch overlap (``llama.tbo_split``) are timed
    eagerly on the CU-masked streams, as the decode roles run them."""
    from dgi.models import llama
    t_start = time.perf_counter()
    base = get_config(model.split("@")[0] if model else model)
    rng = random.Random(seed)
    ctx = prompt_len + output_len // 2
    bs = 16
    pre, dec, mix = {}, {r: {} for r in decode_rows}, {}
    more = {m: {} for m in prefill_more if m != prefill_mbt}
    per_prompt = max(1, prefill_mbt // prompt_len)
    from dgi.sched.request import SamplingParams
    one = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
    if device != "cpu":
        # the MLP row-padding table (dgi.runtime.gemm_pad) once, at the serving engines' row
        # range: every probe engine below and the serving engine reuse it
        eng = _engine(model, dataclasses.replace(base, num_layers=1), device, 8, 4096, 64, graphs=False)
        del eng
        _release(device)
    for n in layers:
        mc = dataclasses.replace(base, num_layers=n)
        # prefill: a step's worth of prompts waiting before every step
        eng = _engine(model, mc, device, 4 * per_prompt, prefill_mbt, 4 * per_prompt * (prompt_len // bs + 2) + 8,
                      graphs=False)

        def top():
            while len(eng.scheduler.waiting) < per_prompt:
                eng.add_request([rng.randrange(1, mc.vocab_size) for _ in range(prompt_len)], one)
        pre[n] = _time_steps(eng, steps, top)
        del eng
        for mbt in more:
            pp = max(1, mbt // prompt_len)
            eng = _engine(model, mc, device, 4 * pp, mbt, 4 * pp * (prompt_len // bs + 2) + 8, graphs=False)

            def topm_(eng=eng, pp=pp):
                while len(eng.scheduler.waiting) < pp:
                    eng.add_request([rng.randrange(1, mc.vocab_size) for _ in range(prompt_len)], one)
            more[mbt][n] = _time_steps(eng, steps, topm_)
            del eng
        # decode: rows at the mean context, graph-captured like the serving engines (two-batch
        # overlap steps eagerly: a graph would drop the CU masks)
        for rows in decode_rows:
            nb = rows * (ctx // bs + 2 + steps + 4) + 8
            graphs = device != "cpu" and not (llama.TBO and llama.tbo_split(rows) is not None)
            eng = _engine(model, mc, device, rows, max(4096, rows), nb, graphs=graphs, buckets=(rows,))
            _adopt(eng, rows, ctx, rng)
            dec[rows][n] = _time_steps(eng, steps)
            del eng
        # mixed: decode rows + prompt/output x rows prefill tokens per step (DP steady state)
        ptoks = mixed_rows * prompt_len // max(1, output_len)
        nprompt = max(1, ptoks // prompt_len)
        nb = mixed_rows * (ctx // bs + 2 + steps + 4) + 4 * nprompt * (prompt_len // bs + 2) + 8
        eng = _engine(model, mc, device, mixed_rows + 4 * nprompt, mixed_rows + ptoks, nb, graphs=False)
        _adopt(eng, mixed_rows, ctx, rng)

        def topm():
            while len(eng.scheduler.waiting) < nprompt:
                eng.add_request([rng.randrange(1, mc.vocab_size) for _ in range(prompt_len)], one)
        mix[n] = _time_steps(eng, steps, topm)
        del eng
        _release(device)
    return ProbeResult(model=model, prefill=_fit(pre), decode={r: _fit(v) for r, v in dec.items()}, mixed=_fit(mix),
                       prefill_mbt=prefill_mbt, mixed_rows=mixed_rows, prompt_len=prompt_len, output_len=output_len,
                       layers=tuple(layers), seconds=round(time.perf_counter() - t_start, 2),
                       prefill_more={m: _fit(v) for m, v in more.items()})


MIXED_CAL = float(os.environ.get("DGI_PROBE_MIXED_CAL", "1.04"))


def capacity_from_probe(p: ProbeResult, num_layers: Optional[int] = None, max_stages: int = 3):
    """``plan.RoleCapacity`` of the full model from a probe (per-GPU rates).

    A k-stage decode replica runs k microbatches of R rows; each stage step is
    ~1/k of a whole-model decode step at R rows (balanced split), so the
    replica emits k * R tokens per whole-model step: k * R / t_dec(L, R)."""
    from dgi.parallel.plan import RoleCapacity
    L = num_layers or get_config(p.model.split("@")[0]).num_layers
    t = lambda fit: fit[0] + fit[1] * L          # noqa: E731  ms at the full depth
    t_pre = t(p.prefill)
    prompts_per_step = max(1, p.prefill_mbt // p.prompt_len)
    prefill_tok_s = prompts_per_step / (t_pre / 1e3) * p.output_len
    rows = sorted(int(r) for r in p.decode)
    fit = {int(r): v for r, v in p.decode.items()}
    r1 = rows[0]
    dec, step, drows, opts = {}, {}, {}, {}
    from dgi.parallel.plan import decode_pool_seqs
    for k in range(1, max_stages + 1):
        # microbatch sizes whose k in-flight microbatches fit one stage's KV pool (the smallest
        # probed size always stays: the engine caps a replica by its credits anyway)
        pool = decode_pool_seqs(p.model, k, p.prompt_len, p.output_len)
        fits = [R for R in rows if pool is None or k * R <= pool] or rows[:1]
        opts[k] = [[R, round(k * R / (t(fit[R]) / 1e3), 1), round(t(fit[R]) / k, 2)] for R in fits]
        # default (no planner choice): the smallest microbatch for a whole-model decode GPU (its
        # KV pool), the largest for a pipeline
        R = r1 if k == 1 else max(o[0] for o in opts[k])
        _, dec[k], step[k] = next(o for o in opts[k] if o[0] == R)
        drows[k] = R
    # the probe's mixed step is a fixed-shape steady state; the closed-loop DP engine it stands
    # for runs slower (prompt chunks crossing tile boundaries, admission churn): bench.py at the
    # same load measured 203-208 ms per step against the probe's 192-195 ms on the same trees
    # (profiles/r5_pd/README.md §5, probe70b_s23_run1/2.log vs profiles/r5_final/)
    t_mix = t(p.mixed) * MIXED_CAL
    psteps = {p.prefill_mbt: round(t_pre, 2)}
    for m, fit in (p.prefill_more or {}).items():
        psteps[int(m)] = round(t(fit), 2)
    return RoleCapacity(prefill_tok_s=round(prefill_tok_s, 1), decode_tok_s=dec,
                        mixed_tok_s=round(p.mixed_rows / (t_mix / 1e3), 1), prefill_step_ms=round(t_pre, 2),
                        prefill_mbt=p.prefill_mbt, decode_step_ms=step, decode_rows=drows,
                        mixed_step_ms=round(t_mix, 2), prefill_steps=psteps, prompt_len=p.prompt_len,
                        output_len=p.output_len, decode_options=opts)


def median_capacity(caps: list):
    """Element-wise median of several ranks' capacities (same keys)."""
    import statistics
    from dgi.parallel.plan import RoleCapacity
    c0 = caps[0]
    med = lambda xs: round(float(statistics.median(xs)), 2)   # noqa: E731
    return RoleCapacity(
        prefill_tok_s=med([c.prefill_tok_s for c in caps]),
        decode_tok_s={k: med([c.decode_tok_s[k] for c in caps]) for k in c0.decode_tok_s},
        mixed_tok_s=med([c.mixed_tok_s for c in caps]), prefill_step_ms=med([c.prefill_step_ms for c in caps]),
        prefill_mbt=c0.prefill_mbt, decode_step_ms={k: med([c.decode_step_ms[k] for c in caps]) for k in c0.decode_step_ms},
        decode_rows=dict(c0.decode_rows), mixed_step_ms=med([c.mixed_step_ms for c in caps]),
        prefill_steps={m: med([c.steps()[m] for c in caps]) for m in c0.steps()},
        prompt_len=c0.prompt_len, output_len=c0.output_len,
        decode_options={k: [[o[0], med([c.decode_options[k][i][1] for c in caps]),
                             med([c.decode_options[k][i][2] for c in caps])] for i, o in enumerate(v)]
                        for k, v in c0.decode_options.items()})


def plan_from_probe(world: int, cap, min_ratio: Optional[float] = None, lat_frac: Optional[float] = None) -> dict:
    """The auto layout under ``cap``: the planner's best P/D split — the
    fastest whose TTFT and TPOT are at most ``lat_frac`` of a data-parallel GPU's, with the
    prefill step size chosen for TTFT — unless its node rate falls below ``min_ratio`` x
    ``world`` data-parallel GPUs (``plan.PD_MIN_RATIO``) or no split meets the latency bound:
    then data parallel.  The DP estimate is reported next to the pick (``dp_reference``)."""
    from dgi.parallel.plan import MAX_FILLER_SHARE, PD_MIN_RATIO, plan_pd
    if min_ratio is None:
        min_ratio = PD_MIN_RATIO
    best, dp, _cands = plan_pd(world, cap, lat_frac=lat_frac)
    if best is None:
        return {"kind": "dp", "dp_reference": dp, "reason": "no P/D candidate", "estimate": None}
    ratio = best["tok_s"] / dp["tok_s"] if dp["tok_s"] else 0.0
    hybrid = best["filler_share"] > MAX_FILLER_SHARE
    pd_ok = best["latency_ok"] and ratio >= min_ratio and not hybrid
    kind = ("pdpp" if best["decode_stages"] > 1 else "pd") if pd_ok else "dp"
    why = (f"P/D {best['layout']} at {best['prefill_mbt']}-token prefill steps, "
           f"{best.get('decode_rows')}-row decode microbatches: est {best['tok_s']:.0f} tok/s = "
           f"{ratio:.2f} x DP {dp['tok_s']:.0f}, TTFT {best['ttft_ms']} vs {dp['ttft_ms']} ms, TPOT "
           f"{best['tpot_ms']} vs {dp['tpot_ms']} ms -> {kind}"
           + ("" if best["latency_ok"] else " (no split meets the latency bound)")
           + ("" if ratio >= min_ratio else f" (below {min_ratio:g} x DP)")
           + (f" (filler share {best['filler_share']:.2f} > {MAX_FILLER_SHARE:g}: a hybrid, not a split)"
              if hybrid else ""))
    return {"kind": kind, "prefill_ranks": best["prefill_ranks"], "decode_stages": best["decode_stages"],
            "decode_replicas": best["decode_replicas"], "prefill_mbt": best["prefill_mbt"],
            "decode_rows": best.get("decode_rows"), "estimate": best,
            "dp_reference": dp, "dp_tok_s": dp["tok_s"], "reason": why}
