"""Distributed (N > 1) serving benchmark bodies used by the top-level bench.py.

Layouts (dgi.parallel.plan):
  pp    one S-stage layer pipeline over all N GPUs (rank 0 drives)
  pd    P prefill ranks + 1 decode rank (KV over RCCL)
  pdpp  P prefill ranks + a decode layer pipeline (KV over RCCL, then
        layer-sliced down the pipeline)  — the BASELINE north-star layout

The decode driver is the clock: its steps are the benchmark steps.  Phase
boundaries (end of warmup, end of timed window) are broadcast to prefill
ranks over the control store and to pipeline stages as PAUSE messages, then
every rank meets in a barrier, so the timed window is [barrier, barrier] on
all ranks; tokens are summed over ranks and the elapsed time is the max.
"""
from __future__ import annotations

import os
import random
import time
from typing import Optional

import torch

from dgi.engine import EngineConfig
from dgi.parallel.fabric import Fabric
from dgi.parallel.plan import plan_node_layout
from dgi.sched.request import SamplingParams

MSG_PHASE = 9


def _prompt(rng, n, vocab):
    lo = min(1000, vocab // 4)
    return [rng.randrange(lo, vocab - lo) for _ in range(n)]


def ctrl_ping(f, a: int, b: int, n: int = 400) -> Optional[dict]:
    """Round trip of one control message between ranks ``a`` and ``b`` over the
    node-local control plane (shared-memory rings), microseconds."""
    from dgi.parallel.fabric import CtrlChannel
    if f.rank not in (a, b) or a == b:
        return None
    ch = CtrlChannel(f, b if f.rank == a else a, 4, tag="ping")
    ts = []
    for _ in range(n):
        if f.rank == a:
            t0 = time.perf_counter()
            ch.send([1])
            ch.wait()
            ts.append((time.perf_counter() - t0) * 1e6)
        else:
            ch.wait()
            ch.send([2])
    if not ts:
        return None
    ts.sort()
    return {"p50": round(ts[len(ts) // 2], 2), "p99": round(ts[int(0.99 * (len(ts) - 1))], 2), "n": n}


def capacity_check(cap, layout, per_rank: list, el: float) -> Optional[dict]:
    """The start-up layout pick against what the run measured, per role (the capacity
    table is one box's numbers: profiles/r3_pd_capacity_70b.jsonl)."""
    if cap is None or layout.kind not in ("pd", "pdpp") or el <= 0:
        return None
    k = len(layout.decode_groups[0])
    pre = [o for o in per_rank if o.get("role") == "prefill"]
    drv = [o for o in per_rank if o.get("role") == "decode_driver"]
    ppg = sum(o.get("prompts", 0) for o in pre) / el / max(1, len(pre))
    dpr = sum(o.get("tokens", 0) for o in drv) / el / max(1, len(drv))
    tab = cap.decode_tok_s.get(k)
    return {"prefill_prompts_s_per_gpu": round(ppg, 2), "table_prompts_s": round(cap.prefill_tok_s / 128, 2),
            "decode_tok_s_per_replica": round(dpr, 1), "table_decode_tok_s": tab,
            "decode_utilization": round(dpr / tab, 3) if tab else None}


def run_distributed(args, layout_kind: str, dist):
    f = Fabric()
    rank, world = f.rank, f.world
    layout = plan_node_layout(world, layout_kind, getattr(args, "prefill_ranks", None) or None,
                              decode_stages=getattr(args, "decode_stages", None) or None,
                              decode_replicas=getattr(args, "decode_replicas", None) or None, model=args.model)
    # every communicator of the layout up front (world KV pairs + pipeline sub-communicators),
    # each warmed with one transfer per pair in a deadlock-free order
    t_pairs = f.setup_layout(layout)
    ctrl_rtt = ctrl_ping(f, 0, world - 1)
    # decode-side concurrency: one microbatch of 768 rows per decode stage keeps the
    # decode GEMMs out of the small-M regime (70B down-proj: 0.76 PF/s at M=512,
    # 1.28 at 1024); a single decode GPU is capped by its KV pool (credits) instead
    k = len(layout.decode_groups[0]) if layout.decode_groups else 1
    from dgi.parallel.plan import capacity_for
    cap = capacity_for(args.model)
    rows = (cap.decode_rows.get(k) if cap is not None else None) or 768
    conc = args.concurrency or (rows * k if k > 1 else 1024)
    # staged rehearsal: every rank shares one GPU, so each takes a slice of its memory
    from dgi.parallel.fabric import shared_gpu
    kv_frac = float(os.environ.get("DGI_KV_FRACTION", 0.5 / world if (f.staged or shared_gpu()) else 0.9))
    cfg = EngineConfig(model=args.model, device=str(f.device), max_num_seqs=conc,
                       max_num_batched_tokens=args.max_batched_tokens,
                       max_model_len=max(2048, args.prompt_len + args.output_len + 64),
                       use_graphs=not args.no_graphs, seed=args.seed, enable_prefix_caching=False,
                       kv_fraction=kv_frac)
    sp = SamplingParams(max_tokens=args.output_len, temperature=getattr(args, "temperature", 0.0),
                        top_k=getattr(args, "top_k", 0), top_p=getattr(args, "top_p", 1.0), ignore_eos=True)
    rng = random.Random(777 + rank)
    role = layout.role(rank)
    try:
        if layout.kind == "pp":
            res = _run_pp(args, f, cfg, layout, role, sp, rng, conc)
        else:
            res = _run_pd(args, f, cfg, layout, role, sp, rng, conc)
    except BaseException as e:
        # tell the other ranks (their watchdogs exit instead of waiting in RCCL forever)
        if f.watchdog is not None:
            f.watchdog.report_failure(f"{role}: {type(e).__name__}: {e}")
        raise
    tokens, elapsed, ttfts, extra = res
    t = torch.tensor([tokens, elapsed], dtype=torch.float64, device=f.device if f.on_gpu else "cpu")
    tl = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(tl, t)
    obj = [None] * world
    from dgi.utils.trace import phase_summary
    dist.all_gather_object(obj, {"ttfts": ttfts, "role": role, "phases": phase_summary(), **extra})
    total = int(sum(x[0].item() for x in tl))
    el = max(x[1].item() for x in tl)
    all_ttfts = [v for o in obj for v in o["ttfts"]]
    all_tpots = [v for o in obj for v in o.get("tpots", [])]
    all_e2es = [v for o in obj for v in o.get("e2es", [])]
    per_rank = [{k: v for k, v in o.items() if k not in ("ttfts", "tpots", "e2es")} for o in obj]
    roles = {}
    for o in per_rank:
        r = roles.setdefault(o["role"], {"ranks": 0, "tokens": 0})
        r["ranks"] += 1
        r["tokens"] += int(o.get("tokens", 0))
    for r in roles.values():
        r["tok_s"] = round(r["tokens"] / el, 1) if el > 0 else 0.0
    mig = [o["migration_ms_p50"] for o in per_rank if o.get("migration_ms_p50") is not None]
    from dgi.parallel.plan import capacity_for, layout_estimate
    cap = capacity_for(args.model)
    est = None
    if cap is not None and layout.kind in ("pd", "pdpp"):
        k = len(layout.decode_groups[0])
        if k in cap.decode_tok_s:
            est = layout_estimate(len(layout.prefill_ranks), k, len(layout.decode_groups), cap)
    check = capacity_check(cap, layout, per_rank, el)
    from dgi.parallel.topology import read_topology, summary
    return total, el, all_ttfts, {"planner_estimate": est, "capacity_check": check,
                                  "topology": summary(read_topology()),
                                  "layout": {"kind": layout.kind, "describe": layout.describe(),
                                             "prefill": layout.prefill_ranks, "decode_groups": layout.decode_groups},
                                  "concurrency": conc, "pair_setup_s": round(t_pairs, 3), "roles": roles,
                                  "ctrl_rtt_us": ctrl_rtt,
                                  "migration_ms_p50": round(float(sorted(mig)[len(mig) // 2]), 3) if mig else None,
                                  "tpots": all_tpots, "e2es": all_e2es, "ranks": per_rank}


# ---------------------------------------------------------------------------- layer pipeline only

def _run_pp(args, f, cfg, layout, role, sp, rng, conc):
    from dgi.parallel.pipeline import PipelineEngine, StageWorker
    ranks = layout.decode_ranks
    if role == "decode_driver":
        eng = PipelineEngine(cfg, f, ranks)
        vocab = eng.model_cfg.vocab_size
        inflight = set()

        def top(limit):
            while len(inflight) < limit:
                inflight.add(eng.add_request(_prompt(rng, args.prompt_len, vocab), sp).rid)

        def step():
            n, firsts = 0, []
            for o in eng.step():
                n += 1
                if len(o.request.output) == 1:
                    firsts.append(o.request.ttft)
                if o.finished:
                    inflight.discard(o.rid)
            return n, firsts

        ramp = args.ramp_steps if args.ramp_steps >= 0 else args.output_len
        per = max(1, -(-conc // max(1, ramp)))
        for i in range(ramp):
            top(min(conc, (i + 1) * per))
            step()
        for _ in range(args.warmup):
            top(conc)
            step()
        eng.pause_stages()
        torch.cuda.synchronize() if f.device.type == "cuda" else None
        f.barrier()
        t0 = time.perf_counter()
        toks, ttfts = 0, []
        for _ in range(args.steps):
            top(conc)
            n, fs = step()
            toks += n
            ttfts += fs
        for o in eng.drain():
            toks += 1
        eng.pause_stages()
        torch.cuda.synchronize() if f.device.type == "cuda" else None
        f.barrier()
        el = time.perf_counter() - t0
        eng.stop_stages()
        return toks, el, ttfts, {"tokens": toks, "steps": eng.stats["steps"],
                                 "token_wait_s": round(eng.wait_s, 3)}
    w = StageWorker(cfg, f, ranks)
    w.run()
    torch.cuda.synchronize() if f.device.type == "cuda" else None
    f.barrier()
    t0 = time.perf_counter()
    w.run()
    torch.cuda.synchronize() if f.device.type == "cuda" else None
    f.barrier()
    el = time.perf_counter() - t0
    w.run()
    return 0, el, [], {"stage_steps": w.steps}


# ---------------------------------------------------------------------------- P/D (+ decode pipelines)

def _tpots(reqs) -> list:
    """Mean inter-token time (s) of each finished request with >= 2 tokens."""
    out = []
    for r in reqs:
        tt = r.token_times
        if len(tt) >= 2:
            out.append((tt[-1] - tt[0]) / (len(tt) - 1))
    return out


def _run_pd(args, f, cfg, layout, role, sp, rng, conc):
    """P prefill ranks + R decode replicas.  The first replica's driver is the
    clock: its productive steps are the benchmark steps, and it broadcasts the
    phase boundaries (end of warm-up, end of the timed window) to every
    prefill rank and every other replica driver."""
    from dgi.parallel.fabric import CtrlChannel
    from dgi.parallel.pd import DecodeDriver, PrefillServer
    from dgi.parallel.pipeline import StageWorker
    from dgi.parallel.plan import decode_local_fraction, prefill_overflow_cap

    clock = layout.drivers[0]
    if role == "prefill":
        lc = getattr(args, "prefill_local_cap", -1)
        lc = prefill_overflow_cap(layout, model=args.model) if lc < 0 else lc
        # prefill step size: the capacity table's (TTFT: a prompt admitted just in time waits ~1 step)
        from dgi.parallel.plan import capacity_for
        cap = capacity_for(args.model)
        pmbt = getattr(args, "prefill_mbt", 0) or (cap.prefill_mbt if cap is not None else args.max_batched_tokens)
        pcfg = EngineConfig(**{**cfg.__dict__, "max_num_seqs": 64 + lc, "max_num_batched_tokens": pmbt})
        srv = PrefillServer(pcfg, f, layout, local_cap=lc)
        ph = CtrlChannel(f, clock, 4, tag="phase")
        vocab = srv.engine.model_cfg.vocab_size
        # one step's worth of prompts, topped up right before each step
        depth = max(1, pmbt // max(1, args.prompt_len))

        # open loop (--arrival-rate, node-wide req/s): this rank's Poisson share; the prompt's
        # arrival is its scheduled time, so TTFT includes every wait (queue, credit, prefill)
        rate = float(getattr(args, "arrival_rate", 0.0) or 0.0) / max(1, len(layout.prefill_ranks))
        nxt = {"t": time.perf_counter()}

        def top_up():
            if rate > 0:
                now = time.perf_counter()
                while nxt["t"] <= now:
                    r = srv.submit(_prompt(rng, args.prompt_len, vocab), sp)
                    r.arrival = nxt["t"]
                    nxt["t"] += rng.expovariate(rate)
                return
            while len(srv.pending) + len(srv.engine.scheduler.waiting) < depth:
                srv.submit(_prompt(rng, args.prompt_len, vocab), sp)

        def serve_until_phase():
            n, ttfts = 0, []
            while ph.poll() is None:
                top_up()
                before = len(srv.ttfts)
                n += len(srv.step())
                ttfts += srv.ttfts[before:]
            return n, ttfts

        # at each phase boundary: fence = drain every KV transfer this rank started (the
        # decode ranks keep servicing their handshakes) and report the migration count;
        # afterwards nothing is in flight and the device can be synchronised
        serve_until_phase()
        srv.fence()
        torch.cuda.synchronize() if f.device.type == "cuda" else None
        f.barrier()
        t0 = time.perf_counter()
        n, ttfts = serve_until_phase()
        srv.fence()
        torch.cuda.synchronize() if f.device.type == "cuda" else None
        f.barrier()
        el = time.perf_counter() - t0
        srv.finish()
        return n, el, ttfts, {"tokens": n, "prompts": len(ttfts), "prefill_mbt": pmbt, "migrated": srv.migrated, "migrate_s": round(srv.migrate_time, 3),
                              "sent_GB": round(srv.sent_bytes / 1e9, 3), "local_cap": lc,
                              "local_tokens": srv.local_tokens, "pd_scheduler": srv.pd_stats(),
                              "migration_ms_p50": srv.pd_stats()["migration_ms_p50"]}

    if role == "decode_driver":
        # a replica the prefill side cannot saturate also serves local prompts with a slice of its pool
        local_frac = float(getattr(args, "decode_local_frac", -1.0))
        if local_frac < 0:
            local_frac = decode_local_fraction(layout, model=args.model)
        drv = DecodeDriver(cfg, f, layout, local_fraction=local_frac)
        is_clock = f.rank == clock
        others = [p for p in layout.prefill_ranks] + [d for d in layout.drivers if d != clock]
        phases = [CtrlChannel(f, p, 4, tag="phase") for p in others] if is_clock else \
            [CtrlChannel(f, clock, 4, tag="phase")]
        vocab = drv.engine.model_cfg.vocab_size
        local_ttfts, finished = [], []

        def top_local():
            while local_frac > 0 and drv.admit_local(_prompt(rng, args.prompt_len, vocab), sp) is not None:
                pass

        def one_step():
            n = 0
            for o in drv.step():
                n += 1
                if o.rid in drv.local_used and len(o.request.output) == 1:
                    local_ttfts.append(o.request.ttft)
                if o.finished:
                    finished.append(o.request)
            return n

        def run_steps(k):
            """k productive decode steps (idle polling while nothing has arrived does not count)."""
            n = done = 0
            while done < k:
                top_local()
                if not drv.engine.has_unfinished():
                    drv.poll()
                    if not drv.engine.has_unfinished():
                        time.sleep(0.0005)
                        continue
                n += one_step()
                done += 1
            return n

        def run_until_phase():
            n = 0
            while phases[0].poll() is None:
                top_local()
                if not drv.engine.has_unfinished():
                    drv.poll()
                    if not drv.engine.has_unfinished():
                        time.sleep(0.0005)
                        continue
                n += one_step()
            return n

        def boundary():
            if is_clock:
                for ph in phases:
                    ph.send([MSG_PHASE])
            drv.await_fences()       # receives of every announced migration are posted
            if hasattr(drv.engine, "pause_stages"):
                drv.engine.pause_stages()
            torch.cuda.synchronize() if f.device.type == "cuda" else None
            f.barrier()

        ramp = args.ramp_steps if args.ramp_steps >= 0 else 2 * args.output_len
        if is_clock:
            run_steps(ramp + args.warmup)
        else:
            run_until_phase()
        boundary()
        t0 = time.perf_counter()
        local_ttfts.clear()
        finished.clear()
        n = run_steps(args.steps) if is_clock else run_until_phase()
        boundary()
        el = time.perf_counter() - t0
        running = len(drv.engine.scheduler.running)
        # receive migrations still in flight so every prefill send completes
        while not drv.all_prefill_done():
            drv.poll()
            time.sleep(0.001)
        drv.finish()
        return n, el, list(local_ttfts), {"tokens": n, "received": drv.received, "running_at_end": running,
                                          "recv_GB": round(drv.recv_bytes / 1e9, 3), "local_fraction": local_frac,
                                          "steps": drv.engine.stats["steps"], "tpots": _tpots(finished),
                                          "kv_transport": drv.kvr.stats(),
                                          "e2es": [r.finish_time - r.arrival for r in finished
                                                   if r.finish_time is not None]}

    # later stages of a decode pipeline replica (receive their KV slices from the prefill ranks)
    w = StageWorker(cfg, f, layout.group_of(f.rank), kv_sources=layout.prefill_ranks)
    w.run()
    torch.cuda.synchronize() if f.device.type == "cuda" else None
    f.barrier()
    t0 = time.perf_counter()
    w.run()
    torch.cuda.synchronize() if f.device.type == "cuda" else None
    f.barrier()
    el = time.perf_counter() - t0
    w.run()
    return 0, el, [], {"tokens": 0, "stage_steps": w.steps, "installed": w.installed,
                       "kv_transport": w.kvr.stats() if w.kvr is not None else None}
