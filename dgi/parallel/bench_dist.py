"""Distributed (N > 1) serving benchmark bodies used by the top-level bench.py.

Layouts (dgi.parallel.plan):
  pp    one S-stage layer pipeline over all N GPUs (rank 0 drives)
  pd    P prefill ranks + 1 decode rank (KV over RCCL)
  pdpp  P prefill ranks + a decode layer pipeline (KV over RCCL, then
        layer-sliced down the pipeline)  — the BASELINE north-star layout

The decode driver is the clock: its micro-steps make the benchmark steps, and
the timed window is a timestamp window on the node's shared monotonic clock
(section "timed window" below): every rank keeps serving across both edges,
counts the tokens it produced inside [t0, t1], and only after t1 fences its KV
transfers, pauses its pipeline, synchronises and meets the others in a
barrier.  Tokens are summed over ranks; the elapsed time is t1 - t0.
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


def dist_serve_budget(args) -> float:
    """Serving-phase deadline (ramp + warm-up + window) of the watchdog's phase clock:
    the ramp (2 x output_len micro-steps) plus (warmup + steps) node steps of up to 8
    micro-steps each, at 0.25 s per micro-step, x3 (``fault.serve_budget``)."""
    from dgi.parallel.fault import serve_budget
    ramp = args.ramp_steps if getattr(args, "ramp_steps", -1) >= 0 else 2 * args.output_len
    return serve_budget(ramp + 8 * (args.warmup + args.steps))


class _FirstHop:
    """``first_hop`` phase until this rank completed its first step, then ``serve``."""

    budget_s = 420.0          # set by run_distributed from the run's step counts

    def __init__(self):
        from dgi.parallel.fault import phase
        self._phase = phase
        self.done = False
        phase("first_hop")

    def step_done(self) -> None:
        if not self.done:
            self.done = True
            self._phase("serve", _FirstHop.budget_s)

    def teardown(self) -> None:
        self.step_done()
        self._phase("teardown")


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
    from dgi.parallel.fault import phase
    f = Fabric()
    rank, world = f.rank, f.world
    layout = plan_node_layout(world, layout_kind, getattr(args, "prefill_ranks", None) or None,
                              decode_stages=getattr(args, "decode_stages", None) or None,
                              decode_replicas=getattr(args, "decode_replicas", None) or None, model=args.model)
    # every communicator of the layout up front (world KV pairs + pipeline sub-communicators),
    # each warmed with one transfer per pair in a deadlock-free order
    phase("pair_warmup")
    t_pairs = f.setup_layout(layout)
    from dgi.parallel.fabric import rccl_transports
    rccl = rccl_transports() if f.on_gpu else None
    ctrl_rtt = ctrl_ping(f, 0, world - 1)
    # model load (+ graph capture) of this rank's role
    from dgi.parallel.fault import BUILD_S
    phase("engine_build", BUILD_S)
    _FirstHop.budget_s = dist_serve_budget(args)
    # decode-side concurrency: k microbatches of the rows the plan priced (a planner output on
    # the 256-row GEMM tile: 512 rows on a whole-model decode GPU, whose KV pool holds ~590
    # sequences, 768 per microbatch of a pipeline; ``plan.plan_pd``)
    k = len(layout.decode_groups[0]) if layout.decode_groups else 1
    from dgi.parallel.plan import capacity_for
    cap = capacity_for(args.model)
    rows = (cap.decode_rows.get(k) if cap is not None else None) or 768
    conc = args.concurrency or rows * k
    # staged rehearsal: every rank shares one GPU, so each takes a slice of its memory
    from dgi.parallel.fabric import shared_gpu
    kv_frac = float(os.environ.get("DGI_KV_FRACTION", 0.35 / world if (f.staged or shared_gpu()) else 0.9))
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
    phase("report")
    extra["rccl"] = rccl
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
    per_rank = [{k: v for k, v in o.items() if k not in ("ttfts", "tpots", "e2es", "rccl")} for o in obj]
    # RCCL transports of the node: each rank's connections (P2P/IPC over xGMI expected on a real
    # node, NET/Socket in the shared-GPU rehearsal)
    rc = [o.get("rccl") for o in obj]
    rccl_node = None
    if any(rc):
        by: dict = {}
        peers: dict = {}
        for o in rc:
            if not o:
                continue
            for k, v in o["by_transport"].items():
                by[k] = by.get(k, 0) + v
            peers.update(o["peers"])
        rccl_node = {"by_transport": by, "peers": dict(sorted(peers.items())),
                     "ranks_logged": sum(1 for o in rc if o)}
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
                                  "ctrl_rtt_us": ctrl_rtt, "rccl": rccl_node,
                                  "migration_ms_p50": round(float(sorted(mig)[len(mig) // 2]), 3) if mig else None,
                                  "tpots": all_tpots, "e2es": all_e2es, "ranks": per_rank}


# ---------------------------------------------------------------------------- timed window
#
# Multi-rank serving runs are timed by a TIMESTAMP window on the node's shared
# monotonic clock (``time.perf_counter`` is CLOCK_MONOTONIC: one clock for every
# process of the node).  The clock rank (a decode driver) steps through ramp +
# warm-up, takes t0 and tells every rank; after K node steps it takes t1 and
# tells every rank again.  Every rank counts the tokens IT produced whose
# application timestamp (``Request.token_times``) lies in [t0, t1]; nothing is
# drained, fenced or paused inside the window (pipelines stay full across both
# edges) — fences, pipeline pauses, the device synchronise and the barrier all
# happen after t1.  A node step is ``micro`` decode micro-steps of the clock
# replica, enough to cover one prefill step: the prefill ranks report their
# measured step time to the clock during the ramp (``MSG_STEPMS``) and the clock
# sizes ``micro`` from it and its own micro-step time (``node_step_micro`` falls
# back to the capacity table), so a --steps 20 window holds ~20 prefill steps of
# every prefill rank.

MSG_T0, MSG_T1, MSG_STEPMS = 1, 2, 3


def _ns(t: float) -> int:
    return int(round(t * 1e9))


def _sec(ns) -> float:
    return int(ns) / 1e9


def node_step_micro(cap, k: int, n_mb: int, prefill_ms: float = 0.0, micro_ms: float = 0.0) -> int:
    """Decode micro-steps of the clock replica per node step: at least one full
    pipeline round (``n_mb``) and at least one prefill step's worth of micro-steps
    — from measured times when given (the slowest prefill rank's step, the clock's
    own micro-step), else from the capacity table (70B 5P+PP3: 202 ms prefill
    step / 42.5 ms stage step -> 5)."""
    micro = max(1, n_mb)
    if prefill_ms > 0 and micro_ms > 0:
        return max(micro, -(-int(prefill_ms * 1000) // max(1, int(micro_ms * 1000))))
    if cap is not None and cap.prefill_step_ms and cap.decode_step_ms.get(k):
        micro = max(micro, -(-int(cap.prefill_step_ms * 1000) // int(cap.decode_step_ms[k] * 1000)))
    return micro


class TokenLog:
    """Tokens this rank produced, by application time; filtered once the window is known."""

    def __init__(self):
        self.times: list = []          # one timestamp per produced token
        self.firsts: list = []         # (time, ttft) of first tokens produced here
        self.finished: list = []       # requests finished here
        self.steps: list = []          # end time of every engine step that ran
        self.seen: dict = {}           # every request this rank produced a token for

    def outputs(self, outs, count_first: bool = True) -> int:
        for o in outs:
            r = o.request
            t = r.token_times[-1] if r.token_times else time.perf_counter()
            self.times.append(t)
            self.seen[id(r)] = r
            if count_first and len(r.output) == 1 and r.ttft is not None:
                self.firsts.append((t, r.ttft))
            if o.finished:
                self.finished.append(r)
        return len(outs)

    def window(self, t0: float, t1: float) -> dict:
        inw = lambda t: t0 <= t <= t1   # noqa: E731
        fin = [r for r in self.finished if r.finish_time is not None and inw(r.finish_time)]
        return {"tokens": sum(1 for t in self.times if inw(t)),
                "ttfts": [v for t, v in self.firsts if inw(t)],
                "tpots": _window_tpots(self.seen.values(), t0, t1),
                "e2es": [r.finish_time - r.arrival for r in fin],
                "steps_in_window": sum(1 for t in self.steps if inw(t))}


def recount(reqs, t0: float, t1: float) -> int:
    """Independent count for the tests: tokens of ``reqs`` (the requests whose tokens this
    rank produced) with a timestamp in the window, read from the requests themselves
    after the run (``DGI_BENCH_RECOUNT=1``)."""
    return sum(1 for r in reqs for t in r.token_times if t0 <= t <= t1)


def _bcast(chans, kind: int, t: float) -> None:
    for ch in chans:
        ch.send([MSG_PHASE, kind, _ns(t)])


# ---------------------------------------------------------------------------- layer pipeline only

def _run_pp(args, f, cfg, layout, role, sp, rng, conc):
    from dgi.parallel.pipeline import PipelineEngine, StageWorker
    ranks = layout.decode_ranks
    if role == "decode_driver":
        eng = PipelineEngine(cfg, f, ranks)
        hop = _FirstHop()
        vocab = eng.model_cfg.vocab_size
        inflight = set()
        log = TokenLog()
        micro = max(1, eng.n_mb)          # node step: one full pipeline round

        def top(limit):
            while len(inflight) < limit:
                inflight.add(eng.add_request(_prompt(rng, args.prompt_len, vocab), sp).rid)

        def step():
            outs = eng.step()
            if outs:
                hop.step_done()
            log.outputs(outs)
            for o in outs:
                if o.finished:
                    inflight.discard(o.rid)

        ramp = args.ramp_steps if args.ramp_steps >= 0 else args.output_len
        per = max(1, -(-conc // max(1, ramp)))
        for i in range(ramp):
            top(min(conc, (i + 1) * per))
            step()
        for _ in range(args.warmup * micro):
            top(conc)
            step()
        t0 = time.perf_counter()
        for _ in range(args.steps * micro):
            top(conc)
            step()
        t1 = time.perf_counter()
        hop.teardown()
        eng.pause_stages()
        torch.cuda.synchronize() if f.device.type == "cuda" else None
        f.barrier()
        eng.stop_stages()
        w = log.window(t0, t1)
        return w["tokens"], t1 - t0, w["ttfts"], {"tokens": w["tokens"], "steps": eng.stats["steps"],
                                                   "micro_per_step": micro, "tpots": w["tpots"], "e2es": w["e2es"],
                                                   "window": {"t0_ns": _ns(t0), "t1_ns": _ns(t1)},
                                                   "token_wait_s": round(eng.wait_s, 3)}
    w = StageWorker(cfg, f, ranks)
    hop = _FirstHop()
    w.on_hop = hop.step_done
    w.run()
    hop.teardown()
    torch.cuda.synchronize() if f.device.type == "cuda" else None
    f.barrier()
    w.run()
    return 0, 0.0, [], {"stage_steps": w.steps}


# ---------------------------------------------------------------------------- P/D (+ decode pipelines)

def _window_tpots(reqs, t0: float, t1: float) -> list:
    """Mean inter-token time (s) of every request with >= 2 tokens inside [t0, t1], finished or
    not.  A window of ~20 node steps is far shorter than a 128-token generation at a 100+ ms
    TPOT, so counting finished requests only would leave TPOT unmeasured (round-5 rehearsal)."""
    out = []
    for r in reqs:
        tt = [t for t in r.token_times if t0 <= t <= t1]
        if len(tt) >= 2:
            out.append((tt[-1] - tt[0]) / (len(tt) - 1))
    return out


def _run_pd(args, f, cfg, layout, role, sp, rng, conc):
    """P prefill ranks + R decode replicas, timed by the timestamp window above.
    The first replica's driver is the clock: it broadcasts t0 / t1 to every
    prefill rank and every other replica driver."""
    from dgi.parallel.fabric import CtrlChannel
    from dgi.parallel.pd import DecodeDriver, PrefillServer
    from dgi.parallel.pipeline import StageWorker
    from dgi.parallel.plan import capacity_for, decode_local_fraction, prefill_overflow_cap

    clock = layout.drivers[0]
    cap = capacity_for(args.model)
    debug_counts = os.environ.get("DGI_BENCH_RECOUNT") == "1"
    if role == "prefill":
        lc = getattr(args, "prefill_local_cap", -1)
        lc = prefill_overflow_cap(layout, model=args.model) if lc < 0 else lc
        # prefill step size: the capacity table's (TTFT: a prompt admitted just in time waits ~1 step)
        pmbt = getattr(args, "prefill_mbt", 0) or (cap.prefill_mbt if cap is not None else args.max_batched_tokens)
        pcfg = EngineConfig(**{**cfg.__dict__, "max_num_seqs": 64 + lc, "max_num_batched_tokens": pmbt})
        srv = PrefillServer(pcfg, f, layout, local_cap=lc)
        hop = _FirstHop()
        ph = CtrlChannel(f, clock, 4, tag="phase")
        vocab = srv.engine.model_cfg.vocab_size
        # one step's worth of prompts, topped up right before each step
        depth = max(1, pmbt // max(1, args.prompt_len))
        log = TokenLog()
        submitted = []

        # open loop (--arrival-rate, node-wide req/s): this rank's Poisson share; the prompt's
        # arrival is its scheduled time, so TTFT includes every wait (queue, credit, prefill)
        rate = float(getattr(args, "arrival_rate", 0.0) or 0.0) / max(1, len(layout.prefill_ranks))
        nxt = {"t": time.perf_counter()}

        def submit():
            r = srv.submit(_prompt(rng, args.prompt_len, vocab), sp)
            if debug_counts:
                submitted.append(r)
            return r

        def top_up():
            if rate > 0:
                now = time.perf_counter()
                while nxt["t"] <= now:
                    submit().arrival = nxt["t"]
                    nxt["t"] += rng.expovariate(rate)
                return
            while len(srv.pending) + len(srv.engine.scheduler.waiting) < depth:
                submit()

        t0 = t1 = None
        step_ms = None
        while t1 is None:
            m = ph.poll()
            if m is not None:
                if int(m[1]) == MSG_T0:
                    t0 = _sec(m[2])
                else:
                    t1 = _sec(m[2])
                continue
            top_up()
            s0 = srv.engine.stats["steps"]
            ts = time.perf_counter()
            log.outputs(srv.step())
            if srv.engine.stats["steps"] > s0:
                hop.step_done()
                log.steps.append(time.perf_counter())
                ms = (log.steps[-1] - ts) * 1e3
                step_ms = ms if step_ms is None else 0.8 * step_ms + 0.2 * ms
                if t0 is None and len(log.steps) % 4 == 0:        # the clock sizes its node step from it
                    ph.send([MSG_PHASE, MSG_STEPMS, int(step_ms * 1000)])
        # after the window: drain every KV transfer this rank started (the decode ranks keep
        # servicing their handshakes) and report the migration count; then synchronise
        hop.teardown()
        srv.fence()
        torch.cuda.synchronize() if f.device.type == "cuda" else None
        f.barrier()
        srv.finish()
        w = log.window(t0, t1)
        ex = {"tokens": w["tokens"], "prompts": len(w["ttfts"]), "prefill_steps_in_window": w["steps_in_window"],
              "prefill_mbt": pmbt, "migrated": srv.migrated, "migrate_s": round(srv.migrate_time, 3),
              "sent_GB": round(srv.sent_bytes / 1e9, 3), "local_cap": lc, "local_tokens": srv.local_tokens,
              "pd_scheduler": srv.pd_stats(), "migration_ms_p50": srv.pd_stats()["migration_ms_p50"],
              "tpots": w["tpots"], "e2es": w["e2es"]}
        if debug_counts:
            ex["recount"] = recount(submitted, t0, t1)
        return w["tokens"], t1 - t0, w["ttfts"], ex

    if role == "decode_driver":
        # a replica the prefill side cannot saturate also serves local prompts with a slice of its pool
        local_frac = float(getattr(args, "decode_local_frac", -1.0))
        if local_frac < 0:
            local_frac = decode_local_fraction(layout, model=args.model)
        drv = DecodeDriver(cfg, f, layout, local_fraction=local_frac)
        hop = _FirstHop()
        is_clock = f.rank == clock
        others = [p for p in layout.prefill_ranks] + [d for d in layout.drivers if d != clock]
        phases = [CtrlChannel(f, p, 4, tag="phase") for p in others] if is_clock else \
            [CtrlChannel(f, clock, 4, tag="phase")]
        vocab = drv.engine.model_cfg.vocab_size
        log = TokenLog()
        seen = {}
        k = len(layout.group_of(f.rank))
        n_mb = getattr(drv.engine, "n_mb", 1)
        micro = node_step_micro(cap, k, n_mb)
        reported: dict = {}          # prefill rank -> its latest step time (ms)
        my_ms = {"ema": None}

        def top_local():
            while local_frac > 0 and drv.admit_local(_prompt(rng, args.prompt_len, vocab), sp) is not None:
                pass

        def one_step() -> bool:
            top_local()
            if not drv.engine.has_unfinished():
                drv.poll()
                if not drv.engine.has_unfinished():
                    time.sleep(0.0005)
                    return False
            ts = time.perf_counter()
            outs = drv.step()
            if outs:
                hop.step_done()
            ms = (time.perf_counter() - ts) * 1e3
            my_ms["ema"] = ms if my_ms["ema"] is None else 0.8 * my_ms["ema"] + 0.2 * ms
            # first tokens of locally admitted prompts are produced here; a migrated request's
            # first token was produced (and is counted) on its prefill rank
            for o in outs:
                if debug_counts:
                    seen[o.rid] = o.request
                r = o.request
                log.times.append(r.token_times[-1] if r.token_times else time.perf_counter())
                log.seen[id(r)] = r
                if o.rid in drv.local_used and len(r.output) == 1 and r.ttft is not None:
                    log.firsts.append((log.times[-1], r.ttft))
                if o.finished:
                    log.finished.append(r)
            log.steps.append(time.perf_counter())
            return True

        def run_steps(n):
            done = 0
            while done < n:
                done += one_step()

        def take_reports():
            for p, ch in zip(others, phases):
                while True:
                    m = ch.poll()
                    if m is None:
                        break
                    if int(m[1]) == MSG_STEPMS:
                        reported[p] = int(m[2]) / 1000.0

        t0 = t1 = None
        if is_clock:
            ramp = args.ramp_steps if args.ramp_steps >= 0 else 2 * args.output_len
            run_steps(ramp)
            take_reports()
            if reported and my_ms["ema"]:
                micro = node_step_micro(cap, k, n_mb, max(reported.values()), my_ms["ema"])
            run_steps(args.warmup * micro)
            take_reports()
            t0 = time.perf_counter()
            _bcast(phases, MSG_T0, t0)
            run_steps(args.steps * micro)
            t1 = time.perf_counter()
            _bcast(phases, MSG_T1, t1)
        else:
            while t1 is None:
                m = phases[0].poll()
                if m is not None:
                    if int(m[1]) == MSG_T0:
                        t0 = _sec(m[2])
                    else:
                        t1 = _sec(m[2])
                    continue
                one_step()
        # after the window: receive every announced migration (prefill ranks fence), drain
        # the decode pipeline, synchronise, barrier
        hop.teardown()
        drv.await_fences()
        if hasattr(drv.engine, "pause_stages"):
            drv.engine.pause_stages()
        torch.cuda.synchronize() if f.device.type == "cuda" else None
        f.barrier()
        running = len(drv.engine.scheduler.running)
        # receive migrations still in flight so every prefill send completes
        while not drv.all_prefill_done():
            drv.poll()
            time.sleep(0.001)
        drv.finish()
        w = log.window(t0, t1)
        ex = {"tokens": w["tokens"], "received": drv.received, "running_at_end": running,
              "recv_GB": round(drv.recv_bytes / 1e9, 3), "local_fraction": local_frac,
              "steps": drv.engine.stats["steps"], "micro_per_step": micro,
              "prefill_step_ms_reported": {str(p): round(v, 2) for p, v in reported.items()},
              "micro_step_ms": round(my_ms["ema"], 3) if my_ms["ema"] else None,
              "micro_steps_in_window": w["steps_in_window"], "tpots": w["tpots"], "e2es": w["e2es"],
              "window": {"t0_ns": _ns(t0), "t1_ns": _ns(t1)}, **drv.stats(),
              "token_wait_s": round(getattr(drv.engine, "wait_s", 0.0), 3)}
        if debug_counts:
            # a migrated request's token_times hold only what this replica produced (its first
            # token was produced on the prefill rank); a local prompt's hold all of its tokens
            ex["recount"] = recount(seen.values(), t0, t1)
        return w["tokens"], t1 - t0, w["ttfts"], ex

    # later stages of a decode pipeline replica (receive their KV slices from the prefill ranks)
    w = StageWorker(cfg, f, layout.group_of(f.rank), kv_sources=layout.prefill_ranks)
    hop = _FirstHop()
    w.on_hop = hop.step_done
    w.run()
    hop.teardown()
    torch.cuda.synchronize() if f.device.type == "cuda" else None
    f.barrier()
    w.run()
    return 0, 0.0, [], {"tokens": 0, "stage_steps": w.steps, "installed": w.installed,
                        "kv_block_s": round(w.kv_block_s, 4),
                        "kv_transport": w.kvr.stats() if w.kvr is not None else None}
