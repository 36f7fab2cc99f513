"""Layer sharding and node layout planning.

* ``get_layer_range_for_worker`` — even split, remainder to the first
  workers (same outputs as reference worker/distributed/model_shard.py:372-394).
* ``plan_layer_split`` — memory/FLOP-balanced split that gives the end stages
  (embedding, LM head) fewer layers.
* ``plan_node_layout`` — how N MI355X GPUs of one node are assigned to
  prefill engines and the decode pipeline.  At 288 GB per GPU a full
  Llama-3-70B (141 GB bf16) fits on one device, so prefill engines are
  whole-model replicas and the decode side is a layer pipeline whose stages
  each hold half (or less) of the layers and therefore several times more KV.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Optional


def get_layer_range_for_worker(total_layers: int, num_workers: int, worker_index: int) -> tuple[int, int]:
    if num_workers <= 0 or not (0 <= worker_index < num_workers):
        raise ValueError("invalid worker index")
    base, rem = divmod(total_layers, num_workers)
    start = worker_index * base + min(worker_index, rem)
    end = start + base + (1 if worker_index < rem else 0)
    return start, end


def plan_layer_split(total_layers: int, stages: int, layer_cost: float = 1.0, embed_cost: float = 0.0,
                     head_cost: float = 0.0) -> list[tuple[int, int]]:
    """Split layers so that per-stage cost (layers * layer_cost + end extras) is balanced."""
    if stages <= 1:
        return [(0, total_layers)]
    extras = [0.0] * stages
    extras[0] += embed_cost
    extras[-1] += head_cost
    target = (total_layers * layer_cost + sum(extras)) / stages
    want = [max(1.0, (target - e) / layer_cost) for e in extras]
    scale = total_layers / sum(want)
    want = [w * scale for w in want]
    counts = [max(1, int(w)) for w in want]
    # largest remainder to make the counts sum to total_layers
    order = sorted(range(stages), key=lambda i: -(want[i] - int(want[i])))
    k = 0
    while sum(counts) < total_layers:
        counts[order[k % stages]] += 1
        k += 1
    while sum(counts) > total_layers:
        i = max(range(stages), key=lambda j: counts[j])
        counts[i] -= 1
    bounds, start = [], 0
    for c in counts:
        bounds.append((start, start + c))
        start += c
    return bounds


@dataclasses.dataclass
class NodeLayout:
    """How the GPUs of one node are assigned.

    ``decode_groups`` lists the decode *replicas*: each is a list of ranks —
    one rank (a whole-model decode GPU) or the stages of a decode layer
    pipeline in order.  A flat list of ints is accepted as ONE group (the
    pre-replica form).  Every prefill rank can migrate to every replica."""
    kind: str                      # single | dp | pp | pd | pdpp
    prefill_ranks: list
    decode_groups: list            # [[driver, stage1, ...], ...]
    replicas: int = 1              # dp: whole-model replicas

    def __post_init__(self):
        g = list(self.decode_groups)
        if g and all(isinstance(x, int) for x in g):
            g = [g]
        self.decode_groups = [list(x) for x in g]

    @property
    def decode_ranks(self) -> list:
        return [r for g in self.decode_groups for r in g]

    @property
    def drivers(self) -> list:
        return [g[0] for g in self.decode_groups]

    @property
    def world(self) -> int:
        return len(self.prefill_ranks) + len(self.decode_ranks)

    def group_of(self, rank: int) -> list:
        for g in self.decode_groups:
            if rank in g:
                return g
        raise KeyError(rank)

    def role(self, rank: int) -> str:
        if rank in self.prefill_ranks:
            return "prefill"
        if rank in self.drivers:
            return "decode_driver"
        return "decode_stage"

    def p2p_pairs(self) -> list:
        """Every rank pair that moves device tensors: prefill -> each decode
        rank (each stage receives its own KV layer slice) and adjacent stages
        of each decode pipeline.  Sorted, so that eager communicator set-up in
        this order cannot deadlock (``Fabric.connect_pairs``)."""
        pairs = set()
        for p in self.prefill_ranks:
            for d in self.decode_ranks:
                pairs.add((min(p, d), max(p, d)))
        for g in self.decode_groups:
            for a, b in zip(g, g[1:]):
                pairs.add((min(a, b), max(a, b)))
        return sorted(pairs)

    def kv_pairs(self) -> list:
        """(prefill, decode rank) pairs that move KV pages on the world communicator."""
        return sorted((min(p, d), max(p, d)) for p in self.prefill_ranks for d in self.decode_ranks)

    def pipeline_groups(self) -> list:
        """Rank lists that get their own activation sub-communicator (every
        multi-stage decode replica; the whole node for a pure pipeline)."""
        return [list(g) for g in self.decode_groups if len(g) > 1]

    def streams_per_rank(self) -> dict:
        """High-priority (communication) streams each rank uses: the world
        communicator, the receive-posting stream (decode ranks) and its
        pipeline's sub-communicator.  Must stay within the hardware queues of
        one priority class (``fabric.GPU_HW_QUEUES``)."""
        out = {}
        for r in range(self.world):
            n = 1                                     # world communicator (KV / collectives)
            if r in self.decode_ranks and self.prefill_ranks:
                n += 1                                # receive-posting stream
            if any(r in g for g in self.pipeline_groups()):
                n += 1                                # activation sub-communicator
            out[r] = n
        return out

    def describe(self) -> str:
        if self.kind in ("single", "dp", "pp"):
            return f"{self.kind}{self.world if self.kind != 'dp' else self.replicas}"
        gs = "+".join(f"pp{len(g)}" if len(g) > 1 else "1" for g in self.decode_groups)
        return f"{len(self.prefill_ranks)}P+{len(self.decode_groups)}D[{gs}]"


@dataclasses.dataclass
class RoleCapacity:
    """Per-role throughput and step latency of one model on one MI355X
    (512-in / 128-out load; ``scripts/pd_capacity.py`` measures it).

    * ``prefill_tok_s``: decode demand one prefill-only GPU creates
      (prompts/s x output_len) at ``prefill_mbt`` tokens per step, whose step
      takes ``prefill_step_ms`` (the TTFT floor of a prompt admitted just in time);
    * ``decode_tok_s[k]``: what one decode replica of k pipeline stages emits
      (k GPUs, k microbatches of ``decode_rows[k]`` rows, one stage step taking
      ``decode_step_ms[k]``: a replica's TPOT is k x that);
    * ``mixed_tok_s`` / ``mixed_step_ms``: one GPU running mixed
      prefill+decode steps (DP, the overflow / local-prompt filler); in DP every
      token of a sequence waits one mixed step, so TTFT ~ TPOT ~ the step."""
    prefill_tok_s: float
    decode_tok_s: dict
    mixed_tok_s: float
    prefill_step_ms: float = 0.0
    prefill_mbt: int = 4096
    decode_step_ms: dict = dataclasses.field(default_factory=dict)
    decode_rows: dict = dataclasses.field(default_factory=dict)
    mixed_step_ms: float = 0.0
    # prefill step time (ms) per prefill step size (tokens): the planner picks the step size
    # for TTFT (a prompt admitted just in time waits ~one step); {prefill_mbt: prefill_step_ms}
    # when only that point was measured
    prefill_steps: dict = dataclasses.field(default_factory=dict)
    prompt_len: int = 512
    output_len: int = 128
    # every measured decode microbatch size per stage count: k -> [[rows, tok_s, step_ms], ...]
    # (the start-up probe fills it; the planner picks the rows per layout, ``decode_choices``)
    decode_options: dict = dataclasses.field(default_factory=dict)

    def decode_choices(self, k: int) -> list:
        """(rows, tok_s, stage step ms) options of a k-stage decode replica."""
        opts = self.decode_options.get(k) or self.decode_options.get(str(k))
        if opts:
            return [tuple(o) for o in opts]
        if k not in self.decode_tok_s:
            return []
        return [(self.decode_rows.get(k), self.decode_tok_s[k], self.decode_step_ms.get(k, 0.0))]

    def with_decode(self, k: int, rows, tok_s: float, step_ms: float) -> "RoleCapacity":
        """This capacity with the k-stage replica run at ``rows``-row microbatches."""
        return dataclasses.replace(self, decode_tok_s={**self.decode_tok_s, k: tok_s},
                                   decode_step_ms={**self.decode_step_ms, k: step_ms},
                                   decode_rows={**self.decode_rows, k: rows})

    def steps(self) -> dict:
        return dict(self.prefill_steps) or {self.prefill_mbt: self.prefill_step_ms}

    def prefill_rate(self, mbt: Optional[int] = None) -> float:
        """Decode demand (output tok/s) one prefill GPU creates at ``mbt`` tokens per step."""
        st = self.steps()
        if mbt is None or mbt not in st or not st[mbt]:
            return self.prefill_tok_s
        return max(1, mbt // self.prompt_len) / (st[mbt] / 1e3) * self.output_len


# Measured on one MI355X with scripts/pd_capacity.py (profiles/r2_pd_capacity.md,
# profiles/r3_pd_capacity.md).  decode_tok_s[k] = R / t(L/k layers, R rows) at the row
# count the layouts use; mixed = the 1-GPU bench.py rate and step (DP / slack filler).
CAPACITY = {
    # r3: prefill at 2048 tokens / step is as fast as 4096 (19.62 vs 19.47 prompts/s) in half the
    # step (TTFT); 2-stage replicas at 768-row microbatches (the KV pool of a 40-layer stage holds
    # ~1800 full sequences), whole-model decode GPUs at 576 rows (their pool holds ~610).
    # Re-measured after the ping-pong MFMA GEMM + tile-aligned mixed steps
    # (profiles/r3_gemm/pd_capacity_70b.jsonl, bench70b_token_align256.json): the mixed (DP) GPU
    # gained 5.5 % (1760 -> 1857 tok/s), the prefill and decode roles ~1 %.
    # r5 (profiles/r5_pd/probe70b_r5.json): start-up probe on one MI355X — prefill at 2048 and
    # 1024 tokens per step, decode replicas at 576 / 768-row microbatches; the mixed (DP) rate and
    # step are the 1-GPU bench's (1,871 tok/s, 204.7 ms: the probe's short-model extrapolation
    # reads mixed steps ~5 % fast).  Re-probed with 256-row-aligned decode microbatches, median of
    # two runs on one box (profiles/r5_pd/probe70b_s23_run1/2.log): 512 rows cost 1.91 us per row
    # per layer against 2.02-2.20 at 576 (past the 512-row GEMM tile step) and 1.86 at 768; a
    # whole-model decode GPU's KV pool holds ~590 sequences, a 2-stage replica's stage ~1,790
    # (``decode_pool_seqs``), so 1,024-row microbatches fit no layout.
    "llama3-70b": RoleCapacity(prefill_tok_s=2588.6, decode_tok_s={1: 6381.5, 2: 13138.4, 3: 19707.6},
                               mixed_tok_s=1871.0, prefill_step_ms=197.8, prefill_mbt=2048,
                               decode_step_ms={1: 80.2, 2: 58.5, 3: 39.0}, decode_rows={1: 512, 2: 768, 3: 768},
                               mixed_step_ms=204.7, prefill_steps={2048: 197.8, 1024: 106.0},
                               decode_options={1: [[512, 6381.5, 80.2], [576, 5837.7, 98.8]],
                                               2: [[512, 12762.9, 40.1], [576, 11675.3, 49.4],
                                                   [768, 13138.4, 58.5]],
                                               3: [[512, 19144.4, 26.7], [576, 17513.0, 33.0],
                                                   [768, 19707.6, 39.0]]}),
    "llama3-8b": RoleCapacity(prefill_tok_s=176.2 * 128, decode_tok_s={1: 31566.0, 2: 58028.0, 3: 69373.0},
                              mixed_tok_s=11842.0, prefill_step_ms=45.4, prefill_mbt=4096,
                              decode_step_ms={1: 32.4, 2: 18.2, 3: 11.2}, decode_rows={1: 1024, 2: 1024, 3: 768},
                              mixed_step_ms=30.6),
}


HBM_BYTES = 288e9           # one MI355X


def decode_pool_seqs(model: str, stages: int, prompt_len: int = 512, output_len: int = 128,
                     hbm_bytes: float = HBM_BYTES, kv_fraction: float = 0.9, workspace: float = 8 * 2 ** 30,
                     block_size: int = 16) -> Optional[int]:
    """Full-length sequences one stage of a ``stages``-deep decode replica keeps in its KV pool
    (as ``engine.engine_block_budget`` sizes it: ``kv_fraction`` of HBM after the stage's bf16
    weights and the workspace).  A replica holds its k microbatches in every stage, so k x rows
    must fit; None for a model without a config."""
    from dgi.models.config import get_config
    try:
        mc = get_config(model.split("@")[0])
    except Exception:       # noqa: BLE001 - unknown model: no constraint
        return None
    L = mc.num_layers
    layers = -(-L // stages)
    weights = 2.0 * mc.param_count() * layers / L
    pool = max(0.0, hbm_bytes - weights - workspace) * kv_fraction
    pages = -(-(prompt_len + output_len) // block_size)
    per_seq = pages * block_size * mc.kv_bytes_per_token(layers=layers)
    return int(pool // per_seq)


_MEASURED: dict = {}     # model -> RoleCapacity measured at start-up (dgi.parallel.probe)


def set_capacity(model: str, cap: Optional[RoleCapacity]) -> None:
    """Plan ``model`` with ``cap`` (this node's start-up probe) instead of the table."""
    key = model.split("@")[0] if model else model
    if cap is None:
        _MEASURED.pop(key, None)
    else:
        _MEASURED[key] = cap


def capacity_for(model: str) -> Optional[RoleCapacity]:
    """This node's measured capacity of ``model`` if the start-up probe ran, else the
    table entry; a layer-truncated rehearsal name (``llama3-70b@L8``) plans like the
    full model it stands in for."""
    key = model.split("@")[0] if model else model
    return _MEASURED.get(key) or CAPACITY.get(key)


def estimate_layout(n_prefill: int, stages: int, replicas: int, cap: RoleCapacity, fill: bool = False) -> float:
    """Node output tok/s of nP + replicas x (stages-deep decode) under ``cap``:
    the slower side sets the rate.  ``fill`` adds the slack filler the
    runtime uses (decode replicas admit local prompts; prefill ranks decode
    overflow sequences) at the mixed-step rate — an upper bound."""
    pre = n_prefill * cap.prefill_tok_s
    dec = replicas * cap.decode_tok_s.get(stages, 0.0)
    if pre <= 0 or dec <= 0:
        return 0.0
    base = min(pre, dec)
    if not fill:
        return base
    if dec >= pre:
        return base + (1.0 - pre / dec) * replicas * stages * cap.mixed_tok_s
    return base + (1.0 - dec / pre) * n_prefill * cap.mixed_tok_s


def layout_estimate(n_prefill: int, stages: int, replicas: int, cap: RoleCapacity) -> dict:
    """Throughput AND latency of a P/D layout under ``cap`` (what ``bench.py --gpus N``
    reports next to its measurement).

    tok_s: with the slack filler; disagg_tok_s: without it; tpot_ms: a sequence
    decoded on a replica (k stage steps per token); ttft_ms: one prefill step
    (prompts admitted just in time); filler_share: fraction of the output the
    filler (mixed steps, DP-like TPOT) produces."""
    pre = n_prefill * cap.prefill_tok_s
    dec = replicas * cap.decode_tok_s.get(stages, 0.0)
    base = min(pre, dec)
    tot = estimate_layout(n_prefill, stages, replicas, cap, fill=True)
    return {"layout": f"{n_prefill}P+{replicas}D[" + "+".join([f"pp{stages}" if stages > 1 else "1"] * replicas) + "]",
            "tok_s": round(tot, 1), "disagg_tok_s": round(base, 1),
            "bound": "prefill" if pre < dec else "decode",
            "tpot_ms": round(stages * cap.decode_step_ms.get(stages, 0.0), 1) or None,
            "ttft_ms": round(cap.prefill_step_ms, 1) or None,
            "filler_share": round((tot - base) / tot, 3) if tot > 0 else 0.0,
            "dp_tok_s": round((n_prefill + stages * replicas) * cap.mixed_tok_s, 1),
            "dp_tpot_ms": cap.mixed_step_ms or None}


def choose_pd_layout(n_gpus: int, cap: RoleCapacity, max_stages: int = 3, prefer_pipeline: bool = True,
                     tol: float = 0.03, objective: str = "node") -> tuple:
    """(n_prefill, stages, replicas, est tok/s).

    ``objective="node"`` (default): among layouts whose replica TPOT beats a
    mixed-step (DP) GPU's, the highest disaggregated rate (the filler only tops
    a layout up towards DP and would otherwise make "1 prefill GPU + a DP node"
    look as good as any P/D split); candidates within ``tol`` of the best are
    ranked by the node rate with the filler, then by TPOT.
    ``objective="disagg"``: the round-2 rule (deeper pipelines first within ``tol``)."""
    cands = []
    for npre in range(1, n_gpus):
        left = n_gpus - npre
        for k in range(1, max_stages + 1):
            if left % k or k not in cap.decode_tok_s:
                continue
            reps = left // k
            pre, dec = npre * cap.prefill_tok_s, reps * cap.decode_tok_s[k]
            tpot = k * cap.decode_step_ms.get(k, 0.0)
            est = estimate_layout(npre, k, reps, cap)
            if objective == "node":
                beats_dp = not (cap.mixed_step_ms and tpot and tpot >= cap.mixed_step_ms)
                cands.append((est, k, npre, reps, (-estimate_layout(npre, k, reps, cap, fill=True), tpot),
                              beats_dp))
            else:
                cands.append((est, k, npre, reps, abs(pre - dec) / max(pre, dec), True))
    if any(c[5] for c in cands):
        cands = [c for c in cands if c[5]]
    top = max(c[0] for c in cands)
    near = [c for c in cands if c[0] >= (1.0 - tol) * top]
    if objective == "node":
        near.sort(key=lambda c: (c[4], -c[0]))
    else:
        near.sort(key=lambda c: ((-c[1] if prefer_pipeline else c[1]), c[4], -c[0]))
    est, k, npre, reps = near[0][:4]
    return npre, k, reps, est


# P/D planning objective: the disaggregated layout exists for latency at throughput
# parity — on a compute-bound GPU it cannot out-run data parallel.  Among P/D candidates whose
# TTFT AND TPOT are at most LATENCY_FRAC of a data-parallel GPU's, the highest node rate (the
# slack filler counted at FILL_WEIGHT: it runs mixed steps with DP-like latency); the pick runs
# unless its rate falls below PD_MIN_RATIO x data parallel.
LATENCY_FRAC = float(os.environ.get("DGI_PD_LATENCY_FRAC", "0.7"))
FILL_WEIGHT = 0.8
# estimates within TOK_TIE of the fastest count as tied (the latency decides): the start-up
# probe's own run-to-run spread on one box is ~3 % (profiles/r5_pd/probe70b_s23_run1/2.log:
# 8-GPU estimates 13.70k / 14.10k tok/s)
TOK_TIE = float(os.environ.get("DGI_PD_TOK_TIE", "0.02"))
# 0.85: below the ~0.9 x DP the kernels allow a P/D node on 70B (a decode row costs 1.86 us per
# layer vs a mixed row's 1.33: profiles/r5_pd/README.md) and below the start-up probe's ~5 %
# optimism about DP mixed steps
PD_MIN_RATIO = float(os.environ.get("DGI_PD_MIN_RATIO", "0.85"))
# a split that needs the slack filler for more than this share of its output is a DP-like hybrid
# (2-4 GPUs of 70B: ~30 %), not disaggregation: data parallel runs there
MAX_FILLER_SHARE = float(os.environ.get("DGI_PD_MAX_FILLER", "0.15"))


def dp_reference(n_gpus: int, cap: RoleCapacity) -> dict:
    """N data-parallel GPUs under ``cap``: every token waits one mixed step (TTFT ~ TPOT ~ step)."""
    return {"layout": f"dp{n_gpus}", "tok_s": round(n_gpus * cap.mixed_tok_s, 1),
            "ttft_ms": cap.mixed_step_ms or None, "tpot_ms": cap.mixed_step_ms or None}


def pd_candidate(n_prefill: int, stages: int, replicas: int, mbt: int, cap: RoleCapacity) -> dict:
    """Rate and latency of nP (``mbt``-token prefill steps) + replicas x (stages-deep decode)."""
    pre = n_prefill * cap.prefill_rate(mbt)
    dec = replicas * cap.decode_tok_s.get(stages, 0.0)
    base = min(pre, dec)
    if dec >= pre:        # decode slack: replicas admit local prompts (mixed microbatches)
        fill = (1.0 - pre / dec) * replicas * stages * cap.mixed_tok_s if dec > 0 else 0.0
    else:                 # prefill slack: prefill ranks decode overflow sequences themselves
        fill = (1.0 - dec / pre) * n_prefill * cap.mixed_tok_s
    tot = base + FILL_WEIGHT * fill
    share = FILL_WEIGHT * fill / tot if tot > 0 else 0.0
    ttft = round(cap.steps().get(mbt, cap.prefill_step_ms), 1) or None
    tpot = round(stages * cap.decode_step_ms.get(stages, 0.0), 1) or None
    # latency of the filler's tokens: overflow sequences decoded on a prefill
    # rank wait one prefill step per token; local prompts of a decode replica run in mixed
    # microbatches at DP-like latency.  Node-wide p95 over tokens: the filler's latency once its
    # share of the output reaches 5 %.
    if dec >= pre:
        f_tpot = f_ttft = cap.mixed_step_ms or None
    else:
        f_tpot, f_ttft = ttft, ttft
    def _p95(main, other):       # noqa: E306
        if main is None:
            return None
        return round(max(main, other), 1) if (other and share >= 0.05) else main
    def _mean(main, other):      # noqa: E306
        if main is None:
            return None
        return round((1.0 - share) * main + share * (other or main), 1)
    return {"layout": f"{n_prefill}P+{replicas}D[" + "+".join([f"pp{stages}" if stages > 1 else "1"] * replicas) + "]",
            "prefill_ranks": n_prefill, "decode_stages": stages, "decode_replicas": replicas, "prefill_mbt": mbt,
            "tok_s": round(tot, 1), "disagg_tok_s": round(base, 1),
            "bound": "prefill" if pre < dec else "decode",
            "ttft_ms": ttft, "tpot_ms": tpot,          # a prompt / sequence of the disaggregated path
            "tpot_replica_ms": tpot,
            "filler_tpot_ms": f_tpot if share > 0 else None, "filler_ttft_ms": f_ttft if share > 0 else None,
            "tpot_mean_ms": _mean(tpot, f_tpot), "tpot_p95_ms": _p95(tpot, f_tpot),
            "ttft_mean_ms": _mean(ttft, f_ttft), "ttft_p95_ms": _p95(ttft, f_ttft),
            "filler_share": round(share, 3)}


def plan_pd(n_gpus: int, cap: RoleCapacity, max_stages: int = 3, lat_frac: Optional[float] = None) -> tuple:
    """(best P/D candidate, DP reference, every candidate): see LATENCY_FRAC above.  Without a
    candidate meeting the latency bound the fastest candidate is returned with
    ``latency_ok`` False."""
    lat = LATENCY_FRAC if lat_frac is None else lat_frac
    dp = dp_reference(n_gpus, cap)
    cands = []
    for npre in range(1, n_gpus):
        left = n_gpus - npre
        for k in range(1, max_stages + 1):
            if left % k:
                continue
            # the decode microbatch size is a planner output too: every measured row count
            for rows, ts, st in cap.decode_choices(k):
                ck = cap.with_decode(k, rows, ts, st)
                for mbt in sorted(cap.steps()):
                    c = pd_candidate(npre, k, left // k, mbt, ck)
                    c["decode_rows"] = rows
                    # the bound holds for the filler-inclusive p95, not only the replica's TPOT
                    c["latency_ok"] = bool(dp["ttft_ms"] and c["ttft_p95_ms"] and c["tpot_p95_ms"]
                                           and c["ttft_p95_ms"] <= lat * dp["ttft_ms"]
                                           and c["tpot_p95_ms"] <= lat * dp["tpot_ms"])
                    cands.append(c)
    if not cands:
        return None, dp, []
    ok = [c for c in cands if c["latency_ok"]] or cands
    # the fastest, unless a candidate within TOK_TIE of its rate cuts the TPOT by >= 10 %: then the
    # fastest of those (a 512-row decode microbatch at the rate of a 768-row one is 2/3 the TPOT)
    key = lambda c: (c["tok_s"], -(c["tpot_ms"] or 0), -(c["ttft_ms"] or 0))     # noqa: E731
    best = max(ok, key=key)
    better = [c for c in ok if c["tok_s"] >= (1.0 - TOK_TIE) * best["tok_s"]
              and (c["tpot_ms"] or 0) <= 0.9 * (best["tpot_ms"] or 0)]
    if better:
        best = max(better, key=key)
    best = dict(best, vs_dp=round(best["tok_s"] / dp["tok_s"], 3) if dp["tok_s"] else None)
    return best, dp, cands


def _groups(first: int, stages: int, replicas: int) -> list:
    return [list(range(first + i * stages, first + (i + 1) * stages)) for i in range(replicas)]


def plan_node_layout(n_gpus: int, kind: str = "pdpp", prefill_ranks: Optional[int] = None,
                     decode_stages: Optional[int] = None, decode_replicas: Optional[int] = None,
                     model: str = "llama3-70b") -> NodeLayout:
    """Assign the node's GPUs to roles.

    ``pd``/``pdpp`` without explicit counts pick the split from the measured
    per-role capacity table (``CAPACITY``, ``choose_pd_layout``): e.g. on
    Llama-3-70B at 8 GPUs the estimate favours 5 prefill GPUs feeding one
    3-stage decode pipeline (``pdpp``) or three whole-model decode GPUs
    (``pd``); below 8, N-1 prefill GPUs feed one decode GPU.  Models without a
    table entry fall back to N-1 prefill ranks + one decode GPU."""
    if n_gpus == 1 or kind == "single":
        return NodeLayout("single", [], [0])
    if kind == "pp":
        return NodeLayout("pp", [], list(range(n_gpus)))
    if kind == "dp":
        return NodeLayout("dp", [], [0], replicas=n_gpus)
    cap = capacity_for(model)
    if decode_stages is None and kind == "pd":
        decode_stages = 1
    if prefill_ranks is None and decode_replicas is None and cap is not None and \
            (decode_stages is None or kind == "pd"):
        best, _dp, _c = plan_pd(n_gpus, cap, max_stages=decode_stages or 3)
        npre, k, reps = best["prefill_ranks"], best["decode_stages"], best["decode_replicas"]
    else:
        k = decode_stages or (3 if (kind == "pdpp" and n_gpus >= 8) else 1)
        reps = decode_replicas
        npre = prefill_ranks
        if npre is None:
            reps = reps or 1
            npre = n_gpus - k * reps
        if reps is None:
            reps = max(1, (n_gpus - npre) // k)
    npre = max(1, min(npre, n_gpus - k))
    reps = max(1, min(reps, (n_gpus - npre) // k))
    npre = n_gpus - k * reps
    groups = _groups(npre, k, reps)
    if k > 2:      # consecutive stages on the cheapest links (identity on a full xGMI mesh)
        from dgi.parallel.topology import order_stages, read_topology
        topo = read_topology() if os.environ.get("DGI_SHARED_GPU", "0") != "1" else None
        groups = [order_stages(topo, g) for g in groups]
    return NodeLayout("pdpp" if k > 1 else "pd", list(range(npre)), groups)


def prefill_overflow_cap(layout: NodeLayout, cap: int = 256, model: str = "llama3-70b") -> int:
    """Sequences a prefill rank may decode itself while the decode side has no
    credit (``PrefillServer(local_cap=...)``): on when the decode side is the
    bottleneck of the capacity estimate (e.g. 70B with 3 prefill GPUs per
    decode GPU: each prefill GPU supplies ~2.5k tok/s, a decode GPU absorbs
    ~4.6k — profiles/r1_pd_capacity_70b.md)."""
    c = capacity_for(model)
    if c is None:
        return cap if layout.kind == "pd" and len(layout.prefill_ranks) >= 2 else 0
    k = len(layout.decode_groups[0])
    pre = len(layout.prefill_ranks) * c.prefill_tok_s
    dec = len(layout.decode_groups) * c.decode_tok_s.get(k, 0.0)
    return cap if pre > dec * 1.05 else 0


def decode_local_fraction(layout: NodeLayout, model: str = "llama3-70b") -> float:
    """Share of a decode replica's KV pool for prompts it admits itself (hybrid
    decode) when the prefill side cannot saturate it."""
    c = capacity_for(model)
    if c is None:
        return {1: 0.35, 2: 0.15}.get(len(layout.prefill_ranks), 0.0) if layout.kind == "pd" else 0.0
    k = len(layout.decode_groups[0])
    pre = len(layout.prefill_ranks) * c.prefill_tok_s
    dec = len(layout.decode_groups) * c.decode_tok_s.get(k, 0.0)
    if dec <= pre * 1.05:
        return 0.0
    return round(min(0.5, 1.0 - pre / dec), 3)
