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
    kind: str                      # single | dp | pp | pd | pdpp
    prefill_ranks: list
    decode_ranks: list             # decode pipeline stages in order (len 1 = no PP)
    replicas: int = 1

    @property
    def world(self) -> int:
        return len(self.prefill_ranks) + len(self.decode_ranks)

    def role(self, rank: int) -> str:
        if rank in self.prefill_ranks:
            return "prefill"
        if self.decode_ranks and rank == self.decode_ranks[0]:
            return "decode_driver"
        return "decode_stage"


def plan_node_layout(n_gpus: int, kind: str = "pdpp", prefill_ranks: Optional[int] = None,
                     decode_stages: Optional[int] = None) -> NodeLayout:
    """Default P:D split for prefill-heavy loads (512-in/128-out on 70B).

    Measured on one MI355X (scripts/pd_capacity.py, profiles/r1_pd_capacity_70b.md):
    a prefill GPU turns 19.3 prompts/s (4096-token steps) = 2.47k output tok/s of
    decode demand; a full-model decode GPU steps 512 rows in 111 ms (4.6k tok/s,
    KV-capped near 640 sequences); a 40-layer stage steps 512 / 1024 / 1536 rows
    in 56 / 89 / 129 ms.  An S-stage decode pipeline with S microbatches of R
    rows emits R / t_stage(R) tok/s: 2 stages top out near 11.9k, 3 stages
    (~27 layers each) reach ~15k at R = 768.  So at 8 GPUs 5 prefill GPUs
    (12.4k demand) feed a 3-stage decode pipeline; below 8, N-1 prefill GPUs
    feed one decode GPU."""
    if n_gpus == 1 or kind == "single":
        return NodeLayout("single", [], [0])
    if kind == "pp":
        return NodeLayout("pp", [], list(range(n_gpus)))
    if kind == "dp":
        return NodeLayout("dp", [], [0], replicas=n_gpus)
    if decode_stages is None:
        decode_stages = 3 if (kind == "pdpp" and n_gpus >= 8) else 1
    if prefill_ranks is None:
        prefill_ranks = n_gpus - decode_stages
    prefill_ranks = max(1, min(prefill_ranks, n_gpus - decode_stages))
    decode_stages = n_gpus - prefill_ranks
    k = "pdpp" if decode_stages > 1 else "pd"
    return NodeLayout(k, list(range(prefill_ranks)), list(range(prefill_ranks, n_gpus)))


def prefill_overflow_cap(layout: NodeLayout, cap: int = 256) -> int:
    """Sequences a prefill rank may decode itself while the decode side has no
    credit (``PrefillServer(local_cap=...)``).  On for one decode GPU fed by 2+
    prefill GPUs — that decode GPU saturates at ~4.6k tok/s on 70B while each
    prefill GPU supplies ~2.5k (profiles/r1_pd_capacity_70b.md) — off where the
    prefill side is the bottleneck (1 prefill GPU, or the 8-GPU 5P + 3-stage
    decode pipeline)."""
    return cap if layout.kind == "pd" and len(layout.prefill_ranks) >= 2 else 0
