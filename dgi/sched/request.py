"""Request and sampling parameter objects of the iteration-level scheduler."""
from __future__ import annotations

import dataclasses
import enum
import itertools
import time
from typing import Optional

_rid = itertools.count()


@dataclasses.dataclass
class SamplingParams:
    """Defaults follow the reference's GenerationConfig (worker/engines/llm_base.py:23-31)."""
    max_tokens: int = 2048
    temperature: float = 0.7
    top_p: float = 0.9
    top_k: int = 50
    stop_token_ids: tuple = ()
    ignore_eos: bool = False
    seed: Optional[int] = None

    @property
    def greedy(self) -> bool:
        return self.temperature <= 1e-5

    @property
    def needs_filter(self) -> bool:
        return not self.greedy and ((0 < self.top_k) or (self.top_p < 1.0))


class Status(enum.Enum):
    WAITING = "waiting"
    RUNNING = "running"
    FINISHED = "finished"


class Request:
    __slots__ = ("rid", "prompt", "params", "output", "blocks", "num_computed", "num_cached", "status",
                 "arrival", "first_token_time", "finish_time", "finish_reason", "radix_path", "seed",
                 "token_times", "user", "preempted", "hidden", "spec_state", "prefill_target", "busy", "swapped", "kv_ready")

    def __init__(self, prompt: list[int], params: SamplingParams, rid=None, user=None):
        self.rid = next(_rid) if rid is None else rid
        self.prompt = list(prompt)
        self.params = params
        self.output: list[int] = []
        self.blocks: list[int] = []
        self.num_computed = 0      # tokens whose KV is in the cache
        self.num_cached = 0        # prompt tokens served by the prefix cache
        self.status = Status.WAITING
        self.arrival = time.perf_counter()
        self.first_token_time: Optional[float] = None
        self.finish_time: Optional[float] = None
        self.finish_reason: Optional[str] = None
        self.radix_path: list = []
        self.seed = params.seed if params.seed is not None else (hash((self.rid, 0x5eed)) & 0x7FFFFFFF)
        self.token_times: list[float] = []
        self.user = user
        self.preempted = 0
        self.hidden = None
        self.spec_state = None
        self.prefill_target = len(self.prompt)  # tokens to (re)compute before sampling
        self.busy = False  # in flight in a pipeline microbatch
        # while preempted to the pinned host KV tier: (host slots, tokens, None), or
        # (None, tokens, GPU pages) once the scheduler restored it one step ahead
        self.swapped = None
        self.kv_ready = None  # event of a host-tier restore of its pages, awaited by its first forward

    @property
    def total_len(self) -> int:
        return len(self.prompt) + len(self.output)

    def all_tokens(self) -> list[int]:
        return self.prompt + self.output

    def sample_seed(self, ahead: int = 0) -> int:
        """Seed of the next sampled token: a function of the request alone (its seed
        and how many tokens it has produced, ``ahead`` of them still in flight), so a
        seeded request draws the same tokens whatever the batching, the engine's step
        count or the parallel layout (single GPU, pipeline, P/D, graph or eager)."""
        return (self.seed * 1000003 + len(self.output) + ahead) & 0x7FFFFFFF

    @property
    def in_prefill(self) -> bool:
        return self.num_computed < self.prefill_target

    @property
    def ttft(self) -> Optional[float]:
        return None if self.first_token_time is None else self.first_token_time - self.arrival
