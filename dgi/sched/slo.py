"""TPOT-SLO step budget for mixed prefill + decode steps.

In a mixed (continuous-batching) step every running sequence gets one token, so
a decode token waits one whole step: TPOT ~ step time.  A step's time grows
with its row count (the projection GEMMs dominate: ~0.1 ms per row on a 70B
MI355X step), so the knob that trades throughput for TPOT is how many prefill
tokens a step may carry.  ``StepBudget`` learns this GPU's cost per row from the
steps the engine ran (an EMA of wall ms / rows over steps with enough rows to be
GEMM-bound) and caps the next step's rows at ``tpot_slo_ms / cost``, leaving
every decode row in and at least ``min_prefill`` prefill tokens so new requests
keep moving.  The reference maps this to ``chunked_prefill_size``
(worker/engines/llm_sglang.py:64) — a fixed token count; here it is a latency
target the budget follows as the load changes.
"""
from __future__ import annotations

from typing import Optional


class StepBudget:
    def __init__(self, tpot_slo_ms: float, min_prefill: int = 128, alpha: float = 0.2, min_rows: int = 256):
        self.slo = float(tpot_slo_ms)
        self.min_prefill = int(min_prefill)
        self.alpha = alpha
        self.min_rows = min_rows
        self.ms_per_row: Optional[float] = None
        self.steps = 0
        self.capped = 0

    def observe(self, rows: int, ms: float) -> None:
        """One executed step: ``rows`` tokens through the model in ``ms`` wall ms."""
        if rows < self.min_rows or ms <= 0:
            return
        c = ms / rows
        self.ms_per_row = c if self.ms_per_row is None else (1 - self.alpha) * self.ms_per_row + self.alpha * c
        self.steps += 1

    def budget(self, max_tokens: int, decode_rows: int) -> int:
        """Token budget of the next step (decode rows included)."""
        if self.ms_per_row is None or self.slo <= 0:
            return max_tokens
        rows = int(self.slo / self.ms_per_row)
        b = min(max_tokens, max(rows, decode_rows + self.min_prefill))
        if b < max_tokens:
            self.capped += 1
        return b

    def stats(self) -> dict:
        return {"tpot_slo_ms": self.slo, "ms_per_row": None if self.ms_per_row is None else round(self.ms_per_row, 5),
                "budget_rows": None if self.ms_per_row is None else int(self.slo / self.ms_per_row),
                "steps_observed": self.steps, "steps_capped": self.capped}
