"""TPOT-SLO step budget and admission cap for mixed prefill + decode steps.

In a mixed (continuous-batching) step every running sequence gets one token, so
a decode token waits one whole step: TPOT ~ step time.  A step's time grows
with its row count (the projection GEMMs dominate: ~0.1 ms per row on a 70B
MI355X step), so the knob that trades throughput for TPOT is how many rows a
step may carry.  ``StepBudget`` learns this GPU's step cost as a line,
``ms = fixed + per_row * rows``, fitted over a window of the prefill / mixed
steps the engine ran, and caps the next step's rows at the row count whose
predicted time meets ``tpot_slo_ms`` — every decode row stays in, plus at least
``min_prefill`` prefill tokens so new requests keep moving.

The fit is a Theil-Sen line (median of pairwise slopes) over the last
``window`` steps of ANY row count, capped steps included: one slow step (cold
start, a lazy allocation, a clock transition) is outvoted by the next few
instead of pinning the budget low for the life of the engine (the
round-4 EMA only learned from >= 256-row steps, and once a pessimistic estimate
capped steps below that it never observed a step again).

Admission: a step budget alone caps the prefill RATE, so with a
closed-loop client the queue, and TTFT, grow without bound.  ``admission_cap``
turns the budget into the number of sequences the engine can keep running at
the SLO: in steady state a request spends ``prompt`` prefill rows and
``output`` decode rows, so a step of R rows carries R * output / (prompt +
output) decode rows, plus the prompts being prefilled.  The engine admits up to
that many (``Scheduler.admit_cap``) and a client can size its load to it.  The
reference maps the two knobs to ``chunked_prefill_size`` and
``max_running_requests`` (worker/engines/llm_sglang.py:61-66) — fixed counts;
here both follow a latency target as the measured cost changes.
"""
from __future__ import annotations

import collections
import statistics
from typing import Optional


class StepBudget:
    def __init__(self, tpot_slo_ms: float, min_prefill: int = 128, window: int = 24, min_spread: int = 16):
        self.slo = float(tpot_slo_ms)
        self.min_prefill = int(min_prefill)
        self.samples: collections.deque = collections.deque(maxlen=window)
        self.min_spread = min_spread
        self.fixed_ms = 0.0
        self.ms_per_row: Optional[float] = None
        self.steps = 0
        self.capped = 0
        # mean prompt / output length of finished requests (the load shape for admission)
        self.prompt_avg: Optional[float] = None
        self.output_avg: Optional[float] = None
        self.n_finished = 0

    # ------------------------------------------------------------------ cost model
    def observe(self, rows: int, ms: float) -> None:
        """One executed step: ``rows`` tokens through the model in ``ms`` wall ms."""
        if rows <= 0 or ms <= 0:
            return
        self.samples.append((int(rows), float(ms)))
        self.steps += 1
        self._fit()

    def _fit(self) -> None:
        xs = list(self.samples)
        slopes = [(y1 - y0) / (x1 - x0) for i, (x0, y0) in enumerate(xs) for (x1, y1) in xs[i + 1:]
                  if abs(x1 - x0) >= self.min_spread]
        if slopes:
            b = max(1e-6, statistics.median(slopes))
            a = max(0.0, statistics.median([y - b * x for x, y in xs]))
        else:       # no row-count spread yet: a line through the origin (over-estimates: safe side)
            a, b = 0.0, statistics.median([y / x for x, y in xs])
        self.fixed_ms, self.ms_per_row = a, b

    def predict_ms(self, rows: int) -> Optional[float]:
        if self.ms_per_row is None:
            return None
        return self.fixed_ms + self.ms_per_row * rows

    def rows_at_slo(self) -> Optional[int]:
        if self.ms_per_row is None or self.slo <= 0:
            return None
        return max(1, int((self.slo - self.fixed_ms) / self.ms_per_row))

    def budget(self, max_tokens: int, decode_rows: int) -> int:
        """Token budget of the next step (decode rows included)."""
        rows = self.rows_at_slo()
        if rows is None:
            return max_tokens
        b = min(max_tokens, max(rows, decode_rows + self.min_prefill))
        if b < max_tokens:
            self.capped += 1
        return b

    # ------------------------------------------------------------------ admission
    def observe_request(self, prompt_len: int, max_tokens: int) -> None:
        """A request arrived: until requests finish, its prompt length and ``max_tokens`` are
        the load shape (so the admission cap holds from the first steps on — a closed-loop
        client that filled the engine before it was known would queue for a whole
        generation's worth of steps)."""
        if self.n_finished == 0:
            self._blend(prompt_len, max_tokens)

    def observe_finished(self, prompt_len: int, output_len: int) -> None:
        self.n_finished += 1
        self._blend(prompt_len, output_len)

    def _blend(self, prompt_len: int, output_len: int, alpha: float = 0.1) -> None:
        if self.prompt_avg is None:
            self.prompt_avg, self.output_avg = float(prompt_len), float(output_len)
        else:
            self.prompt_avg += alpha * (prompt_len - self.prompt_avg)
            self.output_avg += alpha * (output_len - self.output_avg)

    def admission_cap(self, max_tokens: int, prompt_len: Optional[float] = None,
                      output_len: Optional[float] = None) -> Optional[int]:
        """Running sequences the engine sustains at the SLO (None until both the cost and
        the load shape are known): decode rows of an SLO-sized step plus the prompts it
        prefills."""
        rows = self.rows_at_slo()
        p = prompt_len if prompt_len is not None else self.prompt_avg
        o = output_len if output_len is not None else self.output_avg
        if rows is None or not p or not o:
            return None
        rows = min(rows, max_tokens)
        dec = rows * o / (p + o)
        prompts = max(1.0, (rows - dec) / p)
        return max(1, int(dec + prompts + 0.5))

    def stats(self) -> dict:
        rows = self.rows_at_slo()
        return {"tpot_slo_ms": self.slo, "ms_per_row": None if self.ms_per_row is None else round(self.ms_per_row, 5),
                "fixed_ms": round(self.fixed_ms, 3), "budget_rows": rows, "steps_observed": self.steps,
                "steps_capped": self.capped,
                "admission_cap": self.admission_cap(1 << 30)}
