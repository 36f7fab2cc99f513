"""Step-phase tracing for the dgi runtime.

``phase(name)`` marks one phase of an engine iteration (schedule, forward,
apply, migrate, ...) three ways, each off unless asked for:

* **roctx ranges** (``DGI_TRACE=roctx``): ``torch.cuda.nvtx`` is backed by
  roctx on ROCm, so ``rocprofv3 --marker-trace`` (or ``--kernel-trace`` plus
  the marker domain) lines the HIP kernels up under the phase that launched
  them;
* **OpenTelemetry spans** (``set_tracer``): the control plane's
  ``TracingManager`` — the worker installs it when
  ``observability.tracing.enabled``;
* **host timers** (always on, ~0.3 us per phase): cumulative seconds and
  counts per phase in ``PHASE_STATS`` for ``/status`` and the bench JSON.
"""
from __future__ import annotations

import os
import time
from contextlib import contextmanager
from typing import Optional

_MODE = os.environ.get("DGI_TRACE", "").lower()
_ROCTX = _MODE in ("roctx", "1", "all")
_tracer = None
PHASE_STATS: dict = {}


def set_tracer(tracer) -> None:
    """Route phases into a ``TracingManager`` (OpenTelemetry) as well."""
    global _tracer
    _tracer = tracer


def enable_roctx(on: bool = True) -> None:
    global _ROCTX
    _ROCTX = on


def _push(name: str) -> bool:
    if not _ROCTX:
        return False
    try:
        import torch
        torch.cuda.nvtx.range_push(name)
        return True
    except Exception:
        return False


def _pop() -> None:
    try:
        import torch
        torch.cuda.nvtx.range_pop()
    except Exception:
        pass


@contextmanager
def phase(name: str, **attrs):
    pushed = _push(name)
    span_cm = _tracer.span(f"dgi.{name}", attrs or None) if _tracer is not None else None
    if span_cm is not None:
        span_cm.__enter__()
    t0 = time.perf_counter()
    try:
        yield
    finally:
        dt = time.perf_counter() - t0
        st = PHASE_STATS.get(name)
        if st is None:
            PHASE_STATS[name] = [dt, 1]
        else:
            st[0] += dt
            st[1] += 1
        if span_cm is not None:
            span_cm.__exit__(None, None, None)
        if pushed:
            _pop()


def phase_summary(reset: bool = False) -> dict:
    """{phase: {"s": total seconds, "n": count, "ms_avg": mean ms}}."""
    out = {k: {"s": round(v[0], 4), "n": v[1], "ms_avg": round(v[0] / max(1, v[1]) * 1000, 3)}
           for k, v in PHASE_STATS.items()}
    if reset:
        PHASE_STATS.clear()
    return out


def mark(name: str, value: Optional[float] = None) -> None:
    """A zero-length roctx marker (e.g. a migration landing)."""
    if _ROCTX:
        try:
            import torch
            torch.cuda.nvtx.mark(name if value is None else f"{name}={value}")
        except Exception:
            pass
