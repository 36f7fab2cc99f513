"""Step-phase tracing (dgi.utils.trace): host timers, OTel span routing, roctx toggling."""
from unittest.mock import MagicMock

from dgi.utils import trace


def test_phase_timers_and_summary():
    trace.PHASE_STATS.clear()
    for _ in range(3):
        with trace.phase("unit_a"):
            pass
    s = trace.phase_summary(reset=True)
    assert s["unit_a"]["n"] == 3 and s["unit_a"]["s"] >= 0
    assert trace.PHASE_STATS == {}


def test_phases_become_spans_when_a_tracer_is_set():
    span = MagicMock()
    tm = MagicMock()
    tm.span.return_value = span
    trace.set_tracer(tm)
    try:
        with trace.phase("unit_b", rows=4):
            pass
    finally:
        trace.set_tracer(None)
    tm.span.assert_called_once_with("dgi.unit_b", {"rows": 4})
    span.__enter__.assert_called_once()
    span.__exit__.assert_called_once()


def test_roctx_toggle_is_safe_without_gpu():
    trace.enable_roctx(True)
    try:
        with trace.phase("unit_c"):
            trace.mark("m", 1)
    finally:
        trace.enable_roctx(False)


def test_engine_step_reports_phases():
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.sched.request import SamplingParams
    trace.PHASE_STATS.clear()
    e = LLMEngine(EngineConfig(model="llama-tiny", device="cpu", num_blocks=64, max_num_seqs=2, max_model_len=128,
                               max_num_batched_tokens=64, use_graphs=False))
    e.generate([[1, 2, 3]], SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True))
    s = trace.phase_summary()
    assert {"schedule", "execute", "apply"} <= set(s) and s["execute"]["n"] == 3
