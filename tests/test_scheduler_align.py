"""Tile-aligned mixed steps (SchedulerConfig.token_align): with decode rows plus
waiting prompts worth more than one tile, the step's row count is rounded down
to a multiple of the tile and the rest of the prefill runs in a later step; no
prefill token is dropped or duplicated, and every prompt still completes."""
import torch

from dgi.kv.block_pool import BlockPool
from dgi.sched.request import Request, SamplingParams
from dgi.sched.scheduler import Scheduler, SchedulerConfig


def _sched(align):
    pool = BlockPool(6000, 16, num_layers=1, num_kv_heads=1, head_dim=8, dtype=torch.float32, device="cpu")
    return Scheduler(pool, SchedulerConfig(max_num_seqs=512, max_num_batched_tokens=4096, max_model_len=2048,
                                           enable_prefix_caching=False, token_align=align))


def _decoding(s, n, plen=16):
    """n running sequences already past their prefill (one decode row each)."""
    for _ in range(n):
        r = Request(list(range(1, plen + 1)), SamplingParams(max_tokens=64))
        r.output.append(7)
        s.add_prefilled(r, s.pool.allocate(2))


def _apply(s, batch):
    for c in batch.prefill:
        c.req.num_computed += c.length
        if c.sample:
            c.req.output.append(7)
    for r in batch.decode:
        r.num_computed += 1
        r.output.append(7)


def test_mixed_step_rounds_down_to_the_tile():
    s = _sched(256)
    _decoding(s, 381)
    for _ in range(3):
        s.add(Request(list(range(1, 513)), SamplingParams(max_tokens=8)))
    b = s.schedule()
    assert len(b.decode) == 381
    assert b.num_tokens == 1792                     # 381 + 1536 = 1917 -> 7 tiles
    assert sum(c.length for c in b.prefill) == 1792 - 381


def test_deferred_prefill_completes_and_steps_stay_aligned():
    s = _sched(256)
    _decoding(s, 381)
    prompts = [Request(list(range(1, 513)), SamplingParams(max_tokens=8)) for _ in range(9)]
    for r in prompts:
        s.add(r)
    done = 0
    for _ in range(12):
        b = s.schedule()
        if b.empty:
            break
        if b.prefill and b.num_tokens > 256:
            # aligned, unless rounding down would leave no room for any prefill row
            assert b.num_tokens % 256 == 0 or len(b.decode) >= b.num_tokens // 256 * 256
        done += sum(c.length for c in b.prefill)
        _apply(s, b)
    assert done == 9 * 512
    assert all(not r.in_prefill and r.output for r in prompts)


def test_small_steps_and_align_off_unchanged():
    s = _sched(256)
    _decoding(s, 10)
    s.add(Request(list(range(1, 101)), SamplingParams(max_tokens=8)))
    assert s.schedule().num_tokens == 110          # one tile or less: no rounding
    s0 = _sched(0)
    _decoding(s0, 381)
    for _ in range(3):
        s0.add(Request(list(range(1, 513)), SamplingParams(max_tokens=8)))
    assert s0.schedule().num_tokens == 1917


def test_pure_prefill_steps_are_not_rounded():
    """A prefill-only step (P/D prefill rank, idle engine) keeps every waiting token:
    deferring part of a prompt would cost it a whole step of TTFT."""
    s = _sched(256)
    for _ in range(3):
        s.add(Request(list(range(1, 301)), SamplingParams(max_tokens=8)))
    assert s.schedule().num_tokens == 900


def test_tpot_slo_step_budget_caps_rows():
    """dgi.sched.slo.StepBudget: fits ms = fixed + per_row * rows over executed steps and
    caps the next step at the rows whose predicted time meets the SLO, never below the
    decode rows + a minimum prefill chunk."""
    from dgi.sched.slo import StepBudget
    b = StepBudget(100.0, min_prefill=128)
    assert b.budget(4096, 300) == 4096                 # nothing learned yet: no cap
    b.observe(2000, 200.0)                             # one sample: a line through the origin
    assert abs(b.ms_per_row - 0.1) < 1e-9 and b.fixed_ms == 0.0
    assert b.budget(4096, 300) == 1000 and b.capped == 1
    b.observe(1000, 110.0)                             # two samples: 20 ms fixed + 0.09 ms per row
    assert abs(b.ms_per_row - 0.09) < 1e-9 and abs(b.fixed_ms - 20.0) < 1e-6
    assert b.rows_at_slo() == 888
    assert b.budget(4096, 950) == 1078                 # decode rows + the minimum prefill
    assert b.budget(512, 300) == 512
    st = b.stats()
    assert st["budget_rows"] == b.rows_at_slo() and st["steps_observed"] == 2


def test_tpot_slo_budget_recovers_from_a_slow_first_step():
    """a 10x slow first step must not pin the budget low.  Capped steps are
    observed too, and the robust (Theil-Sen) fit outvotes the outlier within a few steps."""
    from dgi.sched.slo import StepBudget
    cost = lambda r: 20.0 + 0.1 * r                    # noqa: E731  the true step cost
    b = StepBudget(150.0, min_prefill=128)
    b.observe(1536, 10 * cost(1536))                   # cold start: 10x slow
    assert b.rows_at_slo() < 200
    for i in range(12):
        rows = b.budget(4096, 100)                     # the engine runs what the budget allows
        b.observe(rows + (i % 3) * 40, cost(rows + (i % 3) * 40))
    assert abs(b.rows_at_slo() - 1300) <= 20, b.stats()


def test_tpot_slo_admission_cap_follows_the_load_shape():
    """The admission cap is the decode rows of an SLO-sized step plus the prompts it
    prefills: 512-in / 128-out at 1300 rows -> 260 decode rows + ~2 prompts."""
    from dgi.sched.slo import StepBudget
    b = StepBudget(150.0)
    assert b.admission_cap(4096) is None
    b.observe(1000, 120.0)
    b.observe(2000, 220.0)                             # 20 ms + 0.1 ms per row: 1300 rows at 150 ms
    assert b.admission_cap(4096) is None               # load shape not known yet
    for _ in range(3):
        b.observe_finished(512, 128)
    assert b.admission_cap(4096) == 262
    assert b.admission_cap(1024) == int(1024 * 0.2 + 1024 * 0.8 / 512 + 0.5)
    assert b.stats()["admission_cap"] == 262


def test_engine_with_tpot_slo_runs_smaller_mixed_steps():
    """An engine with a TPOT SLO schedules mixed steps below the SLO's row budget once it
    has measured its step cost, and admits no more sequences than it sustains at the SLO;
    outputs are unchanged (only the chunking and admission order differ)."""
    import torch
    from dgi.engine import EngineConfig, LLMEngine
    from dgi.sched.request import SamplingParams
    g = torch.Generator().manual_seed(0)
    prompts = [torch.randint(5, 500, (120,), generator=g).tolist() for _ in range(12)]
    sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
    base = dict(model="llama-tiny", device="cpu", num_blocks=512, max_num_seqs=16, max_model_len=256,
                max_num_batched_tokens=1024, use_graphs=False, enable_prefix_caching=False)
    ref = [r.output for r in LLMEngine(EngineConfig(**base)).generate(prompts, sp)]
    eng = LLMEngine(EngineConfig(**base, tpot_slo_ms=1e-3))     # unreachable: always the minimum step
    got = [r.output for r in eng.generate(prompts, sp)]
    assert got == ref
    assert eng.step_budget.capped > 0 and eng.step_budget.steps > 0
    assert eng.scheduler.admit_cap is not None and eng.admission_limit() is not None


def test_admission_limit_counts_the_queue_from_the_running_set():
    """The closed-loop client's in-flight limit is min(cap, running now) + the prompts one
    SLO-sized step prefills, rounded UP: while the running set ramps, at most one step of
    prompts waits (no queue behind the cap), and rounding 1.5 prompts down to 1 would pin the
    running set below the cap (round 5: 128 running instead of ~190 at SLO 120)."""
    import types
    from dgi.engine import LLMEngine
    from dgi.sched.slo import StepBudget
    b = StepBudget(150.0)
    b.observe(1000, 120.0)
    b.observe(2000, 220.0)                              # 1300 rows at the SLO
    for _ in range(3):
        b.observe_finished(512, 128)                    # 260 decode rows + 1040 prefill rows = 2.03 prompts
    cap = b.admission_cap(4096)
    fake = types.SimpleNamespace(step_budget=b, cfg=types.SimpleNamespace(max_num_batched_tokens=4096),
                                 scheduler=types.SimpleNamespace(running=[None] * 40))
    assert LLMEngine.admission_limit(fake) == 40 + 3     # ceil(2.03)
    fake.scheduler.running = [None] * (cap + 50)
    assert LLMEngine.admission_limit(fake) == cap + 3
    fake.step_budget = None
    assert LLMEngine.admission_limit(fake) is None


def test_prefill_tiles_heaviest_first():
    """Prefill-attention tiles are listed by the keys they read, most first (every head walks
    the same order, so the grid's tail is the short tiles), covering every tile exactly once."""
    from dgi import ops
    cu = [0, 300, 301, 1325]                 # sequences of 300, 1, 1024 query rows
    ctx = [300, 641, 1024]                   # the second has a 640-token cached prefix
    t = ops.order_prefill_tiles(cu, ctx, tile=128)
    assert t.dtype.name == "int32" and t.shape == (3 + 1 + 8, 2)
    assert sorted(map(tuple, t.tolist())) == sorted([(0, 0), (0, 128), (0, 256), (1, 0)] +
                                                    [(2, 128 * i) for i in range(8)])
    work = [min(ctx[b], ctx[b] - (cu[b + 1] - cu[b]) + t0 + 128) for b, t0 in t.tolist()]
    assert work == sorted(work, reverse=True)
    assert t[0].tolist() == [2, 896] and t[3].tolist() == [1, 0]     # 1024 keys first; 641 after 896 / 768
    assert ops.prefill_tiles([0, 5], tile=128) == [(0, 0)]
