"""Cluster-level prefill/decode scheduler (server/app/services/pd_scheduler.py).

Behavioural parity with the reference's tests/test_server_pd_scheduler.py:
enums, WorkerCapability capacities, PendingJob ordering, assignment rules
(FLOP-weighted prefill, KV-holder-first decode, migration when the holder
cannot decode), latency estimates, batching, migrator de-duplication, and
the lifecycle / load-balancing integration checks.  The module is loaded by
file path, as the reference suite does, so it must not need the server
package's import side effects.
"""
import asyncio
import importlib.util
import os
import sys
import time

import pytest

_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                     "server", "app", "services", "pd_scheduler.py")
_spec = importlib.util.spec_from_file_location("pd_scheduler_isolated", _PATH)
pds = importlib.util.module_from_spec(_spec)
sys.modules[_spec.name] = pds
_spec.loader.exec_module(pds)

JobPhase, WorkerRole, WorkerCapability = pds.JobPhase, pds.WorkerRole, pds.WorkerCapability
PendingJob, WorkerAssignment = pds.PendingJob, pds.WorkerAssignment
PrefillDecodeScheduler, KVCacheMigrator = pds.PrefillDecodeScheduler, pds.KVCacheMigrator


def _fleet():
    # MI355X-class prefill box, a bandwidth-heavy decode box and a smaller hybrid
    return {
        "p": WorkerCapability("p", WorkerRole.PREFILL, compute_flops=2500.0, memory_bandwidth_gbps=8000.0,
                              reliability_score=0.95),
        "d": WorkerCapability("d", WorkerRole.DECODE, compute_flops=600.0, memory_bandwidth_gbps=5300.0,
                              reliability_score=0.9),
        "h": WorkerCapability("h", WorkerRole.HYBRID, compute_flops=300.0, memory_bandwidth_gbps=3000.0,
                              reliability_score=0.85),
    }


@pytest.fixture
def sched():
    return PrefillDecodeScheduler(enable_migration=True, migration_threshold_ms=50.0)


def _job(jid, phase=JobPhase.PREFILL, **kw):
    return PendingJob(priority=kw.pop("priority", 0.0), created_at=kw.pop("created_at", time.time()), job_id=jid,
                      phase=phase, **kw)


# ----------------------------------------------------------------------------- data classes

def test_enum_values():
    assert [p.value for p in JobPhase] == ["prefill", "decode"]
    assert [r.value for r in WorkerRole] == ["prefill", "decode", "hybrid"]


def test_capability_defaults():
    c = WorkerCapability(worker_id="x")
    assert c.role is WorkerRole.HYBRID
    assert (c.compute_flops, c.memory_bandwidth_gbps, c.active_prefill_jobs, c.active_decode_jobs) == (0.0, 0.0, 0, 0)
    assert c.reliability_score == 1.0


@pytest.mark.parametrize("role,pre,dec", [(WorkerRole.HYBRID, 90.0, 900.0), (WorkerRole.PREFILL, 90.0, 0.0),
                                          (WorkerRole.DECODE, 0.0, 900.0)])
def test_capacity_by_role(role, pre, dec):
    c = WorkerCapability("x", role, compute_flops=100.0, memory_bandwidth_gbps=1000.0, reliability_score=0.9)
    assert c.prefill_capacity == pytest.approx(pre)
    assert c.decode_capacity == pytest.approx(dec)


@pytest.mark.parametrize("used,total,util", [(500, 1000, 0.5), (0, 0, 0.0), (1000, 1000, 1.0)])
def test_kv_utilisation(used, total, util):
    c = WorkerCapability("x", kv_cache_tokens_used=used, kv_cache_tokens_total=total)
    assert c.kv_cache_utilization == util


def test_pending_job_fields_and_priority_order():
    jobs = [_job("a", priority=-1.0, created_at=1.0), _job("b", priority=-2.0, created_at=2.0),
            _job("c", priority=-0.5, created_at=3.0), _job("d", priority=-2.0, created_at=1.5)]
    assert [j.job_id for j in sorted(jobs)] == ["d", "b", "a", "c"]  # priority, then age
    j = _job("k", JobPhase.DECODE, prompt_tokens=512, max_tokens=64, kv_cache_key="kv", kv_cache_worker="w")
    assert (j.prompt_tokens, j.max_tokens, j.kv_cache_key, j.kv_cache_worker) == (512, 64, "kv", "w")


def test_assignment_defaults():
    a = WorkerAssignment(worker_id="w", phase=JobPhase.PREFILL, estimated_latency_ms=12.0)
    assert a.kv_migration_needed is False and a.migration_source == ""
    m = WorkerAssignment("w2", JobPhase.DECODE, 3.0, kv_migration_needed=True, migration_source="w1")
    assert m.kv_migration_needed and m.migration_source == "w1"


# ----------------------------------------------------------------------------- scheduler

def test_init_register_unregister_update(sched):
    assert sched.enable_migration and sched.migration_threshold_ms == 50.0
    assert not sched._workers and not sched._prefill_queue and not sched._decode_queue
    f = _fleet()
    sched.register_worker("h", f["h"])
    sched.update_worker_stats("h", {"active_prefill_jobs": 2, "active_decode_jobs": 5, "prefill_latency_ms": 150.0})
    w = sched._workers["h"]
    assert (w.active_prefill_jobs, w.active_decode_jobs, w.prefill_latency_ms) == (2, 5, 150.0)
    sched.update_worker_stats("missing", {"active_prefill_jobs": 1})  # ignored
    sched.unregister_worker("h")
    assert "h" not in sched._workers


def test_unregister_drops_kv_locations(sched):
    sched.register_worker("h", _fleet()["h"])
    sched._kv_cache_locations.update({"k1": "h", "k2": "other"})
    sched.unregister_worker("h")
    assert sched._kv_cache_locations == {"k2": "other"}


async def test_submit_and_transition(sched):
    assert await sched.submit_job(job_id="j", prompt_tokens=1024, max_tokens=256, priority=2.0) == "j"
    assert len(sched._prefill_queue) == 1 and sched._stats["prefill_jobs"] == 1
    await sched.transition_to_decode(job_id="j", kv_cache_key="kv-j", kv_cache_worker="p")
    assert len(sched._decode_queue) == 1 and sched._stats["decode_jobs"] == 1
    assert sched._kv_cache_locations["kv-j"] == "p"


async def test_prefill_goes_to_strongest_compute(sched):
    f = _fleet()
    for k in ("p", "h", "d"):
        sched.register_worker(k, f[k])
    a = await sched.assign_job(_job("j", prompt_tokens=512))
    assert a.worker_id == "p" and a.phase is JobPhase.PREFILL and a.estimated_latency_ms > 0


async def test_decode_stays_on_kv_holder(sched):
    sched.register_worker("h", _fleet()["h"])
    a = await sched.assign_job(_job("j", JobPhase.DECODE, kv_cache_key="kv", kv_cache_worker="h"))
    assert a.worker_id == "h" and not a.kv_migration_needed


async def test_decode_migrates_off_prefill_only_holder(sched):
    f = _fleet()
    sched.register_worker("p", f["p"])
    sched.register_worker("d", f["d"])
    sched._kv_cache_locations["kv"] = "p"
    a = await sched.assign_job(_job("j", JobPhase.DECODE, kv_cache_key="kv", kv_cache_worker="p"))
    assert a.worker_id == "d" and a.kv_migration_needed and a.migration_source == "p"


async def test_decode_holder_looked_up_from_location_index(sched):
    f = _fleet()
    sched.register_worker("d", f["d"])
    sched.register_worker("h", f["h"])
    sched._kv_cache_locations["kv"] = "h"
    a = await sched.assign_job(_job("j", JobPhase.DECODE, kv_cache_key="kv"))
    assert a.worker_id == "h" and not a.kv_migration_needed


async def test_migration_disabled_never_flags(sched):
    s = PrefillDecodeScheduler(enable_migration=False)
    f = _fleet()
    s.register_worker("p", f["p"])
    s.register_worker("d", f["d"])
    a = await s.assign_job(_job("j", JobPhase.DECODE, kv_cache_key="kv", kv_cache_worker="p"))
    assert a.worker_id == "d" and not a.kv_migration_needed


@pytest.mark.parametrize("phase", [JobPhase.PREFILL, JobPhase.DECODE])
async def test_no_workers_raises(sched, phase):
    with pytest.raises(RuntimeError, match="No available workers"):
        await sched.assign_job(_job("j", phase))


async def test_prefill_only_fleet_cannot_decode(sched):
    sched.register_worker("p", _fleet()["p"])
    with pytest.raises(RuntimeError):
        await sched.assign_job(_job("j", JobPhase.DECODE, kv_cache_key="kv", kv_cache_worker="p"))


async def test_get_batch_respects_size_and_assigns(sched):
    sched.register_worker("h", _fleet()["h"])
    for i in range(5):
        await sched.submit_job(job_id=f"j{i}", prompt_tokens=256, priority=float(i))
    batch = await sched.get_batch(JobPhase.PREFILL, max_batch_size=3)
    assert len(batch) == 3 and all(a.worker_id == "h" for _, a in batch)
    assert [j.job_id for j, _ in batch] == ["j4", "j3", "j2"]  # highest priority first
    assert len(sched._prefill_queue) == 2


async def test_get_batch_requeues_unassignable(sched):
    await sched.submit_job(job_id="j", prompt_tokens=8)
    assert await sched.get_batch(JobPhase.PREFILL) == []
    assert len(sched._prefill_queue) == 1


async def test_assignment_counts_load_and_completion_releases(sched):
    sched.register_worker("h", _fleet()["h"])
    await sched.submit_job(job_id="j", prompt_tokens=64)
    [(job, _)] = await sched.get_batch(JobPhase.PREFILL, 1)
    assert sched._workers["h"].active_prefill_jobs == 1
    await sched.transition_to_decode("j", "kv", "h")
    assert sched._workers["h"].active_prefill_jobs == 0
    await sched.get_batch(JobPhase.DECODE, 1)
    assert sched._workers["h"].active_decode_jobs == 1
    await sched.complete_job("j", JobPhase.DECODE, latency_ms=20.0)
    assert sched._workers["h"].active_decode_jobs == 0


def test_prefill_latency_scales_with_history(sched):
    w = _fleet()["p"]
    w.prefill_latency_ms = 200.0
    assert sched._estimate_prefill_latency(w, 1024) == pytest.approx(400.0)
    assert sched._estimate_prefill_latency(w, 256) == pytest.approx(100.0)


def test_prefill_latency_without_history_favours_more_flops(sched):
    f = _fleet()
    fast = sched._estimate_prefill_latency(f["p"], 512)
    slow = sched._estimate_prefill_latency(f["h"], 512)
    assert 0 < fast < slow


def test_decode_latency_history_and_bandwidth_model(sched):
    w = _fleet()["d"]
    w.decode_latency_ms = 15.0
    assert sched._estimate_decode_latency(w) == 15.0
    w.decode_latency_ms = 0.0
    assert sched._estimate_decode_latency(w) > 0
    assert sched._estimate_decode_latency(w) < sched._estimate_decode_latency(_fleet()["h"])


def test_stats_counts_roles(sched):
    for k, w in _fleet().items():
        sched.register_worker(k, w)
    s = sched.get_stats()
    assert (s["total_workers"], s["prefill_workers"], s["decode_workers"]) == (3, 2, 2)
    assert s["prefill_queue_size"] == 0 and s["decode_queue_size"] == 0


# ----------------------------------------------------------------------------- migrator

async def test_migrate_updates_location_and_stats():
    m = KVCacheMigrator(PrefillDecodeScheduler())
    assert await m.migrate(kv_cache_key="kv", source_worker="a", target_worker="b") is True
    assert m.scheduler._kv_cache_locations["kv"] == "b" and m.scheduler._stats["migrations"] == 1


async def test_identical_concurrent_migrations_run_once():
    m = KVCacheMigrator(PrefillDecodeScheduler())
    res = await asyncio.gather(*(asyncio.ensure_future(m.migrate("kv", "a", "b")) for _ in range(3)))
    assert all(res) and m.scheduler._stats["migrations"] == 1


async def test_distinct_migrations_all_run():
    m = KVCacheMigrator(PrefillDecodeScheduler())
    await asyncio.gather(m.migrate("k1", "a", "b"), m.migrate("k2", "a", "c"))
    assert m.scheduler._kv_cache_locations == {"k1": "b", "k2": "c"}
    assert m.scheduler._stats["migrations"] == 2


async def test_transport_bytes_are_accounted_and_failures_reported():
    calls = []

    async def transport(key, src, dst):
        calls.append((key, src, dst))
        if key == "bad":
            raise IOError("link down")
        return 4096

    m = KVCacheMigrator(PrefillDecodeScheduler(), transport=transport)
    assert await m.migrate("ok", "a", "b")
    assert not await m.migrate("bad", "a", "b")
    assert m.scheduler._stats["migration_bytes"] == 4096 and "bad" not in m.scheduler._kv_cache_locations
    assert calls == [("ok", "a", "b"), ("bad", "a", "b")]


# ----------------------------------------------------------------------------- integration

async def test_full_lifecycle_prefill_then_migrating_decode():
    s = PrefillDecodeScheduler()
    s.register_worker("pw", WorkerCapability("pw", WorkerRole.PREFILL, compute_flops=200.0))
    s.register_worker("dw", WorkerCapability("dw", WorkerRole.DECODE, memory_bandwidth_gbps=800.0))
    await s.submit_job(job_id="life", prompt_tokens=1024, max_tokens=256)
    [(job, a)] = await s.get_batch(JobPhase.PREFILL, max_batch_size=1)
    assert a.worker_id == "pw"
    await s.transition_to_decode(job.job_id, "kv-life", "pw")
    [(job, a)] = await s.get_batch(JobPhase.DECODE, max_batch_size=1)
    assert a.worker_id == "dw" and a.kv_migration_needed


async def test_load_spreads_over_identical_workers():
    s = PrefillDecodeScheduler()
    for i in range(3):
        s.register_worker(f"w{i}", WorkerCapability(f"w{i}", WorkerRole.HYBRID, compute_flops=100.0,
                                                    memory_bandwidth_gbps=500.0))
    for i in range(6):
        await s.submit_job(job_id=f"j{i}", prompt_tokens=256)
    batch = await s.get_batch(JobPhase.PREFILL, max_batch_size=6)
    counts = {}
    for _, a in batch:
        counts[a.worker_id] = counts.get(a.worker_id, 0) + 1
    assert sorted(counts.values()) == [2, 2, 2]
