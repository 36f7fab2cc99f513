"""Shared-memory control plane (dgi/csrc/host/shm_ring.cc, dgi.parallel.shm):
SPSC ring semantics across processes, wrap-around, full-ring back-pressure,
oversize messages, and the per-message cost."""
import multiprocessing as mp
import os
import uuid

import numpy as np
import pytest

from dgi.parallel import shm


def _name():
    return f"/dgi.test.{uuid.uuid4().hex[:10]}"


def _producer(name, n, seed):
    rng = np.random.default_rng(seed)
    r = shm.create_ring(name, 1 << 16)
    for i in range(n):
        k = int(rng.integers(0, 3000))
        r.send(np.full(k, i, np.int32).tobytes() + i.to_bytes(8, "little"), 60.0)


def test_ring_preserves_order_across_processes():
    name, n = _name(), 3000
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_producer, args=(name, n, 7))
    p.start()
    try:
        r = shm.open_ring(name, 60.0)
        assert r is not None
        rng = np.random.default_rng(7)
        for i in range(n):
            b = r.wait(60.0)
            k = int(rng.integers(0, 3000))
            assert len(b) == 4 * k + 8 and int.from_bytes(b[-8:], "little") == i
            assert (np.frombuffer(b[:-8], np.int32) == i).all()
        assert r.poll() is None
    finally:
        p.join(60)
    assert p.exitcode == 0


def test_ring_back_pressure_and_limits():
    name = _name()
    w = shm.create_ring(name, 4096)
    rd = shm.open_ring(name)
    assert w.try_send(b"a" * 1000) and w.try_send(b"b" * 1000) and w.try_send(b"c" * 1000)
    assert not w.try_send(b"d" * 1500)              # full: the consumer must make room
    with pytest.raises(RuntimeError):
        w.send(b"d" * 1500, 0.05)                   # blocking send times out loudly
    assert rd.poll() == b"a" * 1000
    assert w.try_send(b"d" * 1000)                  # wraps around the end of the data area
    assert [rd.poll() for _ in range(3)] == [b"b" * 1000, b"c" * 1000, b"d" * 1000]
    with pytest.raises(ValueError):
        w.send(b"x" * 3000, 0.1)                    # larger than half the ring
    assert rd.poll() is None and rd.wait(0.01) is None
    assert not os.path.exists("/dev/shm" + name)    # the consumer unlinked the name at open


def test_ring_message_cost_is_microseconds():
    lat = shm.ring_latency_us(5000, 64)
    assert lat["us_per_msg"] < 50.0, lat


# ---------------------------------------------------------------- sanitizer builds

def _stress(kind, *args, **kw):
    import subprocess
    from dgi.build import build_sanitized
    exe = build_sanitized(kind, **kw)
    env = {**os.environ, "ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
           "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1", "TSAN_OPTIONS": "halt_on_error=0"}
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=240, env=env)


def test_ring_clean_under_asan_ubsan():
    """The ring core (csrc/host/shm_ring.h) under AddressSanitizer + UBSan: producer and
    consumer threads on one mapping, producer and consumer processes on two mappings,
    back-pressure / wrap / oversize limits — no report, every message intact."""
    r = _stress("asan", "all", "20000")
    assert r.returncode == 0 and "ERROR" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    assert r.stdout.split() == ["ok", "threads", "20000", "ok", "fork", "20000", "ok", "limits", "68"]


def test_ring_clean_under_tsan():
    """ThreadSanitizer over the release / acquire cursor protocol (threads on one mapping)."""
    r = _stress("tsan", "threads", "20000")
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
    r = _stress("tsan", "limits")
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stderr[-3000:]


def test_tsan_catches_a_relaxed_publication():
    """Self-test of the TSan pass: publish the cursors with relaxed stores and the payload
    race between the producer's copy-in and the consumer's copy-out must be reported."""
    r = _stress("tsan", "threads", "3000", defines=("DGI_SHM_PUBLISH_ORDER=std::memory_order_relaxed",),
                tag="_relaxed")
    assert "WARNING: ThreadSanitizer: data race" in r.stderr, (r.returncode, r.stderr[-2000:])
