"""Python side of the shared-memory control rings (``dgi/csrc/host/shm_ring.cc``).

A ring is created by its producer (``create_ring``) and opened by its consumer
(``open_ring``), which unlinks the name right away: both mappings stay valid and
nothing is left in ``/dev/shm`` once both ends are up.  The module is built by
``dgi.build.build_shm`` (``__graft_entry__.build``); a missing module raises.
"""
from __future__ import annotations

import time
from typing import Optional

_mod = None


def _shm():
    global _mod
    if _mod is None:
        try:
            from dgi import _shm as m
        except ImportError:
            from dgi.build import build_shm      # g++ only, ~2 s; no ROCm needed
            build_shm()
            from dgi import _shm as m
        _mod = m
    return _mod


def shm_free_bytes(path: str = "/dev/shm") -> Optional[int]:
    """Free bytes of the shared-memory file system the rings live in (None if unknown)."""
    import os
    try:
        st = os.statvfs(path)
    except OSError:
        return None
    return st.f_bavail * st.f_frsize


def create_ring(name: str, capacity: int):
    return _shm().Ring.create(name, int(capacity))


def open_ring(name: str, wait_s: float = 0.0):
    """The consumer end of ``name``; None if it does not exist within ``wait_s``."""
    m = _shm()
    t0 = time.perf_counter()
    delay = 1e-4
    while True:
        r = m.Ring.try_open(name)
        if r is not None:
            m.unlink(name)
            return r
        if time.perf_counter() - t0 >= wait_s:
            return None
        time.sleep(delay)
        delay = min(delay * 2, 0.01)


def unlink(name: str) -> bool:
    return _shm().unlink(name)


def ring_latency_us(n: int = 2000, size: int = 64) -> dict:
    """Single-process round-trip cost of one message (write + poll), microseconds."""
    import os
    m = _shm()
    name = f"/dgi.lat.{os.getpid()}"
    w = m.Ring.create(name, 1 << 20)
    r = m.Ring.try_open(name)
    m.unlink(name)
    b = b"x" * size
    t0 = time.perf_counter()
    for _ in range(n):
        w.send(b, 1.0)
        r.poll()
    return {"msg_bytes": size, "us_per_msg": round((time.perf_counter() - t0) / n * 1e6, 3)}
